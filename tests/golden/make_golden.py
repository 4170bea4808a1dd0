#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE.

Run here (the build container), never on the GPU box:

    python tests/golden/make_golden.py [--reference /root/reference]

It imports TL-System/plato from --reference and drives its own server-side
aggregation code on inputs made by the counter-based generator of
oracle/synth.py (which the tests, the GPU kernels and bench.py restate bit for
bit), then records only data: recipes, SHA-256 digests of the reference's
outputs, sampled output values, and (for the small LeNet-5 / toy cases) full
output arrays.  Nothing from the reference's sources is copied.

Reference code paths exercised (file:line in the reference):
  * fedavg.Server._process_reports            plato/servers/fedavg.py:161-229
    -> Algorithm.compute_weight_deltas        plato/algorithms/fedavg.py:13-27
    -> Server.aggregate_deltas                plato/servers/fedavg.py:137-159
    -> Algorithm.update_weights / load_weights plato/algorithms/fedavg.py:29-48
  * FedBuff aggregate_deltas                  examples/async/fedbuff/fedbuff_server.py:31-50
  * Port aggregate_deltas                     examples/async/port/port_server.py:54-124
  * Pisces aggregate_deltas                   examples/client_selection/pisces/pisces_server.py:73-99
  * FedAsync aggregate_weights                examples/async/fedasync/fedasync_server.py:67-78,
                                              fedasync_algorithm.py:9-20
  * async simulated-wall-time ordering        plato/servers/base.py:925-1091 (_process_clients)
  * cross-silo _process_reports               plato/servers/fedavg_cs.py:161-199
  * RL smart-weighted aggregate_deltas        plato/utils/reinforcement_learning/rl_server.py:45-80
  * HE hybrid FedAvg (plaintext half)         plato/servers/fedavg_he.py:66-106
  * the reference's own known-answer test     tests/fedavg_tests.py:44-175
Missing third-party packages that the reference imports but this path never
uses (socketio, torchvision, zstd, ...) are replaced by inert module stubs.
"""

from __future__ import annotations

import argparse
import asyncio
import copy
import hashlib
import importlib.abc
import importlib.machinery
import json
import os
import sys
import tempfile
import types
from collections import OrderedDict
from unittest import mock

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import synth  # noqa: E402

STUBBED = [
    "socketio", "torchvision", "zstd", "lightly", "opacus", "torch_optimizer", "gym", "boto3",
    "botocore", "evaluate", "tenseal", "cv2", "pycocotools", "skimage", "ultralytics", "h5py",
    "timm", "mmcv", "wandb", "torchmetrics",
    # polaris_server.py imports these at module level (client selection solver, unused here)
    "cvxopt", "mosek", "turtle",
]

CANON_NAN = np.uint32(0x7FC00000)


class _StubFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    """Inert modules for missing packages the aggregation path never calls."""

    def find_spec(self, name, path, target=None):
        if name.split(".")[0] in STUBBED:
            return importlib.machinery.ModuleSpec(name, self, is_package=True)
        return None

    def create_module(self, spec):
        mod = mock.MagicMock(name=spec.name)
        mod.__path__ = []
        mod.__spec__ = spec
        return mod

    def exec_module(self, module):
        return None


CONFIG = """
clients:
    type: simple
    total_clients: 1024
    per_round: 1024
    do_test: false
server:
    address: 127.0.0.1
    port: 8000
    do_test: false
    synchronous: true
    similarity_weight: 1
    staleness_weight: 3
    staleness_bound: 10
    staleness_factor: 0.5
    exploration_factor: 0.3
    exploration_decaying_factor: 0.99
    min_explore_factor: 0.1
    mixing_hyperparameter: 0.9
    adaptive_mixing: true
    staleness_weighting_function:
        type: hinge
        a: 10
        b: 4
data:
    datasource: MNIST
    partition_size: 20000
    sampler: iid
    random_seed: 1
trainer:
    type: basic
    rounds: 1
    max_concurrency: 1
    epochs: 1
    batch_size: 32
    optimizer: SGD
    model_name: resnet_18
algorithm:
    type: fedavg
parameters:
    model:
        num_classes: 10
    optimizer:
        lr: 0.01
        momentum: 0.9
        weight_decay: 0.0
"""


def boot_reference(ref_root: str, workdir: str):
    sys.meta_path.insert(0, _StubFinder())
    cfg = os.path.join(workdir, "golden.yml")
    with open(cfg, "w") as f:
        f.write(CONFIG)
    os.environ["config_file"] = cfg
    sys.argv = ["make_golden", "-b", workdir]
    sys.path.insert(0, ref_root)
    for sub in ("examples/async/fedbuff", "examples/async/port", "examples/async/fedasync",
                "examples/client_selection/pisces", "examples/server_aggregation/fedatt",
                "examples/server_aggregation/fedadp", "examples/client_selection/polaris"):
        sys.path.insert(0, os.path.join(ref_root, sub))
    from plato.config import Config

    Config()


# --------------------------------------------------------------------------
def canon(a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float32).copy()
    bits = a.view(np.uint32)
    bits[np.isnan(a)] = CANON_NAN
    return a


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def f32hex(x) -> str:
    return "%08x" % int(np.float32(x).view(np.uint32))


def layout_of(state_dict):
    entries = []
    nf = ni = 0
    for name, t in state_dict.items():
        if t.dtype == torch.float32:
            entries.append((name, "f32", nf, t.numel(), list(t.shape)))
            nf += t.numel()
        elif t.dtype == torch.int64:
            entries.append((name, "i64", ni, t.numel(), list(t.shape)))
            ni += t.numel()
        else:
            raise TypeError(name)
    return entries, nf, ni


def unpack(entries, flat_f, flat_i):
    out = OrderedDict()
    for name, reg, off, n, shape in entries:
        src = flat_f if reg == "f32" else flat_i
        out[name] = src[off : off + n].reshape(shape)
    return out


def flatten(entries, sd, region, dtype):
    parts = [sd[name].reshape(-1).to(dtype) for name, reg, *_ in entries if reg == region]
    return torch.cat(parts).numpy() if parts else np.zeros(0, dtype=np.float32)


def apply_overrides(bf, bi, xs_f, xs_i, overrides):
    for tgt, region, idx, val in overrides:
        if region == "f32":
            arr = bf if tgt == "base" else xs_f[tgt]
            arr.view(np.uint32)[idx] = np.uint32(int(val, 16))
        else:
            arr = bi if tgt == "base" else xs_i[tgt]
            arr[idx] = np.int64(int(val))


def make_model(name):
    if name in HF_MODELS:
        if name not in _HF_BUILT:  # built before boot_reference (see main)
            _HF_BUILT[name] = HF_MODELS[name]()
        return _HF_BUILT[name]
    from plato.models import lenet5, resnet

    if name == "lenet5":
        return lenet5.Model(num_classes=10)
    if name == "resnet18":
        return resnet.Model.get("resnet_18", num_classes=10)
    if name == "resnet50_200":
        return resnet.Model.get("resnet_50", num_classes=200)
    raise ValueError(name)


def _vit_large_hf():
    """C5's ViT-L/16 classifier as the reference's models/vit.py builds it from HuggingFace
    (AutoModelForImageClassification; here from its config, offline: random init, the same module
    and state_dict layout as the installed transformers gives)."""
    from transformers import ViTConfig, ViTForImageClassification

    return ViTForImageClassification(ViTConfig(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                                               intermediate_size=4096, image_size=224, patch_size=16, num_labels=10))


def _gpt2_medium_hf():
    """C5's GPT-2-medium as the reference's models/huggingface.py builds it (AutoModelForCausalLM), from its
    config, offline; its state_dict lists the tied lm_head beside transformer.wte."""
    from transformers import GPT2Config, GPT2LMHeadModel

    return GPT2LMHeadModel(GPT2Config(n_embd=1024, n_layer=24, n_head=16, n_positions=1024, vocab_size=50257))


HF_MODELS = {"vit_large_hf": _vit_large_hf, "gpt2_medium_hf": _gpt2_medium_hf}
_HF_BUILT: dict = {}


def make_updates(num_samples, payloads, order, staleness):
    ups = []
    for pos, c in enumerate(order):
        ups.append(types.SimpleNamespace(
            client_id=c + 1,
            report=types.SimpleNamespace(client_id=c + 1, num_samples=num_samples[c], accuracy=0.5,
                                         training_time=0, processing_time=0, comm_time=0,
                                         update_response=False, statistical_utility=1.0,
                                         start_round=0),
            payload=payloads[c],
            staleness=staleness[c],
        ))
    return ups


def server_class(mode):
    if mode == "fedavg":
        from plato.servers import fedavg
        return fedavg.Server
    if mode == "fedbuff":
        import fedbuff_server
        return fedbuff_server.Server
    if mode == "port":
        import port_server
        return port_server.Server
    if mode == "pisces":
        import pisces_server
        return pisces_server.Server
    if mode == "fedasync":
        import fedasync_server
        return fedasync_server.Server
    if mode == "fedatt":
        import fedatt_server
        return fedatt_server.Server
    if mode == "fedadp":
        import fedadp_server
        return fedadp_server.Server
    if mode == "polaris":
        import polaris_server
        return polaris_server.Server
    if mode == "cross_silo":
        from plato.servers import fedavg_cs
        return fedavg_cs.Server
    if mode == "async_wall":
        from plato.servers import fedavg
        return fedavg.Server
    if mode in ("rl", "rl_f32"):
        return rl_server_class()
    raise ValueError(mode)


class _StubAgent:
    """The RL agent surface rl_server.RLServer.aggregate_deltas touches (rl_server.py:45-90)."""

    def __init__(self, action):
        self.current_step = 0
        self.planned = action
        self.action = None
        self.num_samples = None

    def prep_action(self):
        self.action = self.planned

    async def prep_agent_update(self):
        return None

    def process_env_update(self):
        return None


async def drive_async_wall_time(server, case, payloads):
    """base.Server._process_clients in asynchronous mode with simulated wall time
    (plato/servers/base.py:925-1091): every client has reported (heap of
    (finish_time, client_id, info), :896-910); the server pops the
    minimum_clients earliest finishers, then the clients that violate the
    staleness bound, in finish-time order (:1007-1079), and aggregates them in
    that order.  Returns the client indices in the order the updates were formed.
    """
    import heapq

    k = case["k"]
    finish = case["finish_times"]
    starting = case["starting_rounds"]
    server.asynchronous_mode = True
    server.simulate_wall_time = True
    server.request_update = False
    server.minimum_clients = case["minimum_clients"]
    server.staleness_bound = case["staleness_bound"]
    server.selected_clients = list(range(1, k + 1))
    server.current_reported_clients = {}
    server.current_processed_clients = {}
    server.reported_clients = []
    server.updates = []
    server.training_clients = {}
    info = None
    for c in case["arrival_order"]:
        report = types.SimpleNamespace(client_id=c + 1, num_samples=case["num_samples"][c], accuracy=0.5,
                                       training_time=0, processing_time=0, comm_time=0, update_response=False,
                                       statistical_utility=1.0, start_round=starting[c])
        info = (float(finish[c]), c + 1, {"client_id": c + 1, "sid": f"s{c}", "starting_round": starting[c],
                                         "start_time": 0.0, "report": report, "payload": payloads[c]})
        heapq.heappush(server.reported_clients, info)
        server.current_reported_clients[c + 1] = True

    async def nothing(*a, **kw):
        return None

    server.wrap_up = nothing
    server._select_clients = nothing
    order = []
    orig = server._process_reports

    async def spy():
        order.extend(u.client_id - 1 for u in server.updates)
        return await orig()

    server._process_reports = spy
    await server._process_clients(info)
    return order


def rl_server_class():
    from plato.utils.reinforcement_learning import rl_server

    class GoldenRLServer(rl_server.RLServer):
        action_dtype = np.float64

        def prep_state(self):
            return None

        def apply_action(self):
            # what examples/outdated/fei/fei_server.py:43 does with the agent's action
            self.smart_weighting = np.array(self.agent.action, dtype=self.action_dtype)

    return GoldenRLServer


def rl_action(case):
    return [[float.fromhex(h)] for h in case["action"]]


def run_he_case(case):
    """fedavg_he.Server._fedavg_hybrid (servers/fedavg_he.py:66-106) on float64 plaintext vectors.

    The vectors are built as homo_enc.encrypt_weights builds them
    (homo_enc.py:50-63: np.append of every weight into a float64 vector, the
    encrypted indices deleted); the encrypted half is an fp32 torch stand-in
    (tenseal is absent), recorded but not part of the check.
    """
    from plato.servers import fedavg_he
    from plato.utils import homo_enc

    model = make_model(case["model"])
    entries, nf, ni = layout_of(model.state_dict())
    k, seed = case["k"], case["seed"]
    bf, bi = synth.baseline_arena(nf, ni, seed)
    enc_idx = list(case["encrypt_indices"])
    msgs = []
    for c in range(k):
        xf, xi = synth.client_arena(bf, bi, seed, c)
        sd = unpack(entries, torch.from_numpy(xf), torch.from_numpy(xi))
        vec = np.array([])
        for w in sd.values():
            vec = np.append(vec, w)
        msgs.append({"unencrypted_weights": np.delete(vec, enc_idx),
                     "encrypted_weights": torch.from_numpy(vec[enc_idx].astype(np.float32)),
                     "indices": list(enc_idx)})
    updates = make_updates(case["num_samples"], msgs, list(range(k)), [0] * k)
    fake = types.SimpleNamespace(context=None, trainer=types.SimpleNamespace(
        zeros=lambda shape: torch.zeros(shape)))
    orig = homo_enc.deserialize_weights
    homo_enc.deserialize_weights = lambda w, ctx: w
    try:
        res = fedavg_he.Server._fedavg_hybrid(fake, updates)
    finally:
        homo_enc.deserialize_weights = orig
    unenc = res["unencrypted_weights"]
    out = {"unencrypted_avg_sha256": sha(np.ascontiguousarray(unenc.numpy())), "dtype": str(unenc.dtype),
           "n_unencrypted": int(unenc.numel()), "total_samples": fake.total_samples}
    if case.get("full"):
        out["_full"] = {"unencrypted_avg": unenc.numpy()}
    return out, entries


def run_case(case):
    """Run the reference on one recipe; return the recorded outputs."""
    model = make_model(case["model"])
    entries, nf, ni = layout_of(model.state_dict())
    k, seed = case["k"], case["seed"]
    bf, bi = synth.baseline_arena(nf, ni, seed)
    xs = [synth.client_arena(bf, bi, seed, c) for c in range(k)]
    xs_f = [x[0] for x in xs]
    xs_i = [x[1] for x in xs]
    apply_overrides(bf, bi, xs_f, xs_i, case.get("overrides", []))
    # tied weights (GPT-2's lm_head = transformer.wte): the model's state_dict holds one storage under both
    # keys, so a real baseline and real payloads carry equal values there (the baseline is read back from
    # the server's model after load_weights, where the later key's copy wins)
    by_name = {n: (r, o, c) for n, r, o, c, _ in entries}
    for dst, src in case.get("tied", []):
        (rd, od, nd), (rs, os_, ns_) = by_name[dst], by_name[src]
        assert rd == rs == "f32" and nd == ns_
        for arr in [bf, *xs_f]:
            arr[od:od + nd] = arr[os_:os_ + ns_]
    baseline = unpack(entries, torch.from_numpy(bf), torch.from_numpy(bi))
    payloads = [unpack(entries, torch.from_numpy(xs_f[c]), torch.from_numpy(xs_i[c]))
                for c in range(k)]
    if case.get("codec") == "bf16":
        # the reference's own codec pair: client model_quantize, server model_dequantize
        from plato.processors import model_dequantize, model_quantize

        q = model_quantize.Processor(client_id=1)
        dq = model_dequantize.Processor(server_id=0)
        payloads = [dq.process(q.process(p)) for p in payloads]
    if case.get("codec") == "qsgd":
        # QSGD wire payloads (oracle/qsgd.py, the format of model_quantize_qsgd.py:130-139)
        # decoded by the reference's own server-side processor
        from plato.processors import model_dequantize_qsgd

        from oracle import qsgd

        ents = [types.SimpleNamespace(name=n, region=r, offset=o, numel=c, shape=tuple(s))
                for n, r, o, c, s in entries]
        dq = model_dequantize_qsgd.Processor(server_id=0)
        payloads = [dq.process(qsgd.client_wire(ents, seed, c)[0]) for c in range(k)]
    order = case.get("order", list(range(k)))
    staleness = case.get("staleness", [0] * k)
    mode = case.get("mode", "fedavg")

    cls = server_class(mode)
    if mode == "fedasync":
        from fedasync_algorithm import Algorithm as FedAsyncAlgorithm

        server = cls(model=lambda: model, algorithm=FedAsyncAlgorithm)
        server.init_trainer()
        # what FedAsync's configure() reads from the config (fedasync_server.py:37-65)
        server.mixing_hyperparam = 0.9
        server.adaptive_mixing = True
    elif mode == "fedatt":
        import fedatt_algorithm

        server = cls(model=lambda: model, algorithm=fedatt_algorithm.Algorithm)
        server.init_trainer()
    elif mode in ("rl", "rl_f32"):
        server = cls(agent=_StubAgent(rl_action(case)), model=lambda: model)
        server.action_dtype = np.float64 if mode == "rl" else np.float32
        server.init_trainer()
    else:
        server = cls(model=lambda: model)
        server.init_trainer()
    if mode == "polaris":
        # what Polaris' configure() sets (polaris_server.py:43-51)
        server.number_of_client = case.get("total_clients", 1024)
        server.local_gradient_bounds = 0.5 * np.ones(server.number_of_client)
        server.local_stalenesses = 0.01 * np.ones(server.number_of_client)
        server.aggregation_weights = np.ones(server.number_of_client) * (1.0 / server.number_of_client)
        server.unexplored_clients = list(range(server.number_of_client))
        server.alpha = 10
    if mode == "fedadp":
        server.selected_clients = [c + 1 for c in order]
        server.local_angles = {int(c): np.float32(float.fromhex(a)) for c, a in case.get("local_angles", {}).items()}
    if mode == "pisces":
        server.client_staleness = {c + 1: [] for c in range(k)}
    server.algorithm.load_weights(copy.deepcopy(baseline))
    server.updates = make_updates(case["num_samples"], payloads, order, staleness)
    server.current_round = case.get("current_round", 0)
    if "previous" in case:
        # the round-(r-2) global model Port compares against (port_server.py:28-36)
        from plato.config import Config

        pv = case["previous"]
        prev_f = synth.synth_f32(nf, seed, pv["stream"], pv["scale"], add=bf)
        prev_i = synth.synth_i64(ni, seed, pv["stream"], 3, add=bi)
        model_path = Config().params["model_path"]
        os.makedirs(model_path, exist_ok=True)
        torch.save(unpack(entries, torch.from_numpy(prev_f), torch.from_numpy(prev_i)),
                   f"{model_path}/model_{server.current_round - 2}.pth")

    captured = {}
    orig_agg = server.aggregate_deltas if mode != "fedasync" else None
    if orig_agg is not None:
        async def spy_agg(updates, deltas):
            avg = await orig_agg(updates, deltas)
            captured["avg"] = {n: t.clone() for n, t in avg.items()}
            return avg
        server.aggregate_deltas = spy_agg
    if mode == "port":
        orig_cs = server.cosine_similarity

        async def spy_cs(update, st):
            sim = await orig_cs(update, st)
            captured.setdefault("sims", []).append(
                f32hex(sim.item()) if isinstance(sim, torch.Tensor) else float(sim))
            return sim
        server.cosine_similarity = spy_cs
    if mode == "fedatt":
        import fedatt_algorithm

        real_softmax = fedatt_algorithm.F.softmax

        def spy_softmax(t, dim=0):
            out = real_softmax(t, dim=dim)
            captured.setdefault("norms", []).append([f32hex(v) for v in t.numpy()])
            captured.setdefault("atts", []).append([f32hex(v) for v in out.numpy()])
            return out
        fedatt_algorithm.F = types.SimpleNamespace(softmax=spy_softmax)
        torch.manual_seed(case["noise_seed"])
    if mode == "fedadp":
        orig_w = server.calc_adaptive_weighting

        def spy_w(deltas, num_samples):
            captured["global_grads"] = {n: t.clone() for n, t in server.global_grads.items()}
            res = orig_w(deltas, num_samples)
            captured["adaptive"] = [float(x).hex() for x in res]
            return res
        server.calc_adaptive_weighting = spy_w
    orig_load = server.algorithm.load_weights

    def spy_load(weights):
        captured["updated"] = OrderedDict((n, t.clone()) for n, t in weights.items())
        return orig_load(weights)
    server.algorithm.load_weights = spy_load

    if mode == "cross_silo":
        # fedavg_cs.get_logged_items reads algorithm.local_rounds, which only a cross-silo
        # config carries; the CSV row written after the aggregation is not part of the check
        orig_event = server.callback_handler.call_event

        def call_event(event, *a, **kw):
            if event != "on_clients_processed":
                return orig_event(event, *a, **kw)
        server.callback_handler.call_event = call_event
    if mode == "async_wall":
        captured["order"] = asyncio.run(drive_async_wall_time(server, case, payloads))
    elif mode in ("fedavg", "fedbuff", "port", "fedasync", "fedatt", "fedadp", "polaris", "cross_silo", "rl",
                  "rl_f32"):
        asyncio.run(server._process_reports())
    else:  # pisces: drive the hot path directly (its weights_aggregated needs client selection state)
        weights_received = [u.payload for u in server.updates]
        base_w = server.algorithm.extract_weights()
        deltas = server.algorithm.compute_weight_deltas(base_w, weights_received)
        avg = asyncio.run(server.aggregate_deltas(server.updates, deltas))
        server.algorithm.load_weights(server.algorithm.update_weights(avg))

    loaded = model.state_dict()
    upd = captured["updated"]
    out = {
        "layout": {"n_f32": nf, "n_i64": ni, "tensors": len(entries)},
        "updated_f32_sha256": sha(canon(flatten(entries, upd, "f32", torch.float32))),
        "updated_i64f_sha256": sha(canon(flatten(entries, upd, "i64", torch.float32))),
        "loaded_i64_sha256": sha(flatten(entries, loaded, "i64", torch.int64)),
    }
    uf = flatten(entries, upd, "f32", torch.float32)
    rng = np.random.default_rng(1234)
    idx = np.unique(np.concatenate([np.arange(min(64, nf)), rng.integers(0, nf, 192), [nf - 1]]))
    out["samples_f32"] = [[int(i), f32hex(uf[i])] for i in idx]
    ui = flatten(entries, upd, "i64", torch.float32)
    out["samples_i64f"] = [[int(i), f32hex(ui[i])] for i in range(min(ni, 64))]
    li = flatten(entries, loaded, "i64", torch.int64)
    out["samples_loaded_i64"] = [[int(i), int(li[i])] for i in range(min(ni, 64))]
    if "sims" in captured:
        out["port_similarities"] = captured["sims"]
    if mode == "fedatt":
        out["fedatt_norms"] = captured["norms"]   # [entry][client], baseline key order
        out["fedatt_atts"] = captured["atts"]
    if mode == "fedadp":
        gg = captured["global_grads"]
        out["global_grads_f32_sha256"] = sha(canon(flatten(entries, gg, "f32", torch.float32)))
        out["global_grads_i64f_sha256"] = sha(canon(flatten(entries, gg, "i64", torch.float32)))
        out["adaptive_weighting"] = captured["adaptive"]
        out["local_angles"] = {str(c): f32hex(a) for c, a in server.local_angles.items()}
    if mode in ("cross_silo", "rl", "rl_f32", "async_wall"):
        out["total_samples"] = server.total_samples
    if mode == "async_wall":
        out["updates_order"] = captured["order"]  # client index per position of self.updates
    if mode == "polaris":
        sq = server.squared_deltas_current_round
        out["squared_deltas"] = {str(i): float(sq[i]).hex() for i in range(len(sq)) if sq[i] != 0}
        out["total_samples"] = server.total_samples
    if "avg" in captured:
        out["avg_f32_sha256"] = sha(canon(flatten(entries, captured["avg"], "f32", torch.float32)))
        out["avg_i64f_sha256"] = sha(canon(flatten(entries, captured["avg"], "i64", torch.float32)))
    if case.get("full"):
        out["_full"] = {"updated_f32": uf, "updated_i64f": ui, "loaded_i64": li}
        if "avg" in captured:
            out["_full"]["avg_f32"] = flatten(entries, captured["avg"], "f32", torch.float32)
    return out, entries


def cases():
    c2_ns = synth.num_samples(128, 0)
    ovr_edge = [
        [3, "f32", 5, "7fc00000"],    # NaN in one client
        [1, "f32", 6, "7f800000"],    # +Inf
        [2, "f32", 7, "ff800000"],    # -Inf
        ["base", "f32", 8, "00000001"],  # smallest denormal baseline
        [0, "f32", 8, "80000003"],    # denormal client
        ["base", "f32", 9, "80000000"],  # -0 baseline
        [0, "f32", 9, "00000000"],
        [1, "f32", 9, "80000000"],
        [4, "f32", 10, "7f7fffff"],   # FLT_MAX -> overflow in the sum
        [5, "f32", 10, "7f7fffff"],
        ["base", "f32", 11, "3f800000"],
        [0, "f32", 11, "3f800001"],   # 1 ulp deltas
        [6, "f32", 12, "00800000"],   # FLT_MIN normal
    ]
    ovr_i64 = [
        ["base", "i64", 0, str(2**40 + 3)], [0, "i64", 0, str(2**40 + 11)],
        [1, "i64", 0, str(2**40 + 1)], [2, "i64", 0, str(2**40 - 7)], [3, "i64", 0, str(2**40 + 3)],
        [4, "i64", 0, str(2**40 + 5)],
        ["base", "i64", 1, "5000"], [0, "i64", 1, "4000"], [1, "i64", 1, "3"], [2, "i64", 1, "-20"],
        ["base", "i64", 2, str(2**24 + 1)], [3, "i64", 2, str(2**24 + 2**20)],
        ["base", "i64", 3, str(-1)], [1, "i64", 3, str(2**63 - 1)],  # int64 wrap in x - b
    ]
    return [
        dict(name="C1_lenet5_k10_iid", model="lenet5", k=10, seed=1, num_samples=[20000] * 10, full=True),
        dict(name="lenet5_k10_skewed", model="lenet5", k=10, seed=2,
             num_samples=synth.num_samples(10, 2), full=True),
        dict(name="lenet5_k7_edge_values", model="lenet5", k=7, seed=9,
             num_samples=[300, 10, 7, 1000, 55, 55, 2], overrides=ovr_edge, full=True),
        dict(name="resnet18_k16", model="resnet18", k=16, seed=3, num_samples=synth.num_samples(16, 3)),
        dict(name="resnet18_k16_permuted", model="resnet18", k=16, seed=3,
             num_samples=synth.num_samples(16, 3), order=[5, 0, 15, 3, 2, 9, 1, 14, 4, 8, 11, 7, 6, 13, 10, 12]),
        dict(name="resnet18_k1", model="resnet18", k=1, seed=5, num_samples=[777]),
        dict(name="resnet18_k5_int64_edges", model="resnet18", k=5, seed=6,
             num_samples=[10, 20, 30, 40, 50], overrides=ovr_i64),
        dict(name="C2_resnet18_k128", model="resnet18", k=128, seed=0, num_samples=c2_ns),
        dict(name="C2_resnet18_k128_equal", model="resnet18", k=128, seed=0, num_samples=[1000] * 128),
        dict(name="C3_resnet50_200cls_k8", model="resnet50_200", k=8, seed=4,
             num_samples=synth.num_samples(8, 4)),
        dict(name="fedbuff_resnet18_k16", model="resnet18", k=16, seed=7, mode="fedbuff",
             num_samples=synth.num_samples(16, 7)),
        dict(name="port_resnet18_k16", model="resnet18", k=16, seed=8, mode="port",
             num_samples=synth.num_samples(16, 8), staleness=[i % 11 for i in range(16)]),
        dict(name="pisces_resnet18_k8", model="resnet18", k=8, seed=10, mode="pisces",
             num_samples=synth.num_samples(8, 10), staleness=[0, 1, 2, 3, 5, 8, 13, 1]),
        dict(name="fedasync_resnet18_k1", model="resnet18", k=1, seed=12, mode="fedasync",
             num_samples=[500], staleness=[7]),
        dict(name="port_similarity_lenet5_k8", model="lenet5", k=8, seed=14, mode="port",
             num_samples=synth.num_samples(8, 14), staleness=[0, 1, 2, 3, 5, 2, 0, 4],
             current_round=5, previous={"stream": 999, "scale": -26}, full=True),
        dict(name="port_similarity_resnet18_k4", model="resnet18", k=4, seed=15, mode="port",
             num_samples=synth.num_samples(4, 15), staleness=[3, 0, 2, 7],
             current_round=9, previous={"stream": 998, "scale": -25}),
        dict(name="bf16_codec_resnet18_k16", model="resnet18", k=16, seed=16, codec="bf16",
             num_samples=synth.num_samples(16, 16)),
        dict(name="bf16_codec_lenet5_k9", model="lenet5", k=9, seed=17, codec="bf16",
             num_samples=synth.num_samples(9, 17), full=True),
        dict(name="gan_lenet5_resnet18_k5", mode="gan", models=["lenet5", "resnet18"], k=5, seed=18,
             num_samples=synth.num_samples(5, 18)),
        dict(name="fedatt_lenet5_k6", model="lenet5", k=6, seed=19, mode="fedatt", noise_seed=7,
             num_samples=synth.num_samples(6, 19), full=True),
        dict(name="fedatt_resnet18_k8", model="resnet18", k=8, seed=20, mode="fedatt", noise_seed=11,
             num_samples=synth.num_samples(8, 20)),
        dict(name="fedadp_lenet5_k6", model="lenet5", k=6, seed=21, mode="fedadp", current_round=3,
             num_samples=synth.num_samples(6, 21), local_angles={"2": "0x1.8p+0", "5": "0x1.2p-1"}, full=True),
        dict(name="fedadp_resnet18_k8", model="resnet18", k=8, seed=22, mode="fedadp", current_round=1,
             num_samples=synth.num_samples(8, 22), order=[3, 0, 7, 1, 2, 6, 4, 5]),
        dict(name="polaris_resnet18_k8", model="resnet18", k=8, seed=23, mode="polaris",
             num_samples=synth.num_samples(8, 23), order=[2, 0, 5, 7, 1, 3, 6, 4]),
        dict(name="qsgd_codec_lenet5_k6", model="lenet5", k=6, seed=24, codec="qsgd",
             num_samples=synth.num_samples(6, 24), full=True),
        dict(name="qsgd_codec_resnet18_k3", model="resnet18", k=3, seed=25, codec="qsgd",
             num_samples=synth.num_samples(3, 25), order=[2, 0, 1]),
        dict(name="C4_port_resnet18_k256", model="resnet18", k=256, seed=13, mode="port",
             num_samples=synth.num_samples(256, 13), staleness=[(7 * i) % 11 for i in range(256)]),
        dict(name="async_wall_resnet18_k12", model="resnet18", k=12, seed=33, mode="async_wall",
             num_samples=synth.num_samples(12, 33), current_round=20, minimum_clients=5, staleness_bound=6,
             finish_times=[7.5, 3.25, 9.0, 1.5, 12.0, 3.25, 6.0, 15.5, 2.75, 11.0, 8.25, 4.0],
             starting_rounds=[19, 18, 11, 20, 17, 19, 16, 10, 19, 18, 20, 17],
             arrival_order=[4, 0, 7, 2, 9, 1, 11, 3, 6, 10, 5, 8]),
        dict(name="cross_silo_resnet18_k6", model="resnet18", k=6, seed=26, mode="cross_silo",
             num_samples=synth.num_samples(6, 26), order=[4, 1, 0, 5, 2, 3]),
        dict(name="cross_silo_lenet5_k4_edges", model="lenet5", k=4, seed=27, mode="cross_silo",
             num_samples=[20000 * 3, 20000 * 2, 20000 * 4, 20000], full=True),
        dict(name="rl_float64_resnet18_k6", model="resnet18", k=6, seed=28, mode="rl",
             num_samples=synth.num_samples(6, 28), action=rl_weights(6, 28)),
        dict(name="rl_float64_lenet5_k5", model="lenet5", k=5, seed=29, mode="rl",
             num_samples=synth.num_samples(5, 29), action=rl_weights(5, 29), full=True),
        dict(name="rl_float32_resnet18_k4", model="resnet18", k=4, seed=30, mode="rl_f32",
             num_samples=synth.num_samples(4, 30), action=rl_weights(4, 30)),
        # coded payloads reaching the variant servers: the reference dequantizes them in its inbound
        # processor (model_dequantize / model_dequantize_qsgd) before FedAtt / FedAdp / Polaris / Port run
        dict(name="fedatt_bf16_lenet5_k5", model="lenet5", k=5, seed=34, mode="fedatt", codec="bf16", noise_seed=5,
             num_samples=synth.num_samples(5, 34), full=True),
        dict(name="fedatt_qsgd_resnet18_k3", model="resnet18", k=3, seed=35, mode="fedatt", codec="qsgd",
             noise_seed=9, num_samples=synth.num_samples(3, 35)),
        dict(name="fedadp_bf16_resnet18_k4", model="resnet18", k=4, seed=36, mode="fedadp", codec="bf16",
             current_round=2, num_samples=synth.num_samples(4, 36), order=[1, 3, 0, 2]),
        dict(name="fedadp_qsgd_lenet5_k5", model="lenet5", k=5, seed=37, mode="fedadp", codec="qsgd",
             current_round=1, num_samples=synth.num_samples(5, 37)),
        dict(name="polaris_bf16_resnet18_k4", model="resnet18", k=4, seed=38, mode="polaris", codec="bf16",
             num_samples=synth.num_samples(4, 38), order=[2, 0, 3, 1]),
        dict(name="port_similarity_qsgd_lenet5_k6", model="lenet5", k=6, seed=39, mode="port", codec="qsgd",
             num_samples=synth.num_samples(6, 39), staleness=[0, 3, 2, 5, 1, 4],
             current_round=6, previous={"stream": 997, "scale": -26}),
        dict(name="he_plain_lenet5_k5", model="lenet5", k=5, seed=31, mode="he",
             num_samples=synth.num_samples(5, 31), encrypt_indices=list(range(0, 61706, 97)), full=True),
        dict(name="he_plain_resnet18_k3", model="resnet18", k=3, seed=32, mode="he",
             num_samples=synth.num_samples(3, 32), encrypt_indices=list(range(100, 2000))),
        # C5: the transformer models at full size, a few clients (the reference's CPU
        # aggregation of K = 32 would need ~80 GB here); the kernel's arithmetic does not depend on K
        dict(name="C5_vit_large_hf_k3", model="vit_large_hf", k=3, seed=40, num_samples=synth.num_samples(3, 40)),
        dict(name="C5_gpt2_medium_hf_k2", model="gpt2_medium_hf", k=2, seed=41,
             num_samples=synth.num_samples(2, 41), tied=[["transformer.wte.weight", "lm_head.weight"]]),
    ]


def rl_weights(k, seed):
    """An RL action: k positive float64 weights summing to ~1 (float.hex for the recipe)."""
    rng = np.random.default_rng(1000 + seed)
    w = rng.uniform(0.2, 1.0, k)
    return [float(v).hex() for v in (w / w.sum())]


def run_gan_case(case):
    """fedavg_gan.Server.aggregate_deltas (servers/fedavg_gan.py:13-43) on (gen, disc) deltas."""
    from plato.servers import fedavg_gan

    k, seed = case["k"], case["seed"]
    parts = []
    for j, name in enumerate(case["models"]):
        model = make_model(name)
        entries, nf, ni = layout_of(model.state_dict())
        bf, bi = synth.baseline_arena(nf, ni, seed + j)
        base = unpack(entries, torch.from_numpy(bf), torch.from_numpy(bi))
        deltas = []
        for c in range(k):
            xf, xi = synth.client_arena(bf, bi, seed + j, c)
            x = unpack(entries, torch.from_numpy(xf), torch.from_numpy(xi))
            deltas.append(OrderedDict((n, x[n] - base[n]) for n in x))  # algorithm: current - baseline
        parts.append((entries, deltas))
    server = fedavg_gan.Server(model=lambda: make_model(case["models"][0]))
    server.init_trainer()
    updates = make_updates(case["num_samples"], [None] * k, list(range(k)), [0] * k)
    pairs = [(parts[0][1][c], parts[1][1][c]) for c in range(k)]
    gen, disc = asyncio.run(server.aggregate_deltas(updates, pairs))
    out = {}
    for tag, (entries, _), avg in (("gen", parts[0], gen), ("disc", parts[1], disc)):
        out[f"{tag}_avg_f32_sha256"] = sha(canon(flatten(entries, avg, "f32", torch.float32)))
        out[f"{tag}_avg_i64f_sha256"] = sha(canon(flatten(entries, avg, "i64", torch.float32)))
    out["total_samples"] = server.total_samples
    return out, None


def dump_shapes(out_dir, names=("lenet5", "resnet18", "resnet50_200", "vit_large_hf", "gpt2_medium_hf")):
    for name in names:
        sd = make_model(name).state_dict()
        spec = [[k, list(v.shape), "f32" if v.dtype == torch.float32 else "i64"] for k, v in sd.items()]
        with open(os.path.join(out_dir, f"shapes_{name}.json"), "w") as f:
            json.dump(spec, f)


def run_reference_known_answer(ref_root):
    """tests/fedavg_tests.py's aggregation: record the 4 payloads and the server model after FedAvg."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("ref_fedavg_tests",
                                                  os.path.join(ref_root, "tests", "fedavg_tests.py"))
    # The test module re-points config_file at its own yml; keep ours.
    saved = os.environ["config_file"]
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    os.environ["config_file"] = saved
    from plato.servers import fedavg as fedavg_server

    captured = {}
    orig = fedavg_server.Server.aggregate_deltas

    async def spy(self, updates, deltas):
        captured["payloads"] = [copy.deepcopy(u.payload) for u in updates]
        captured["num_samples"] = [u.report.num_samples for u in updates]
        captured["server"] = self
        return await orig(self, updates, deltas)

    fedavg_server.Server.aggregate_deltas = spy
    try:
        test = mod.FedAvgTest("test_fedavg_aggregation")
        test.setUp()
        test.test_fedavg_aggregation()
    finally:
        fedavg_server.Server.aggregate_deltas = orig
    server_model = captured["server"].trainer.model
    result = {
        "source": "reference tests/fedavg_tests.py:44-175 (aggregated server model, never asserted there)",
        "num_samples": captured["num_samples"],
        "baseline": {"layer.weight": [f32hex(v) for v in np.arange(10, dtype=np.float32)],
                     "head.weight": [f32hex(1.0)]},
        "payloads": [{n: [f32hex(v) for v in t.reshape(-1).numpy()] for n, t in p.items()}
                     for p in captured["payloads"]],
        "aggregated": {n: [f32hex(v) for v in t.reshape(-1).numpy()]
                       for n, t in server_model.state_dict().items()},
    }
    return result


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    workdir = tempfile.mkdtemp(prefix="golden_")
    # transformers' import-time version checks must see the real packages, before boot_reference's stub
    # finder turns the missing ones into mocks: build the HuggingFace models first
    for case in cases():
        if case.get("model") in HF_MODELS and (not args.only or case["name"] == args.only):
            make_model(case["model"])
    boot_reference(args.reference, workdir)
    os.chdir(workdir)
    if not args.only:
        dump_shapes(HERE)
        ka = run_reference_known_answer(args.reference)
        with open(os.path.join(HERE, "known_answer_fedavg_tests.json"), "w") as f:
            json.dump(ka, f, indent=1)
    cases_path = os.path.join(HERE, "fedavg_cases.json")
    full_path = os.path.join(HERE, "fedavg_full_small.npz")
    results = []
    full = {}
    if args.only and os.path.exists(cases_path):  # merge into the existing fixtures
        with open(cases_path) as f:
            results = [c for c in json.load(f)["cases"] if c["recipe"]["name"] != args.only]
        with np.load(full_path, allow_pickle=False) as z:
            full = {k: z[k] for k in z.files if not k.startswith(args.only + "/")}
    for case in cases():
        if args.only and case["name"] != args.only:
            continue
        if args.only and case.get("model") in HF_MODELS:
            dump_shapes(HERE, (case["model"],))
        print("case", case["name"], flush=True)
        runner = {"gan": run_gan_case, "he": run_he_case}.get(case.get("mode"), run_case)
        out, _ = runner(case)
        arrays = out.pop("_full", None)
        if arrays:
            for key, arr in arrays.items():
                full[f"{case['name']}/{key}"] = arr
        results.append({"recipe": case, "expected": out})
    order = {c["name"]: i for i, c in enumerate(cases())}
    results.sort(key=lambda c: order.get(c["recipe"]["name"], 1 << 30))
    with open(cases_path, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "synth": "oracle/synth.py",
                   "nan_policy": "NaN outputs canonicalised to 0x7fc00000 before hashing",
                   "cases": results}, f, indent=1)
    np.savez_compressed(full_path, **full)
    print("wrote", len(results), "cases")


if __name__ == "__main__":
    main()
