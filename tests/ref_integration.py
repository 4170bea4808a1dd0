"""Run the product's server hooks inside the REAL reference server (CPU, this container).

Launched as a subprocess by tests/test_reference_integration.py, only where
/root/reference exists.  It boots TL-System/plato like the fixture generator
does, builds ``class Server(FusedAggregationMixin, plato.servers.fedavg.Server)``
and lets the reference's own ``_process_reports`` (plato/servers/fedavg.py:161)
dispatch to the product hook, call ``algorithm.load_weights`` and fire its
callbacks.  No GPU exists here, so the engine is replaced by a test double with
the same begin/put/launch/ready/result API whose arithmetic is the oracle; the
point is the wiring (hook signature, dispatch, returned dict, load_weights
truncation, total_samples), the numerics are covered on the GPU.
"""

import asyncio
import json
import os
import sys
import tempfile
from collections import OrderedDict

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(HERE, "golden"))

import make_golden as MG  # noqa: E402  (boot helpers: stubs + config)
from oracle import fedavg_oracle as ref  # noqa: E402
from oracle import synth  # noqa: E402
from plato_amd.arena import ArenaLayout  # noqa: E402


class OracleRound:
    def __init__(self, layout, capacity):
        self.layout, self.slots, self.base = layout, {}, None

    def put_baseline(self, sd):
        self.base = sd

    def put_client(self, slot, sd, what=None):
        self.slots[slot] = sd

    def adopt(self, slot, sd):
        return False

    def _flat(self, sd, region):
        parts = [sd[e.name].reshape(-1) for e in self.layout.entries if e.region == region]
        if not parts:
            return np.zeros(0, np.float32 if region == "f32" else np.int64)
        return torch.cat(parts).numpy()

    def launch(self, weights, scales=None, order=None, deltas=False):
        order = list(range(len(weights))) if order is None else list(order)
        xs = [self.slots[i] for i in order]
        self.order_seen = order
        if deltas:
            nf, ni = ref.deltas_numpy([self._flat(x, "f32") for x in xs], [self._flat(x, "i64") for x in xs],
                                      weights, scales)
        else:
            nf, ni = ref.fedavg_numpy(self._flat(self.base, "f32"), self._flat(self.base, "i64"),
                                      [self._flat(x, "f32") for x in xs], [self._flat(x, "i64") for x in xs],
                                      weights, scales)
        self.out = self.layout.unpack(torch.from_numpy(nf), torch.from_numpy(ni))

    def launch_w64(self, weights64, weights_i64=None, order=None, deltas=False):
        order = list(range(len(weights64))) if order is None else list(order)
        xs = [self.slots[i] for i in order]
        assert deltas
        nf, ni = ref.w64_numpy([self._flat(x, "f32") for x in xs], [self._flat(x, "i64") for x in xs], weights64,
                               weights64 if weights_i64 is None else weights_i64)
        self.out = self.layout.unpack(torch.from_numpy(nf), torch.from_numpy(ni))

    def ready(self):
        return True

    def wait(self):
        pass

    timings = {}

    def algorithmic_bytes(self):
        return 0

    def result(self):
        return self.out


class OracleEngine:
    def begin(self, template, capacity, codec="native"):
        self.last = OracleRound(ArenaLayout.from_state_dict(template), capacity)
        return self.last

    def release_arrivals(self):
        pass

    def weighted_sum(self, vectors, weights):
        acc = np.zeros(np.asarray(vectors[0]).size, dtype=np.float64)
        for v, w in zip(vectors, weights):
            acc = acc + np.asarray(v, dtype=np.float64) * w
        return torch.from_numpy(acc)


def _case(name):
    sys.path.insert(0, ROOT)
    from tests import golden_cases as G

    return next(c for c in G.load_cases() if c["recipe"]["name"] == name), G


def _recipe_inputs(recipe, model):
    entries, nf, ni = MG.layout_of(model.state_dict())
    k, seed = recipe["k"], recipe["seed"]
    bf, bi = synth.baseline_arena(nf, ni, seed)
    xs = [synth.client_arena(bf, bi, seed, c) for c in range(k)]
    baseline = MG.unpack(entries, torch.from_numpy(bf), torch.from_numpy(bi))
    payloads = [MG.unpack(entries, torch.from_numpy(x[0]), torch.from_numpy(x[1])) for x in xs]
    return entries, baseline, payloads


def _spy_load(server):
    got = {}
    orig = server.algorithm.load_weights

    def spy(w):
        got["updated"] = OrderedDict((n, t.clone()) for n, t in w.items())
        return orig(w)

    server.algorithm.load_weights = spy
    return got


def more_wiring():
    """Cross-silo, RL, HE and async-wall-time callers of the hooks, in the reference process."""
    import copy

    from plato.servers import fedavg, fedavg_cs

    from plato_amd.servers import FusedAggregationMixin
    from plato_amd.servers.variants import HEHybridMixin, RLDeltasAggregationMixin

    res = {}
    # cross-silo: fedavg_cs._process_reports (servers/fedavg_cs.py:161-199) -> aggregate_weights
    case, G = _case("cross_silo_resnet18_k6")
    recipe = case["recipe"]
    eng = OracleEngine()

    class CS(FusedAggregationMixin, fedavg_cs.Server):
        def aggregation_engine(self):
            return eng

    model = MG.make_model("resnet18")
    entries, baseline, payloads = _recipe_inputs(recipe, model)
    server = CS(model=lambda: model)
    server.init_trainer()
    server.algorithm.load_weights(copy.deepcopy(baseline))
    server.updates = MG.make_updates(recipe["num_samples"], payloads, G.order_of(recipe), [0] * recipe["k"])
    orig_event = server.callback_handler.call_event
    server.callback_handler.call_event = lambda ev, *a, **kw: None if ev == "on_clients_processed" else \
        orig_event(ev, *a, **kw)
    got = _spy_load(server)
    asyncio.run(server._process_reports())
    res["cross_silo"] = MG.sha(MG.canon(MG.flatten(entries, got["updated"], "f32", torch.float32))) == \
        case["expected"]["updated_f32_sha256"]

    # RL: the reference's RLServer with the mixin's aggregate_deltas (rl_server.py:45-80)
    case, G = _case("rl_float64_resnet18_k6")
    recipe = case["recipe"]
    base_cls = MG.rl_server_class()

    class RL(RLDeltasAggregationMixin, base_cls):
        def aggregation_engine(self):
            return eng

    model = MG.make_model("resnet18")
    entries, baseline, payloads = _recipe_inputs(recipe, model)
    server = RL(agent=MG._StubAgent(MG.rl_action(recipe)), model=lambda: model)
    server.init_trainer()
    server.algorithm.load_weights(copy.deepcopy(baseline))
    server.updates = MG.make_updates(recipe["num_samples"], payloads, G.order_of(recipe), [0] * recipe["k"])
    got = _spy_load(server)
    asyncio.run(server._process_reports())
    res["rl"] = MG.sha(MG.canon(MG.flatten(entries, got["updated"], "f32", torch.float32))) == \
        case["expected"]["updated_f32_sha256"]

    # HE: the mixin's _fedavg_hybrid with the reference's homo_enc helpers (fedavg_he.py:66-106)
    case, G = _case("he_plain_lenet5_k5")
    recipe = case["recipe"]
    from plato.utils import homo_enc

    from tests.test_oracle import he_vectors

    vecs = he_vectors(recipe)
    msgs = [homo_enc.wrap_encrypted_model(v, torch.zeros(len(recipe["encrypt_indices"])),
                                          list(recipe["encrypt_indices"])) for v in vecs]
    updates = MG.make_updates(recipe["num_samples"], msgs, list(range(recipe["k"])), [0] * recipe["k"])

    class HE(HEHybridMixin):
        context = None
        trainer = type("T", (), {"zeros": staticmethod(lambda shape: torch.zeros(shape))})()

        def aggregation_engine(self):
            return eng

    orig = homo_enc.deserialize_weights
    homo_enc.deserialize_weights = lambda w, ctx: w
    try:
        out = HE()._fedavg_hybrid(updates)
    finally:
        homo_enc.deserialize_weights = orig
    res["he"] = MG.sha(np.ascontiguousarray(out["unencrypted_weights"].numpy())) == \
        case["expected"]["unencrypted_avg_sha256"]

    # async simulated wall time: the reference's _process_clients orders the updates (base.py:925-1091)
    case, G = _case("async_wall_resnet18_k12")
    recipe = case["recipe"]

    class Async(FusedAggregationMixin, fedavg.Server):
        def aggregation_engine(self):
            return eng

    model = MG.make_model("resnet18")
    entries, baseline, payloads = _recipe_inputs(recipe, model)
    server = Async(model=lambda: model)
    server.init_trainer()
    server.algorithm.load_weights(copy.deepcopy(baseline))
    server.current_round = recipe["current_round"]
    got = _spy_load(server)
    order = asyncio.run(MG.drive_async_wall_time(server, recipe, payloads))
    res["async_order"] = order == case["expected"]["updates_order"]
    res["async_model"] = MG.sha(MG.canon(MG.flatten(entries, got["updated"], "f32", torch.float32))) == \
        case["expected"]["updated_f32_sha256"]
    return res


def main():
    out_path = sys.argv[1]
    workdir = tempfile.mkdtemp(prefix="refint_")
    MG.boot_reference(os.environ.get("PLATO_REFERENCE", "/root/reference"), workdir)
    os.chdir(workdir)
    from plato.servers import fedavg

    from plato_amd.servers import FusedAggregationMixin

    calls = {"hook": 0, "load": 0, "cb_received": 0, "cb_aggregated": 0}

    class Server(FusedAggregationMixin, fedavg.Server):
        def aggregation_engine(self):
            calls["hook"] += 1
            return OracleEngine()

    model = MG.make_model("resnet18")
    server = Server(model=lambda: model)
    server.init_trainer()
    entries, nf_, ni_ = MG.layout_of(model.state_dict())
    k, seed = 6, 31
    bf, bi = synth.baseline_arena(nf_, ni_, seed)
    xs = [synth.client_arena(bf, bi, seed, c) for c in range(k)]
    baseline = MG.unpack(entries, torch.from_numpy(bf), torch.from_numpy(bi))
    payloads = [MG.unpack(entries, torch.from_numpy(x[0]), torch.from_numpy(x[1])) for x in xs]
    server.algorithm.load_weights({n: t.clone() for n, t in baseline.items()})
    ns = synth.num_samples(k, seed)
    server.updates = MG.make_updates(ns, payloads, list(range(k)), [0] * k)
    orig_load = server.algorithm.load_weights

    def spy_load(w):
        calls["load"] += 1
        calls["load_dtypes"] = sorted({str(t.dtype) for t in w.values()})
        return orig_load(w)

    server.algorithm.load_weights = spy_load

    class CB:
        def __getattr__(self, name):
            def f(*a, **kw):
                if name == "on_weights_received":
                    calls["cb_received"] += 1
                if name == "on_weights_aggregated":
                    calls["cb_aggregated"] += 1
            return f

    server.callback_handler.add_callbacks([CB()])
    asyncio.run(server._process_reports())
    state = model.state_dict()
    exp = ref.fedavg_torch_ops(baseline, payloads, num_samples=ns)
    same = all(torch.equal(state[n], exp[n].to(state[n].dtype)) for n in state)
    calls["model_matches_reference_chain"] = bool(same)
    calls["total_samples"] = server.total_samples == sum(ns)
    # clones: each payload tensor with its own storage, as a client's state_dict has
    calls["ingest"] = ingest_wiring(fedavg, model, [OrderedDict((n, t.clone()) for n, t in p.items())
                                                    for p in payloads[:2]])
    calls["more"] = more_wiring()
    with open(out_path, "w") as f:
        json.dump(calls, f)


def ingest_wiring(fedavg, model, payloads):
    """WireIngestMixin inside the reference's own arrival path (servers/base.py:775-857).

    The reference's _client_report_arrived and _client_chunk_arrived run
    unmodified; the mixin replaces the join + pickle.loads and the re-pickling
    size accounting.  Compared with an unmodified reference server fed the same
    socket chunks: the payload handed to process_client_info and comm_overhead.
    """
    import pickle
    import types

    from plato_amd.servers import WireIngestMixin

    class Wire(WireIngestMixin, fedavg.Server):
        ingest_pinned = False

    def run(cls, simulated=False):
        from plato.config import Config

        server = cls(model=lambda: model)
        server.init_trainer()
        handed = []

        async def process_client_info(client_id, sid):
            handed.append(server.client_payload[sid])

        server.process_client_info = process_client_info
        server.comm_simulation = simulated  # files (:775-811) or socket.io chunks (:813-857)
        server.comm_overhead = 0.0
        for c, payload in enumerate(payloads):
            sid = f"sid{c}"
            server.training_clients[c + 1] = {"start_time": 0.0, "starting_round": 0}
            report = types.SimpleNamespace(client_id=c + 1, num_samples=10, training_time=0.0,
                                           processing_time=0.0, comm_time=0.0)
            data = pickle.dumps(payload)
            if simulated:  # what the client's _send writes (clients/base.py:372-386)
                os.makedirs(Config().params["checkpoint_path"], exist_ok=True)
                name = Config().trainer.model_name.replace("/", "_")
                with open(f"{Config().params['checkpoint_path']}/{name}_client_{c + 1}.pth", "wb") as f:
                    pickle.dump(payload, f)
                server.uplink_comm_time = {}
                asyncio.run(server._client_report_arrived(sid, c + 1, pickle.dumps(report)))
                continue
            asyncio.run(server._client_report_arrived(sid, c + 1, pickle.dumps(report)))
            for i in range(0, len(data), 2**20):
                asyncio.run(server._client_chunk_arrived(sid, data[i:i + 2**20]))
            asyncio.run(server._client_payload_arrived(sid, c + 1))
            asyncio.run(server._client_payload_done(sid, c + 1))
        return handed, server.comm_overhead

    result = {}
    for mode, simulated in (("socket", False), ("simulated", True)):
        got, got_mb = run(Wire, simulated)
        exp, exp_mb = run(fedavg.Server, simulated)
        same = len(got) == len(exp) == len(payloads) and all(
            list(g) == list(e) and all(torch.equal(g[k], e[k]) and g[k].dtype == e[k].dtype for k in e)
            for g, e in zip(got, exp))
        result[mode] = {"payload_matches": bool(same),
                        "arena_backed": all(type(g).__name__ == "ArenaStateDict" for g in got),
                        "comm_overhead_bytes": [got_mb * 1024**2, exp_mb * 1024**2]}
    return result


if __name__ == "__main__":
    main()
