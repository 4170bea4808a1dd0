"""QSGD payloads decoded inside the FedAvg kernel (plato_agg_fedavg_qsgd) vs the reference.

The qsgd_codec_* fixtures hold what the reference's model_dequantize_qsgd
processor + FedAvg produced from the same wire bytes; here the bytes go
through plato_amd.processors.qsgd.Processor (headers parsed, codes gathered),
one byte per element to HBM, and the kernel's decode tables.  Bit-exact.
"""

import asyncio
import types

import numpy as np
import pytest
import torch

from oracle import fedavg_oracle as ref
from oracle import qsgd as Q
from oracle import synth
from plato_amd import weights as W
from plato_amd.arena import ArenaLayout
from plato_amd.engine import FedAvgEngine
from plato_amd.processors.qsgd import Processor
from tests import golden_cases as G

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
QSGD = [c for c in G.load_cases() if c["recipe"].get("codec") == "qsgd"
        and G.plain_fedavg_weights(c["recipe"])]


@pytest.fixture(scope="module")
def engine():
    return FedAvgEngine(DEV)


def _flat(layout, sd, region):
    parts = [sd[e.name].reshape(-1).float() for e in layout.entries if e.region == region]
    return torch.cat(parts).numpy() if parts else np.zeros(0, np.float32)


@pytest.mark.parametrize("case", QSGD, ids=[c["recipe"]["name"] for c in QSGD])
def test_qsgd_server_hook_matches_reference(engine, case):
    from plato_amd.servers import FusedAggregationMixin

    recipe, exp = case["recipe"], case["expected"]
    layout = ArenaLayout.from_shapes(G.model_spec(recipe["model"]))
    k, seed = recipe["k"], recipe["seed"]
    bf, bi = synth.baseline_arena(layout.n_f32, layout.n_i64, seed)
    baseline = layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi))
    proc = Processor()
    payloads = {c: proc.process(Q.client_wire(layout.entries, seed, c)[0]) for c in range(k)}
    order = G.order_of(recipe)
    updates = [types.SimpleNamespace(client_id=c + 1, report=types.SimpleNamespace(num_samples=recipe["num_samples"][c]),
                                     payload=payloads[c], staleness=0) for c in order]

    class Server(FusedAggregationMixin):
        aggregation_device = DEV

    server = Server()
    server._plato_amd_engine = engine
    updated = asyncio.run(server.aggregate_weights(updates, baseline, [u.payload for u in updates]))
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(G.canon(_flat(layout, updated, "i64"))) == exp["updated_i64f_sha256"]
    assert G.sha(ref.trunc_to_int64(_flat(layout, updated, "i64"))) == exp["loaded_i64_sha256"]
    if recipe.get("full"):
        full = G.load_full()
        assert G.canon(_flat(layout, updated, "f32")).tobytes() == \
            G.canon(full[f"{recipe['name']}/updated_f32"]).tobytes()


SPEC = [("a", (3,), "f32"), ("n0", (), "i64"), ("b", (17,), "f32"), ("c", (5, 7), "f32"), ("n1", (4,), "i64"),
        ("e", (1000,), "f32"), ("g", (4099,), "f32"), ("h", (2,), "f32"), ("big", (3, 4097), "f32")]


# the product default (libplato_agg.so) and the tuning library's FedAvg shapes: 0 the default's plain
# form, 1 the pipelined form of rounds 2-3, 5 the round-1 plain form, 6 a 256-thread shape; 2-4 are
# timing probes (not the FedAvg)
@pytest.mark.parametrize("variant", [None, 0, 1, 5, 6, 7, 13, 18, 24, 25, 29, 31, 32, 33, 36, 37, 38, 39, 40, 41, 42])
@pytest.mark.parametrize("cap,k,two", [(8, 3, False), (20, 9, True), (4096, 17, False), (64, 16, True), (1 << 20, 5, False)])
def test_qsgd_kernel_matches_oracle(engine, monkeypatch, cap, k, two, variant):
    """Chunk pieces of every alignment (caps 8/20: partial 16-byte groups everywhere;
    2^20: pieces longer than one pass), K not a multiple of the 8-client table batch,
    all 256 code values, second scalar (Pisces) on and off; every kernel variant."""
    monkeypatch.setattr(FedAvgEngine, "QSGD_CHUNK", cap)
    monkeypatch.setattr(engine, "qsgd_variant", variant)
    layout = ArenaLayout.from_shapes(SPEC)
    rng = np.random.default_rng(cap + k)
    bf = rng.standard_normal(layout.n_f32).astype(np.float32)
    bi = rng.integers(-50, 50, layout.n_i64)
    baseline = layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi))
    proc = Processor(quantization_level=32)
    wires = []
    for c in range(k):
        ents = {}
        for e in layout.entries:
            codes = rng.integers(0, 256, e.numel).astype(np.uint8)
            ents[e.name] = Q.encode_layer(codes, np.float32(rng.uniform(0.01, 3.0)), e.shape)
        wires.append(ents)
    pays = [proc.process(w) for w in wires]
    deq = []
    for w in wires:
        vals = {n: Q.decode_layer(b, 32).reshape(-1) for n, b in w.items()}
        deq.append((np.concatenate([vals[e.name] for e in layout.entries if e.region == "f32"]),
                    np.concatenate([vals[e.name] for e in layout.entries if e.region == "i64"])))
    ns = list(rng.integers(1, 1000, k))
    weights = W.fedavg(ns)
    scales = list(rng.uniform(0.5, 1.5, k)) if two else None
    order = list(rng.permutation(k))
    rnd = engine.begin(baseline, k, "qsgd")
    rnd.put_baseline(baseline)
    for slot in range(k):
        rnd.put_client(slot, pays[slot])
    rnd.launch([weights[i] for i in order], None if scales is None else [scales[i] for i in order], order=order)
    got = rnd.result()
    exp_f, exp_i = ref.fedavg_numpy(bf, bi, [deq[i][0] for i in order], [deq[i][1] for i in order],
                                    [weights[i] for i in order], None if scales is None else [scales[i] for i in order])
    assert G.canon(_flat(layout, got, "f32")).tobytes() == G.canon(exp_f).tobytes()
    assert G.canon(_flat(layout, got, "i64")).tobytes() == G.canon(exp_i).tobytes()


@pytest.mark.parametrize("variant", [None, 7, 13, 24, 25, 28])
def test_qsgd_decode_at_float32_extremes(engine, monkeypatch, variant):
    """max_v at the ends of float32 (subnormal, tiny, huge, so that |zeta| * max_v / divisor overflows or
    lands among the subnormals) and divisors of awkward quotients: the arithmetic decode (a float64
    reciprocal product, variants 7 and 9) gives the float32 division's bits, like the table kernel."""
    monkeypatch.setattr(engine, "qsgd_variant", variant)
    spec = [("a", (4096,), "f32"), ("b", (333,), "f32"), ("c", (8192,), "f32"), ("n", (), "i64")]
    layout = ArenaLayout.from_shapes(spec)
    rng = np.random.default_rng(5)
    bf = (rng.standard_normal(layout.n_f32) * 1e-3).astype(np.float32)
    bi = rng.integers(-50, 50, layout.n_i64)
    baseline = layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi))
    extremes = [1e-45, 3e-39, 1.1754944e-38, 7e-36, 2.5e37, 3.4e38, 0.37, 1.0, 1e-8]
    k = len(extremes)
    for level in (3, 64, 129):
        proc = Processor(quantization_level=level)
        wires = []
        for c in range(k):
            ents = {}
            for e in layout.entries:
                codes = rng.integers(0, 256, e.numel).astype(np.uint8)
                ents[e.name] = Q.encode_layer(codes, np.float32(extremes[(c + len(ents)) % k]), e.shape)
            wires.append(ents)
        pays = [proc.process(w) for w in wires]
        deq = []
        for w in wires:
            vals = {n: Q.decode_layer(b, level).reshape(-1) for n, b in w.items()}
            deq.append((np.concatenate([vals[e.name] for e in layout.entries if e.region == "f32"]),
                        np.concatenate([vals[e.name] for e in layout.entries if e.region == "i64"])))
        weights = W.fedavg(list(range(1, k + 1)))
        rnd = engine.begin(baseline, k, "qsgd")
        rnd.put_baseline(baseline)
        for slot in range(k):
            rnd.put_client(slot, pays[slot])
        rnd.launch(weights)
        got = rnd.result()
        exp_f, exp_i = ref.fedavg_numpy(bf, bi, [d[0] for d in deq], [d[1] for d in deq], weights)
        assert G.canon(_flat(layout, got, "f32")).tobytes() == G.canon(exp_f).tobytes(), level
        assert G.canon(_flat(layout, got, "i64")).tobytes() == G.canon(exp_i).tobytes(), level
