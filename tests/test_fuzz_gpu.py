"""Seeded random-shape parity sweep of the fused FedAvg kernel (the hot path) through the C ABI.

The golden fixtures pin the kernel on the reference's own model shapes; this sweep drives
``plato_agg_fedavg_weights`` / ``plato_agg_fedavg_deltas`` (``FedAvgEngine.launch_fedavg``) over
shapes and values no fixture holds — any K from 1 to 300, fp32 arenas of 0 to 70,000 elements
(ragged float4 tails included), 0 to 40 int64 entries, clients in a permuted order, a second
per-client scalar (Pisces) or none — and over special values: NaN, +-inf, +-0, subnormals, values
near FLT_MAX, int64 extremes whose differences wrap, weights that are 0, negative, subnormal or
huge.  Each case is compared bit for bit with the oracle's restatement of the reference's op
sequence (``oracle/fedavg_oracle.py`` fedavg_numpy / deltas_numpy, pinned to the reference's
fixtures by tests/test_oracle.py); NaN payload bits are not compared.
Reference: plato/algorithms/fedavg.py:13-37, plato/servers/fedavg.py:137-159.
"""

import numpy as np
import pytest
import torch

from oracle import fedavg_oracle as ref
from plato_amd.arena import ArenaLayout
from plato_amd.engine import ClientSlab, DeviceArena, FedAvgEngine, fp32_weights
from tests import golden_cases as G

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
N_CASES = 48

SPECIAL_F32 = np.array([np.nan, np.inf, -np.inf, 0.0, -0.0, 1e-45, -1e-45, 1.17e-38, 3.4e38, -3.4e38, 1.0, -1.0],
                       dtype=np.float32)
SPECIAL_I64 = np.array([0, 1, -1, 2**62, -2**62, 2**63 - 1, -2**63, 2**24 + 1, -(2**24 + 1), 2**53 + 1],
                       dtype=np.int64)


def _case(seed: int):
    rng = np.random.default_rng(1000 + seed)
    k = int(rng.choice([1, 2, 3, 5, 8, 17, 64, 128, 129, 200, 300]))
    n_f = int(rng.choice([0, 1, 3, 4, 5, 63, 64, 65, 255, 257, 1023, 4097, 16_387, 70_001]))
    n_i = int(rng.choice([0, 0, 1, 2, 7, 20, 40]))
    if n_f == 0 and n_i == 0:
        n_f = 5
    special = seed % 3 == 0
    base_f = (rng.standard_normal(n_f) * 0.05).astype(np.float32)
    xs_f = (base_f[None, :] + rng.standard_normal((k, n_f)).astype(np.float32) * np.float32(0.01)).astype(np.float32)
    base_i = rng.integers(0, 10_000, n_i, dtype=np.int64)
    xs_i = base_i[None, :] + rng.integers(0, 9, (k, n_i), dtype=np.int64)
    if special:
        for arr in (base_f, xs_f.reshape(-1)):
            if arr.size:
                m = rng.random(arr.size) < 0.02
                arr[m] = rng.choice(SPECIAL_F32, int(m.sum()))
        for arr in (base_i, xs_i.reshape(-1)):
            if arr.size:
                m = rng.random(arr.size) < 0.2
                arr[m] = rng.choice(SPECIAL_I64, int(m.sum()))
    kind = seed % 4
    if kind == 0:  # fedavg: num_samples / total
        ns = rng.integers(100, 2000, k)
        weights = [float(n) / float(ns.sum()) for n in ns]
    elif kind == 1:  # equal
        weights = [1.0 / k] * k
    elif kind == 2:  # arbitrary signs and magnitudes
        weights = list(rng.standard_normal(k) * 10.0 ** rng.integers(-3, 3, k))
    else:  # zeros, subnormals, huge
        weights = list(rng.choice([0.0, -0.0, 1e-42, -1e-40, 1e30, 0.5, -2.0, 1.0 / 3.0], k))
    scales = list(rng.uniform(0.1, 3.0, k)) if seed % 5 == 1 else None
    order = list(rng.permutation(k))
    deltas = seed % 6 == 5
    return k, n_f, n_i, base_f, xs_f, base_i, xs_i, weights, scales, order, deltas


@pytest.fixture(scope="module")
def engine():
    return FedAvgEngine(DEV)


@pytest.mark.parametrize("seed", range(N_CASES))
def test_fused_kernel_random_shapes_match_oracle(engine, seed):
    k, n_f, n_i, base_f, xs_f, base_i, xs_i, weights, scales, order, deltas = _case(seed)
    dev = torch.device(DEV)
    layout = ArenaLayout([], n_f, n_i)
    base = DeviceArena(layout, dev)
    slab = ClientSlab(layout, k, dev)
    base.f32[:n_f].copy_(torch.from_numpy(base_f))
    base.i64[:n_i].copy_(torch.from_numpy(base_i))
    for r in range(k):
        slab.f32[r][:n_f].copy_(torch.from_numpy(xs_f[r]))
        slab.i64[r][:n_i].copy_(torch.from_numpy(xs_i[r]))
    pf, pi = slab.row_pointers(order)
    tf, ti = torch.from_numpy(pf).to(dev), torch.from_numpy(pi).to(dev)
    w = torch.from_numpy(fp32_weights([weights[j] for j in order])).to(dev)
    s = None if scales is None else torch.from_numpy(fp32_weights([scales[j] for j in order])).to(dev)
    out_f = torch.full((layout.row_f32,), float("nan"), device=dev)
    out_i = torch.full((max(layout.row_i64, 1),), float("nan"), device=dev)
    if deltas:  # aggregate_deltas on client deltas (x - b formed on the host, as the oracle does)
        with np.errstate(over="ignore", invalid="ignore"):
            d_f = [np.subtract(xs_f[j], base_f, dtype=np.float32) for j in order]
            d_i = [(xs_i[j] - base_i) for j in order]
        for r, j in enumerate(order):
            slab.f32[j][:n_f].copy_(torch.from_numpy(d_f[r]))
            slab.i64[j][:n_i].copy_(torch.from_numpy(d_i[r]))
        engine.launch_fedavg(layout, tf, ti, w, s, k, None, None, out_f, out_i)
        with np.errstate(over="ignore", invalid="ignore"):
            want_f, want_i = ref.deltas_numpy(d_f, d_i, [weights[j] for j in order],
                                              None if scales is None else [scales[j] for j in order])
    else:
        engine.launch_fedavg(layout, tf, ti, w, s, k, base.f32, base.i64, out_f, out_i)
        with np.errstate(over="ignore", invalid="ignore"):
            want_f, want_i = ref.fedavg_numpy(base_f, base_i, [xs_f[j] for j in order], [xs_i[j] for j in order],
                                              [weights[j] for j in order],
                                              None if scales is None else [scales[j] for j in order])
    torch.cuda.synchronize()
    got_f = out_f[:n_f].cpu().numpy()
    got_i = out_i[:n_i].cpu().numpy()
    bad = np.nonzero(G.canon(got_f).view(np.uint32) != G.canon(want_f).view(np.uint32))[0]
    assert bad.size == 0, (f"K={k} n_f32={n_f} deltas={deltas}: {bad.size} fp32 mismatches, first at {bad[0]}: "
                           f"got {got_f[bad[0]]!r} want {want_f[bad[0]]!r}")
    bad_i = np.nonzero(G.canon(got_i).view(np.uint32) != G.canon(want_i).view(np.uint32))[0]
    assert bad_i.size == 0, f"K={k} n_i64={n_i} deltas={deltas}: int64-entry mismatches at {bad_i[:5]}"


def _widen(bits: np.ndarray) -> np.ndarray:
    """bf16 bit patterns -> float32 (model_dequantize's .to(float32), exact)."""
    return (bits.astype(np.uint32) << 16).view(np.float32)


@pytest.mark.parametrize("seed", range(24))
def test_bf16_kernel_random_shapes_match_oracle(seed):
    """plato_agg_fedavg_weights_bf16 (model_quantize / model_dequantize codec, plato/processors/
    model_dequantize.py:15-18, then the FedAvg chain) on random shapes and bf16 bit patterns — NaN,
    +-inf, subnormal bf16 included — against the oracle on the widened payloads."""
    from plato_amd import _lib

    k, n_f, n_i, base_f, xs_f, base_i, _, weights, scales, order, _ = _case(7000 + seed)
    rng = np.random.default_rng(seed)
    dev = torch.device(DEV)
    # the payload: the clients' fp32 values rounded to bf16 by truncation, then random patterns mixed in
    bits_f = (xs_f.view(np.uint32) >> 16).astype(np.uint16)
    bits_i = (rng.integers(0, 10_000, (k, n_i)).astype(np.float32).view(np.uint32) >> 16).astype(np.uint16)
    if seed % 2 == 0:
        for arr in (bits_f.reshape(-1), bits_i.reshape(-1)):
            if arr.size:
                m = rng.random(arr.size) < 0.03
                arr[m] = rng.integers(0, 1 << 16, int(m.sum())).astype(np.uint16)
    pad_f, pad_i = max(8, -(-n_f // 8) * 8), max(8, -(-n_i // 8) * 8)  # 16-byte rows
    xf = torch.zeros((k, pad_f), dtype=torch.int16, device=dev)
    xi = torch.zeros((k, pad_i), dtype=torch.int16, device=dev)
    xf[:, :n_f].copy_(torch.from_numpy(bits_f.view(np.int16)))
    xi[:, :n_i].copy_(torch.from_numpy(bits_i.view(np.int16)))
    tf = torch.tensor([xf[j].data_ptr() for j in order], dtype=torch.int64, device=dev)
    ti = torch.tensor([xi[j].data_ptr() for j in order], dtype=torch.int64, device=dev)
    w = torch.from_numpy(fp32_weights([weights[j] for j in order])).to(dev)
    s = None if scales is None else torch.from_numpy(fp32_weights([scales[j] for j in order])).to(dev)
    row = max(64, -(-n_f // 64) * 64)  # the arenas' row padding (ArenaLayout.row_f32)
    bf = torch.zeros(row, device=dev)
    bf[:n_f].copy_(torch.from_numpy(base_f))
    bi = torch.from_numpy(base_i).to(dev)
    out_f = torch.full((row,), float("nan"), device=dev)
    out_i = torch.full((max(n_i, 1),), float("nan"), device=dev)
    h = torch.cuda.current_stream().cuda_stream
    _lib.call("plato_agg_fedavg_weights_bf16", tf.data_ptr(), ti.data_ptr() if n_i else None, w.data_ptr(),
              None if s is None else s.data_ptr(), k, bf.data_ptr(), bi.data_ptr() if n_i else None,
              out_f.data_ptr(), out_i.data_ptr() if n_i else None, n_f, n_i, h)
    with np.errstate(over="ignore", invalid="ignore"):
        want_f, want_i = ref.fedavg_numpy(base_f, base_i, [_widen(bits_f[j]) for j in order],
                                          [_widen(bits_i[j]) for j in order], [weights[j] for j in order],
                                          None if scales is None else [scales[j] for j in order])
    torch.cuda.synchronize()
    got_f, got_i = out_f[:n_f].cpu().numpy(), out_i[:n_i].cpu().numpy()
    bad = np.nonzero(G.canon(got_f).view(np.uint32) != G.canon(want_f).view(np.uint32))[0]
    assert bad.size == 0, f"K={k} n_f32={n_f}: {bad.size} mismatches, first at {bad[0]}"
    bad_i = np.nonzero(G.canon(got_i).view(np.uint32) != G.canon(want_i).view(np.uint32))[0]
    assert bad_i.size == 0, f"K={k} n_i64={n_i}: int64-entry mismatches at {bad_i[:5]}"


@pytest.mark.parametrize("seed", range(12))
def test_qsgd_kernel_random_layouts_match_oracle(seed):
    """plato_agg_fedavg_qsgd through the QSGD processor (model_dequantize_qsgd.py:34-60 restated by
    oracle/qsgd.py) on random layouts (tests/test_fuzz_variants_gpu.py), random quantization levels,
    every code byte, and per-entry max_v that is negative, zero, subnormal, huge, inf or NaN."""
    from oracle import qsgd as Q
    from plato_amd import weights as W
    from plato_amd.processors.qsgd import Processor
    from tests.test_fuzz_variants_gpu import _spec

    spec, k = _spec(100 + seed)
    # the wire header holds each dimension as a big-endian int16 (model_quantize_qsgd.py:130-139)
    spec = [(n, (8, -(-shape[0] // 8)) if len(shape) == 1 and shape[0] > 32767 else shape, r) for n, shape, r in spec]
    layout = ArenaLayout.from_shapes(spec)
    rng = np.random.default_rng(seed)
    level = int(rng.choice([2, 3, 16, 64, 128, 129]))
    bf = (rng.standard_normal(layout.n_f32) * 0.05).astype(np.float32)
    bi = rng.integers(-50, 50, layout.n_i64)
    baseline = layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi))
    max_vs = np.array([0.37, 1.0, 2.5, -0.75, 0.0, 1e-45, 3e38, np.inf, np.nan], dtype=np.float32)
    proc = Processor(quantization_level=level)
    wires = []
    for _ in range(k):
        wires.append({e.name: Q.encode_layer(rng.integers(0, 256, e.numel).astype(np.uint8),
                                             np.float32(rng.choice(max_vs) if rng.random() < 0.3 else rng.uniform(0.01, 3)),
                                             e.shape) for e in layout.entries})
    deq = []
    for w in wires:
        vals = {n: Q.decode_layer(b, level).reshape(-1) for n, b in w.items()}
        parts_f = [vals[e.name] for e in layout.entries if e.region == "f32"]
        parts_i = [vals[e.name] for e in layout.entries if e.region == "i64"]
        deq.append((np.concatenate(parts_f) if parts_f else np.zeros(0, np.float32),
                    np.concatenate(parts_i) if parts_i else np.zeros(0, np.float32)))
    weights = W.fedavg(list(rng.integers(1, 1000, k)))
    order = list(rng.permutation(k))
    engine = FedAvgEngine(DEV)
    rnd = engine.begin(baseline, k, "qsgd")
    rnd.put_baseline(baseline)
    for slot in range(k):
        rnd.put_client(slot, proc.process(wires[slot]))
    rnd.launch([weights[i] for i in order], order=order)
    got = rnd.result()
    with np.errstate(over="ignore", invalid="ignore"):
        exp_f, exp_i = ref.fedavg_numpy(bf, bi, [deq[i][0] for i in order], [deq[i][1] for i in order],
                                        [weights[i] for i in order])

    def flat(sd, region):
        parts = [sd[e.name].reshape(-1).float() for e in layout.entries if e.region == region]
        return torch.cat(parts).numpy() if parts else np.zeros(0, np.float32)

    assert G.canon(flat(got, "f32")).tobytes() == G.canon(exp_f).tobytes(), (level, k)
    assert G.canon(flat(got, "i64")).tobytes() == G.canon(exp_i).tobytes(), (level, k)
