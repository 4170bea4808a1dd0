"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the FedAvg aggregation path.

Never imported by the product path (plato_amd/); only tests/, the smoke test
in __graft_entry__.py and bench.py's ``cpu_baseline`` leg use it, as the
checker.  Two restatements of the reference's arithmetic:

1. ``fedavg_numpy`` — sequential fp32 numpy over flat arenas, one explicit
   rounding per op (numpy ufuncs never contract to FMA):

       acc = +0 ; for i in self.updates order:
           d   = fp32(x_i - b)                  plato/algorithms/fedavg.py:23
           t   = fp32(d * fp32(n_i / N))        plato/servers/fedavg.py:154
           acc = fp32(acc + t)                  plato/servers/fedavg.py:154 (+=)
       new = fp32(b + acc)                      plato/algorithms/fedavg.py:35
       int64 keys: d = int64(x - b) -> fp32 ; new = fp32(fp32(b) + acc) ;
       load_state_dict truncates toward zero    plato/algorithms/fedavg.py:48

2. ``fedavg_torch_ops`` — the reference's own torch op sequence on CPU
   tensors, tensor by tensor (sub -> mul(Python float) -> add_ -> add ->
   load_state_dict copy), i.e. plato/algorithms/fedavg.py:13-48 and
   plato/servers/fedavg.py:137-159 restated without the server object.  This
   is the "port" CPU baseline bench.py times on the GPU box.

Parity pin: tests/golden/*.json were produced by the reference itself
(tests/golden/make_golden.py imports /root/reference and runs its
Server.aggregate_deltas / Algorithm chain); tests/test_oracle.py checks both
restatements against them bit for bit.
"""

from __future__ import annotations

from collections import OrderedDict
from typing import Mapping, Sequence

import numpy as np


# --------------------------------------------------------------------------
# weights
# --------------------------------------------------------------------------
def fedavg_weights(num_samples: Sequence[int]) -> list[float]:
    """n_i / N in Python double (servers/fedavg.py:140,154)."""
    total = sum(num_samples)
    return [n / total for n in num_samples]


def fedbuff_weights(k: int) -> list[float]:
    """examples/async/fedbuff/fedbuff_server.py:33,45: 1 / len(updates)."""
    return [1 / k] * k


def port_staleness_factor(staleness: int, bound: float = 10) -> float:
    """examples/async/port/port_server.py:135-144."""
    return bound / (staleness + bound)


def port_weights(num_samples: Sequence[int], staleness: Sequence[int], similarity=None,
                 similarity_weight: float = 1, staleness_weight: float = 1,
                 staleness_bound: float = 10) -> list[float]:
    """examples/async/port/port_server.py:57-103 with Python-float similarities."""
    total = sum(num_samples)
    raw = []
    for i, n in enumerate(num_samples):
        sim = 1.0 if similarity is None else similarity[i]
        factor = port_staleness_factor(staleness[i], staleness_bound)
        raw.append(n / total * ((sim + 1) / 2 * similarity_weight + factor * staleness_weight))
    return [r / sum(raw) for r in raw]


def port_weights_torch(num_samples, staleness, similarity, similarity_weight=1, staleness_weight=1,
                       staleness_bound=10):
    """examples/async/port/port_server.py:57-103 evaluated as written, with the
    similarities as the reference holds them: the Python float 1.0, or a 0-dim
    fp32 torch tensor from F.cosine_similarity."""
    import torch

    total = sum(num_samples)
    raw = []
    for i, n in enumerate(num_samples):
        sim = similarity[i]
        if not isinstance(sim, float):
            sim = torch.tensor(np.float32(sim))
        factor = port_staleness_factor(staleness[i], staleness_bound)
        raw.append(n / total * ((sim + 1) / 2 * similarity_weight + factor * staleness_weight))
    return [r / sum(raw) for r in raw]


def cosine_similarity_fp64(current_minus_previous: np.ndarray, delta: np.ndarray, eps: float = 1e-8) -> float:
    """F.cosine_similarity(a, b, dim=0) restated in fp64 (port_server.py:50)."""
    a = current_minus_previous.astype(np.float64)
    b = delta.astype(np.float64)
    return float(np.dot(a, b) / (max(np.linalg.norm(a), eps) * max(np.linalg.norm(b), eps)))


def fp32(values) -> np.ndarray:
    out = []
    for v in values:
        if hasattr(v, "item") and not isinstance(v, np.floating):
            v = v.item()  # 0-dim torch tensor (fp32): exact
        out.append(np.float32(float(v)))
    return np.asarray(out, dtype=np.float32)


# --------------------------------------------------------------------------
# 1. numpy restatement over flat arenas
# --------------------------------------------------------------------------
def fedavg_numpy(base_f32: np.ndarray, base_i64: np.ndarray, clients_f32, clients_i64,
                 weights: Sequence[float], scales: Sequence[float] | None = None):
    """Fused FedAvg (deltas -> weighted sum -> update) on flat arenas.

    Returns (new_f32, new_i64_as_f32); the int64 entries' results are fp32
    exactly as the reference's update_weights returns them.
    """
    w = fp32(weights)
    s = None if scales is None else fp32(scales)
    acc = np.zeros(base_f32.shape, dtype=np.float32)
    acc_i = np.zeros(base_i64.shape, dtype=np.float32)
    for i in range(len(w)):
        d = np.subtract(clients_f32[i], base_f32, dtype=np.float32)
        t = np.multiply(d, w[i], dtype=np.float32)
        if s is not None:
            t = np.multiply(t, s[i], dtype=np.float32)
        acc = np.add(acc, t, dtype=np.float32)
        if base_i64.size:
            if clients_i64[i].dtype == np.float32:
                # dequantized (bf16 codec) payload: fp32 tensor - int64 tensor
                # promotes to fp32 (plato/algorithms/fedavg.py:23)
                di = np.subtract(clients_i64[i], base_i64.astype(np.float32), dtype=np.float32)
            else:
                with np.errstate(over="ignore"):
                    di = (clients_i64[i].astype(np.int64) - base_i64.astype(np.int64)).astype(np.float32)
            ti = np.multiply(di, w[i], dtype=np.float32)
            if s is not None:
                ti = np.multiply(ti, s[i], dtype=np.float32)
            acc_i = np.add(acc_i, ti, dtype=np.float32)
    new_f = np.add(base_f32, acc, dtype=np.float32)
    new_i = np.add(base_i64.astype(np.float32), acc_i, dtype=np.float32)
    return new_f, new_i


def deltas_numpy(deltas_f32, deltas_i64, weights, scales=None):
    """Server.aggregate_deltas on flat arenas (servers/fedavg.py:143-157)."""
    w = fp32(weights)
    s = None if scales is None else fp32(scales)
    acc = np.zeros(deltas_f32[0].shape, dtype=np.float32)
    acc_i = np.zeros(np.asarray(deltas_i64[0]).shape, dtype=np.float32)
    for i in range(len(w)):
        t = np.multiply(deltas_f32[i], w[i], dtype=np.float32)
        ti = np.multiply(np.asarray(deltas_i64[i]).astype(np.float32), w[i], dtype=np.float32)
        if s is not None:
            t = np.multiply(t, s[i], dtype=np.float32)
            ti = np.multiply(ti, s[i], dtype=np.float32)
        acc = np.add(acc, t, dtype=np.float32)
        acc_i = np.add(acc_i, ti, dtype=np.float32)
    return acc, acc_i


def w64_numpy(xs_f32, xs_i64, weights64, weights_i64, base_f32=None, base_i64=None):
    """Float64 weights on fp32 entries (rl_server.py:66-71 with a float64 action,
    fedavg_he.py:88-98 on float64 plaintext vectors): the product in float64,
    the in-place add into the fp32 average in float64, then the cast;
    int64 entries keep the fp32 chain with fp32(weights_i64[i])."""
    n_f = xs_f32[0].size if xs_f32 else 0
    acc = np.zeros(n_f, dtype=np.float32)
    for x, w in zip(xs_f32, weights64):
        d = x if base_f32 is None else np.subtract(x, base_f32, dtype=np.float32)
        acc = (acc.astype(np.float64) + d.astype(np.float64) * float(w)).astype(np.float32)
    n_i = xs_i64[0].size if xs_i64 else 0
    acc_i = np.zeros(n_i, dtype=np.float32)
    for x, w in zip(xs_i64, weights_i64):
        with np.errstate(over="ignore"):
            d = x.astype(np.int64) if base_i64 is None else x.astype(np.int64) - base_i64.astype(np.int64)
        acc_i = np.add(acc_i, np.multiply(d.astype(np.float32), np.float32(float(w)), dtype=np.float32),
                       dtype=np.float32)
    if base_f32 is not None:
        acc = np.add(base_f32, acc, dtype=np.float32)
    if base_i64 is not None:
        acc_i = np.add(base_i64.astype(np.float32), acc_i, dtype=np.float32)
    return acc, acc_i


def mix_numpy(base_f32, base_i64, x_f32, x_i64, mixing: float):
    """FedAsync (fedasync_algorithm.py:15-18): b * fp32(1-m) + x * fp32(m)."""
    om = np.float32(1 - mixing)
    m = np.float32(mixing)
    out = np.add(np.multiply(base_f32, om, dtype=np.float32), np.multiply(x_f32, m, dtype=np.float32),
                 dtype=np.float32)
    out_i = np.add(np.multiply(base_i64.astype(np.float32), om, dtype=np.float32),
                   np.multiply(np.asarray(x_i64).astype(np.float32), m, dtype=np.float32),
                   dtype=np.float32)
    return out, out_i


def bf16_roundtrip(values: np.ndarray) -> np.ndarray:
    """model_quantize then model_dequantize (processors/model_quantize.py:15,
    model_dequantize.py:15-18): .to(bfloat16).to(float32), via torch's CPU cast."""
    import torch

    return torch.from_numpy(np.ascontiguousarray(values)).to(torch.bfloat16).to(torch.float32).numpy()


def trunc_to_int64(values_f32: np.ndarray) -> np.ndarray:
    """load_state_dict fp32 -> int64 copy: truncation toward zero (x86: NaN/overflow -> INT64_MIN)."""
    v = np.asarray(values_f32, dtype=np.float32)
    out = np.full(v.shape, np.iinfo(np.int64).min, dtype=np.int64)
    ok = (v >= np.float32(-(2.0**63))) & (v < np.float32(2.0**63))
    out[ok] = np.trunc(v[ok]).astype(np.int64)
    return out


# --------------------------------------------------------------------------
# 2. the reference's torch op sequence (CPU), per tensor
# --------------------------------------------------------------------------
def fedavg_torch_ops(baseline: Mapping, weights_received: Sequence[Mapping], num_samples=None,
                     weights: Sequence[float] | None = None) -> "OrderedDict":
    """compute_weight_deltas -> aggregate_deltas -> update_weights, as torch ops.

    Mirrors plato/algorithms/fedavg.py:13-37 and plato/servers/fedavg.py:137-159
    line by line (without the asyncio yields and the Server object).  Returns
    the updated-weights dict (fp32 for every key, like update_weights).
    """
    import torch

    deltas = []
    for weight in weights_received:
        delta = OrderedDict()
        for name, current in weight.items():
            delta[name] = current - baseline[name]
        deltas.append(delta)
    if weights is None:
        total = sum(num_samples)
        weights = [n / total for n in num_samples]
    avg = {name: torch.zeros(d.shape) for name, d in deltas[0].items()}
    for i, update in enumerate(deltas):
        for name, delta in update.items():
            avg[name] += delta * weights[i]
    updated = OrderedDict()
    for name, weight in baseline.items():
        updated[name] = weight + avg[name]
    return updated


def load_into(model_state: Mapping, updated: Mapping) -> None:
    """load_state_dict's per-key copy_ (fp32 -> int64 truncation included)."""
    for name, dst in model_state.items():
        dst.copy_(updated[name])


# --------------------------------------------------------------------------
# 3. per-entry variants (FedAtt, FedAdp, Polaris)
# --------------------------------------------------------------------------
def _region_deltas(entries, region, base, x):
    """Flat region delta as compute_weight_deltas forms it (int64: wrap, then fp32)."""
    if region == "f32":
        return np.subtract(x, base, dtype=np.float32)
    with np.errstate(over="ignore"):
        return (x.astype(np.int64) - base.astype(np.int64)).astype(np.float32)


def entry_index(entries, region: str, n: int) -> np.ndarray:
    """Element -> entry index (position in ``entries``) for one region; -1 = padding."""
    idx = np.full(n, -1, dtype=np.int64)
    for e_i, e in enumerate(entries):
        if e.region == region:
            idx[e.offset:e.offset + e.numel] = e_i
    return idx


def entry_stats_fp64(entries, bf, bi, xs_f, xs_i, vf=None, vi=None):
    """Per (client, entry) fp64 sums d.v and d.d, per entry v.v (plato_agg_entry_stats).

    The deltas are fp32 as the reference forms them; the sums are exact-ish
    fp64 (np.add.reduceat), a restatement of the device kernel's contract
    rather than of a reference line.
    """
    n_e = len(entries)
    k = len(xs_f)
    dd = np.zeros((k, n_e))
    dv = np.zeros((k, n_e))
    vv = np.zeros(n_e)
    for region, base, xs, v in (("f32", bf, xs_f, vf), ("i64", bi, xs_i, vi)):
        ents = [(e_i, e) for e_i, e in enumerate(entries) if e.region == region and e.numel]
        if not ents:
            continue
        for i in range(k):
            d = _region_deltas(entries, region, base, xs[i]).astype(np.float64)
            for e_i, e in ents:
                seg = d[e.offset:e.offset + e.numel]
                dd[i, e_i] = np.dot(seg, seg)
                if v is not None:
                    dv[i, e_i] = np.dot(seg, np.asarray(v[e.offset:e.offset + e.numel], dtype=np.float64))
        if v is not None:
            for e_i, e in ents:
                seg = np.asarray(v[e.offset:e.offset + e.numel], dtype=np.float64)
                vv[e_i] = np.dot(seg, seg)
    return dv, dd, vv


def entrywise_numpy(entries, bf, bi, xs_f, xs_i, w_ek, scale=1.0, noise_f=None, noise_i=None,
                    noise_scale=0.0, add_base=True):
    """plato_agg_fedavg_entrywise on flat arenas, one rounding per op:

        acc = +0; for i: acc = fp32(acc + fp32(fp32(x_i - b) * W[entry, i]))
        u = fp32(acc * scale) [+ fp32(noise * noise_scale)];  out = fp32(b + u) if add_base

    With W = -softmax(norms), scale = -epsilon, noise_scale = magnitude this is
    examples/server_aggregation/fedatt/fedatt_algorithm.py:44-69 + update_weights.
    """
    w = np.asarray(w_ek, dtype=np.float64).astype(np.float32)
    outs = []
    for region, base, xs, nz in (("f32", bf, xs_f, noise_f), ("i64", bi, xs_i, noise_i)):
        idx = entry_index(entries, region, base.size)
        acc = np.zeros(base.size, dtype=np.float32)
        for i in range(len(xs)):
            d = _region_deltas(entries, region, base, xs[i])
            wi = np.where(idx >= 0, w[np.maximum(idx, 0), i], np.float32(0)).astype(np.float32)
            acc = np.add(acc, np.multiply(d, wi, dtype=np.float32), dtype=np.float32)
        u = np.multiply(acc, np.float32(scale), dtype=np.float32)
        if nz is not None:
            u = np.add(u, np.multiply(nz, np.float32(noise_scale), dtype=np.float32), dtype=np.float32)
        if add_base:
            u = np.add(base.astype(np.float32), u, dtype=np.float32)
        outs.append(u)
    return outs[0], outs[1]


def fedatt_torch(baseline: Mapping, weights_received: Sequence[Mapping], epsilon=1.2, magnitude=0.001):
    """FedAtt's aggregation as torch CPU ops (fedatt_algorithm.py:23-69 + algorithms/fedavg.py:13-37).

    The caller seeds torch's CPU generator; the noise is one ``torch.randn``
    per key in baseline order, drawn after all attention weights.  Returns
    (updated dict, norms [E][K] fp32, atts [E][K] fp32).
    """
    import torch
    import torch.nn.functional as F

    names = list(baseline.keys())
    deltas = [OrderedDict((n, x[n] - baseline[n]) for n in x) for x in weights_received]
    norms = np.zeros((len(names), len(deltas)), dtype=np.float32)
    atts = {}
    for e, name in enumerate(names):
        col = torch.zeros(len(deltas))
        for i, d in enumerate(deltas):
            col[i] = torch.linalg.norm(-(d[name].to(torch.float32)))
        norms[e] = col.numpy()
        atts[name] = F.softmax(col, dim=0)
    updated = OrderedDict()
    for name, weight in baseline.items():
        acc = torch.zeros(weight.shape)
        for i, d in enumerate(deltas):
            acc += torch.mul(-(d[name].float()), atts[name][i])
        step = -torch.mul(acc, epsilon) + torch.mul(torch.randn(weight.shape), magnitude)
        updated[name] = weight + step
    return updated, norms, np.stack([atts[n].numpy() for n in names])


def torch_cpu_norm_f32(rows: np.ndarray) -> np.ndarray:
    """``torch.linalg.norm`` of each row of an fp32 ``[K, n]`` matrix, in x86-64
    PyTorch's CPU order (ATen's vectorised last-dim 2-norm, as measured for
    torch 2.10 here): 8 lanes of fp32 fma(v, v, acc) over the first n - n%8
    elements, lanes summed in order, then the tail: 4 separately rounded
    products added in order if 4+ remain, the last 1-3 fma'd; fp32 sqrt.
    (The fma below is emulated in float64: exact product, one rounding of the
    sum to float64, then to float32 — double rounding can flip a last bit in
    rare ties; oracle/reductions.c has the exact fmaf version.)"""
    rows = np.asarray(rows, dtype=np.float32)
    k, n = rows.shape
    m = n - n % 8
    acc = np.zeros((k, 8), dtype=np.float32)
    blocks = rows[:, :m].reshape(k, -1, 8).astype(np.float64)
    for t in range(blocks.shape[1]):  # fma: exact product + one rounding
        acc = (acc + blocks[:, t] * blocks[:, t]).astype(np.float32)
    s = acc[:, 0].copy()
    for j in range(1, 8):
        s = np.add(s, acc[:, j], dtype=np.float32)
    for e in range(m, n):
        if n - m >= 4 and e < m + 4:  # 4 products of one SSE multiply, added in order
            s = np.add(s, np.multiply(rows[:, e], rows[:, e], dtype=np.float32), dtype=np.float32)
        else:  # the last 1-3: vfmadd231ss
            v = rows[:, e].astype(np.float64)
            s = (s + v * v).astype(np.float32)
    return np.sqrt(s, dtype=np.float32)


def fedadp_flatten(named: Mapping, lr: float) -> np.ndarray:
    """FedAdp's process_grad (fedadp_server.py:122-133): entries sorted by name.lower(),
    the first as is, every other as fp32 ``-x / lr``, concatenated."""
    import torch

    items = sorted(named.items(), key=lambda kv: kv[0].lower())
    parts = [np.asarray(items[0][1]).reshape(-1)]
    for _, t in items[1:]:
        parts.append(np.asarray(-t / lr).reshape(-1))
    return np.concatenate(parts)


def fedadp_angles_numpy(global_grads: Mapping, deltas: Sequence[Mapping], lr: float) -> list:
    """fedadp_server.py:91-99: float32 np.inner / np.linalg.norm / arccos of the flattened vectors."""
    g = fedadp_flatten(global_grads, lr)
    angles = []
    for d in deltas:
        loc = fedadp_flatten(d, lr)
        inner = np.inner(g, loc)
        norms = np.linalg.norm(g) * np.linalg.norm(loc)
        angles.append(np.arccos(np.clip(inner / norms, -1.0, 1.0)))
    return angles


def polaris_norms_numpy(deltas: Sequence[Mapping]) -> list:
    """polaris_server.py:76-89: sqrt of the float32 sum over 'conv' layers of np.sum(np.square(delta))."""
    out = []
    for d in deltas:
        squared = 0
        for layer, value in d.items():
            if "conv" in layer:
                squared += np.sum(np.square(np.asarray(value)))
        out.append(np.sqrt(squared))
    return out
