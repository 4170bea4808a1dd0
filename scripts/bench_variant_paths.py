"""Timing of the variant servers' whole-model reductions on C2-sized inputs (K ResNet-18 clients in HBM).

Each path is what the mixin calls, end to end on the device, host sync included:

* port      AggregationRound.model_similarities: flatten (current - previous, K deltas) ->
            torch-order vector norms (8 serial fma chains over the whole flattened model) ->
            torch-order cascade cosine sums (examples/async/port/port_server.py:24-52)
* fedadp    launch_entrywise (global gradient, device) + fedadp_dots: g flattened in name order,
            the K client deltas gathered from their arenas inside the OpenBLAS-order sdot kernel
            (plato_agg_fedadp_dots; fedadp_server.py:91-99)
* fedadp_flat  the round-2 path: the K deltas flattened into HBM, then plato_agg_sdot_shared
* polaris   np_sumsq: numpy pairwise-order squared deltas per fp32 entry (polaris_server.py:78-81)
* fedatt    entry_norms: torch-order per-entry norms of every client delta (fedatt_algorithm.py:34-39)

One JSON line per path: median wall ms over --reps after one warm-up, the bytes the path
reads/writes at minimum, and the serial-chain length that bounds it (the reference's own
float32 evaluation order).

Usage: python scripts/bench_variant_paths.py [--clients 128] [--reps 5]
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sdot", action="store_true",
                    help="also time the sdot kernels alone on K+1 flat ResNet-18-sized pairs sharing x")
    ap.add_argument("--sdot-only", action="store_true", help="only the sdot kernels (for PMC passes)")
    ap.add_argument("--fedadp-kernel", action="store_true",
                    help="HIP-event time of plato_agg_fedadp_dots alone (+ bitwise check against the flat path)")
    ap.add_argument("--fedadp-only", action="store_true", help="only the fedadp kernel timing (for PMC passes)")
    ap.add_argument("--fedadp-variants", default=None, help="comma-separated fedadp_dots tuning variants to time (default all)")
    ap.add_argument("--port-only", action="store_true", help="only the port path (for kernel traces)")
    ap.add_argument("--fedadp-align", default="fedadp", help="arena alignment of the FedAdp rounds ('' = packed)")
    ap.add_argument("--only", default=None, help="comma-separated paths to time")
    ap.add_argument("--norms-threshold", type=int, default=-1,
                    help="FedAvgEngine.norms_long_threshold for the fedatt path (0 = None; -1 = the default)")
    ap.add_argument("--polaris-variants", action="store_true",
                    help="HIP-event time of every plato_agg_tune_np_sumsq variant (bitwise vs the default)")
    ap.add_argument("--port-gathered", action="store_true",
                    help="HIP-event time of every plato_agg_tune_port_norms variant on the arenas")
    ap.add_argument("--port-norms", action="store_true",
                    help="time the entry_norms variants on Port's K+1 flattened vectors (one entry each)")
    ap.add_argument("--cosine-variants", action="store_true",
                    help="HIP-event time of every plato_agg_tune_torch_cosine_sum_scaled variant, interleaved")
    ap.add_argument("--threads", type=int, default=None, help="torch threads of the cosine chunking (default: this host's)")
    args = ap.parse_args()
    args.sdot = args.sdot or args.sdot_only
    args.fedadp_kernel = args.fedadp_kernel or args.fedadp_only

    from plato_amd import workloads
    from plato_amd.arena import ArenaLayout
    from plato_amd.engine import DeviceArena, FedAvgEngine
    from plato_amd.synthetic import fill_baseline, fill_clients

    dev = torch.device("cuda", 0)
    k = args.clients
    layout = ArenaLayout.from_shapes(workloads.resnet(18, 10))
    engine = FedAvgEngine(dev)
    if args.norms_threshold >= 0:
        engine.norms_long_threshold = args.norms_threshold or None
    base = DeviceArena(layout, dev)
    fill_baseline(base, 0)
    n_f, n_i = layout.n_f32, layout.n_i64
    baseline = layout.unpack(base.f32[:n_f].cpu(), base.i64[:n_i].cpu())
    prev = DeviceArena(layout, dev)
    fill_baseline(prev, 1)
    previous = layout.unpack(prev.f32[:n_f].cpu(), prev.i64[:n_i].cpu())
    del prev
    def make_round(eng):
        r = eng.begin(baseline, k)
        r.put_baseline(baseline)
        torch.cuda.synchronize(dev)  # the baseline's H2D (copy stream) before the fill reads it
        fill_clients(r.slab, r.engine._base, 0, k)  # the round's own slab, filled on the device
        for s in range(k):
            pf, pi = r.slab.row_pointers([s])
            r._pf[s], r._pi[s] = int(pf[0]), int(pi[0])
            r.staged[s] = True
        torch.cuda.synchronize(dev)
        return r

    rnd = make_round(engine)
    # FedAdp's rounds run on arenas aligned to the flattened positions (FedAdpServerMixin.arena_alignment)
    adp_engine = FedAvgEngine(dev)
    adp_engine.layout_align = args.fedadp_align or None
    rnd_adp = make_round(adp_engine) if (args.fedadp_kernel or not args.only or "fedadp" in args.only) else rnd
    slots = list(range(k))
    n_e = len(layout.entries)
    longest = max(e.numel for e in layout.entries)
    client_bytes = k * (n_f * 4 + n_i * 8)

    def fedadp():
        w = np.full((n_e, k), 1.0 / k)
        grads = rnd_adp.launch_entrywise(w, add_base=False, device=True)
        rnd_adp.fedadp_dots(grads, slots, 0.01)

    def fedadp_flat():
        w = np.full((n_e, k), 1.0 / k)
        grads = rnd_adp.launch_entrywise(w, add_base=False, device=True)
        rnd_adp.fedadp_dots_flat(grads, slots, 0.01)

    prev_arena = rnd.stage_reference(previous)
    paths = {
        "port": (lambda: rnd.model_similarities(previous, slots),
                 client_bytes + 3 * n_f * 4, (n_f + n_i) // 8,
                 "stage the reference model (H2D) + norms gathered from the arenas (8 fma chains over the flattened "
                 "model; the kernel stores the flat vectors) + cascade cosine sums"),
        "port_staged": (lambda: rnd.model_similarities(prev_arena, slots),
                        client_bytes + 3 * n_f * 4, (n_f + n_i) // 8,
                        "the same with the reference model staged ahead (AggregationRound.stage_reference)"),
        "port_flat": (lambda: rnd.model_similarities(prev_arena, slots, flat_norms=True),
                      client_bytes + 3 * n_f * 4, (n_f + n_i) // 8,
                      "round 2: flatten + vector_norm over the flat rows + cascade cosine sums (reference staged)"),
        "fedadp": (fedadp, 2 * client_bytes, (n_f + n_i) // 64,
                   "global gradient + g flatten + fused gather/sdot (64 fma chains over the flattened model)"),
        "fedadp_flat": (fedadp_flat, 2 * client_bytes, (n_f + n_i) // 64,
                        "global gradient + flatten of g and the K deltas + sdot_shared (round 2)"),
        "polaris": (lambda: rnd.np_sumsq(slots), client_bytes, 0,
                    "numpy pairwise sums per entry (8-way unrolled blocks of 128)"),
        "fedatt": (lambda: rnd.entry_norms(slots), client_bytes, longest // 8,
                   "per-entry torch norms: 8 fma chains per (entry, client)"),
    }
    for name, (fn, nbytes, chain, what) in paths.items():
        if (args.sdot_only or args.fedadp_only or args.port_gathered
                or args.polaris_variants or args.cosine_variants):
            break
        if args.port_only and not name.startswith("port"):
            continue
        if args.only and name not in args.only.split(","):
            continue
        fn()
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        med = statistics.median(ts) * 1e3
        print(json.dumps({"path": name, "clients": k, "norms_long_threshold": engine.norms_long_threshold,
                          "ms_median": round(med, 3), "ms_min": round(min(ts) * 1e3, 3),
                          "min_bytes": int(nbytes), "GBps_of_min_bytes": round(nbytes / (med * 1e-3) / 1e9, 1),
                          "serial_chain_steps": int(chain), "what": what}), flush=True)
    if args.fedadp_kernel:
        fedadp_kernel(dev, rnd_adp, slots, rnd_adp.layout, args.reps,
                      None if not args.fedadp_variants else {int(v) for v in args.fedadp_variants.split(",")})
    if args.sdot:
        sdot_kernels(dev, k, n_f + n_i, args.reps)
    if args.port_norms:
        port_norms(dev, k, n_f + n_i, args.reps)
    if args.port_gathered:
        port_gathered(dev, rnd, slots, layout, previous, args.reps)
    if args.polaris_variants:
        polaris_variants(dev, rnd, slots, layout, args.reps)
    if args.cosine_variants:
        cosine_variants(dev, k, n_f + n_i, args.reps, args.threads or torch.get_num_threads())


def fedadp_kernel(dev, rnd, slots, layout, reps, only=None):
    """plato_agg_fedadp_dots alone (HIP events on the launch stream), against the flatten + sdot_shared path."""
    from plato_amd import _lib

    k, n_e = len(slots), len(layout.entries)
    grads = rnd.launch_entrywise(np.full((n_e, k), 1.0 / k), add_base=False, device=True)
    want = rnd.fedadp_dots_flat(grads, slots, 0.01)
    got = rnd.fedadp_dots(grads, slots, 0.01)
    same = all(np.asarray(a).tobytes() == np.asarray(b).tobytes() for a, b in zip(got, want))
    g_flat, ptrs, ws = rnd._keep_flat
    eng = rnd.engine
    order = rnd._fedadp_order()
    segs, n_flat = rnd._flat_segments(order, True)
    xy = torch.empty(k + 1, device=dev)
    yy = torch.empty(k + 1, device=dev)
    h = torch.cuda.current_stream(dev).cuda_stream

    # delta arenas for the delta variants (null baseline): every slot's x - b in a second slab
    from plato_amd.engine import ClientSlab

    dslab = ClientSlab(layout, k, dev)
    for i, j in enumerate(slots):
        _lib.call("plato_agg_compute_deltas", rnd._pf[j], rnd._pi[j], eng._base.f32.data_ptr(),
                  eng._base.i64.data_ptr(), dslab.f32[i].data_ptr(), dslab.i64[i].data_ptr(), layout.n_f32,
                  layout.n_i64, h)
    dpf, dpi = dslab.row_pointers(range(k))
    dptrs = torch.from_numpy(np.concatenate([dpf, dpi]).astype(np.int64)).to(dev)

    def call(name, v, delta):
        p = dptrs if delta else ptrs
        base_f = None if delta else eng._base.f32.data_ptr()
        base_i = None if delta else eng._base.i64.data_ptr()
        args = (g_flat.data_ptr(), p.data_ptr(), p.data_ptr() + 8 * k, k, base_f, base_i, segs.data_ptr(),
                len(order), n_flat, layout.n_f32, layout.n_i64, 0.01, 1, ws.data_ptr(), xy.data_ptr(), yy.data_ptr(), h)
        if v is None:
            _lib.call(name, *args)
        else:
            _lib.tune_call(name, v, *args)

    runs = {"default": lambda: call("plato_agg_fedadp_dots", None, False),
            "default_delta": lambda: call("plato_agg_fedadp_dots", None, True)}
    for v in range(_lib.tune().plato_agg_tune_num_fedadp_variants()):
        if only is not None and v not in only:
            continue
        delta = bool(_lib.tune().plato_agg_tune_fedadp_is_delta(v))
        runs[f"v{v}{'_delta' if delta else ''}"] = (lambda v=v, d=delta: call("plato_agg_tune_fedadp_dots", v, d))
    # unique bytes: each client's fp32 arena + int64 counters once, the baseline and g_flat once
    uniq = k * (layout.n_f32 * 4 + layout.n_i64 * 8) + 2 * layout.n_f32 * 4 + n_flat * 4
    oks = {}
    for name, fn in runs.items():
        fn()
        torch.cuda.synchronize(dev)
        oks[name] = (xy.cpu().numpy()[:k].tobytes() == np.asarray(want[0]).tobytes()
                     and xy.cpu().numpy()[k:].tobytes() == np.float32(want[1]).tobytes()
                     and yy.cpu().numpy()[:k].tobytes() == np.asarray(want[2]).tobytes())
    tss = {name: [] for name in runs}
    for _ in range(reps):  # interleaved: box drift hits every variant alike
        for name, fn in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            tss[name].append(e0.elapsed_time(e1))
    for name in runs:
        ok, ts = oks[name], tss[name]
        med = statistics.median(ts)
        print(json.dumps({"fedadp_dots": name, "pairs": k + 1, "n_flat": n_flat, "ms_median": round(med, 4),
                          "ms_min": round(min(ts), 4), "GBps_unique_bytes": round(uniq / (med * 1e-3) / 1e9, 1),
                          "unique_bytes": uniq, "bitwise_equal_to_flat_path": ok and same}), flush=True)


def polaris_variants(dev, rnd, slots, layout, reps):
    """plato_agg_np_sumsq kernels: one client per workgroup vs G clients sharing the baseline."""
    from plato_amd import _lib

    k = len(slots)
    want = rnd.np_sumsq(slots)
    pieces, first, entry_of, n_chunks = rnd.layout._cache[("np_sumsq_pieces", str(dev))]
    tf = torch.from_numpy(np.asarray([rnd._pf[i] for i in slots], dtype=np.int64)).to(dev)
    ws = torch.empty(max(1, rnd.engine.lib.plato_agg_np_sumsq_workspace(k, n_chunks) // 4), device=dev)
    out = torch.empty((k, int(entry_of.size)), device=dev)
    h = torch.cuda.current_stream(dev).cuda_stream
    uniq = k * layout.n_f32 * 4 + layout.n_f32 * 4
    fns, ok, ts = {}, {}, {}
    for v in range(_lib.tune().plato_agg_tune_num_np_sumsq_variants()):
        def fn(v=v):
            _lib.tune_call("plato_agg_tune_np_sumsq", v, tf.data_ptr(), k, rnd._base.f32.data_ptr(), pieces.data_ptr(),
                           first.data_ptr(), int(entry_of.size), n_chunks, ws.data_ptr(), out.data_ptr(), h)
        fn()
        torch.cuda.synchronize(dev)
        fns[v], ok[v], ts[v] = fn, out.cpu().numpy().tobytes() == want[:, entry_of].tobytes(), []
    for _ in range(3):  # interleaved rounds: box drift hits every variant alike
        for v, fn in fns.items():
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                e1.synchronize()
                ts[v].append(e0.elapsed_time(e1))
    for v in fns:
        med = statistics.median(ts[v])
        print(json.dumps({"np_sumsq_variant": v, "clients": k, "ms_median": round(med, 4), "ms_min": round(min(ts[v]), 4),
                          "GBps_unique_bytes": round(uniq / (med * 1e-3) / 1e9, 1),
                          "bitwise_equal_to_default": ok[v]}), flush=True)


def port_gathered(dev, rnd, slots, layout, previous, reps):
    """plato_agg_port_norms (norms from the arenas) per tuning variant vs the flatten + entry_norms norms."""
    from plato_amd import _lib
    from plato_amd.engine import _ptr

    k = len(slots)
    rnd.model_similarities(previous, slots, flat_norms=True)
    want = rnd.last_norms.copy()
    prev = rnd._stage_model(previous, "reference model", torch.cuda.current_stream(dev))
    segs, n_flat = rnd._flat_segments(list(range(len(layout.entries))), False)
    bf, bi = _ptr(rnd._base.f32), _ptr(rnd._base.i64)
    vec = np.asarray([bf] + [rnd._pf[i] for i in slots] + [bi] + [rnd._pi[i] for i in slots]
                     + [_ptr(prev.f32)] + [bf] * k + [_ptr(prev.i64)] + [bi] * k, dtype=np.int64)
    stride = max(64, -(-n_flat // 64) * 64)
    flat = torch.empty((k + 1, stride), device=dev)
    vec = np.concatenate([vec, np.asarray([flat.data_ptr() + r * stride * 4 for r in range(k + 1)], dtype=np.int64)])
    vt = torch.from_numpy(vec).to(dev)
    v8 = vt.data_ptr()
    out = torch.empty(k + 1, device=dev)
    h = torch.cuda.current_stream(dev).cuda_stream
    def make(v, store):
        def fn():
            _lib.tune_call("plato_agg_tune_port_norms", v, v8, v8 + 8 * (k + 1), v8 + 16 * (k + 1), v8 + 24 * (k + 1),
                           k + 1, None, segs.data_ptr(), len(layout.entries), n_flat, layout.n_f32,
                           _lib.PLATO_AGG_PORT_CAST_FIRST, out.data_ptr(), v8 + 32 * (k + 1) if store else None, h)
        return fn
    # the stores-flat form (the product's) of every variant, interleaved rep by rep
    runs = {(v, True): make(v, True) for v in range(_lib.tune().plato_agg_tune_num_port_norms_variants())}
    oks = {}
    for key, fn in runs.items():
        fn()
        torch.cuda.synchronize(dev)
        oks[key] = out.cpu().numpy().tobytes() == want.tobytes()
    tss = {key: [] for key in runs}
    for _ in range(reps):
        for key, fn in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            tss[key].append(e0.elapsed_time(e1))
    for (v, store), ts in tss.items():
        ok = oks[(v, store)]
        med = statistics.median(ts)
        print(json.dumps({"port_norms_gathered_variant": v, "stores_flat": store, "vectors": k + 1, "n": n_flat,
                          "ms_median": round(med, 4),
                          "cycles_per_step_at_2.4GHz": round(med * 1e-3 * 2.4e9 / (n_flat // 8), 2),
                          "bitwise_equal_to_flat_path": ok}), flush=True)


def cosine_variants(dev, k, n, reps, threads):
    """Port's cascade cosine sums (a already divided by its norm) per tuning variant, interleaved
    rep by rep so that box drift hits every variant alike, bitwise compared."""
    from plato_amd import _lib

    stride = -(-n // 64) * 64
    a = torch.randn(stride, device=dev)
    bs = torch.randn((k, stride), device=dev) * 1e-2
    tab = torch.tensor([bs.data_ptr() + r * stride * 4 for r in range(k)], dtype=torch.int64, device=dev)
    nb = torch.linalg.vector_norm(bs, dim=1)
    ws = torch.empty(max(1, _lib.lib().plato_agg_torch_cosine_workspace(k, threads) // 4), device=dev)
    h = torch.cuda.current_stream(dev).cuda_stream
    nv = _lib.tune().plato_agg_tune_num_cosine_variants()
    outs = [torch.empty(k, device=dev) for _ in range(nv)]

    def fn(v):
        _lib.tune_call("plato_agg_tune_torch_cosine_sum_scaled", v, a.data_ptr(), tab.data_ptr(), k, n, nb.data_ptr(),
                       1e-8, threads, ws.data_ptr(), outs[v].data_ptr(), h)
    for v in range(nv):
        fn(v)
    torch.cuda.synchronize(dev)
    ref = outs[0].cpu().numpy().tobytes()
    same = [o.cpu().numpy().tobytes() == ref for o in outs]
    ts = [[] for _ in range(nv)]
    for _ in range(reps):
        for v in range(nv):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn(v)
            e1.record()
            e1.synchronize()
            ts[v].append(e0.elapsed_time(e1))
    uniq = (k + 1) * n * 4
    for v in range(nv):
        med = statistics.median(ts[v])
        print(json.dumps({"cosine_variant": v, "clients": k, "n": n, "threads": threads, "ms_median": round(med, 4),
                          "ms_min": round(min(ts[v]), 4), "GBps_unique_bytes": round(uniq / (med * 1e-3) / 1e9, 1),
                          "bitwise_equal_to_v0": same[v]}), flush=True)


def port_norms(dev, k, n, reps):
    """The vector norms of Port's similarity (8 torch-order fma chains over each whole flattened
    vector) through every producer/consumer entry_norms variant, bitwise compared."""
    from plato_amd import _lib

    stride = -(-n // 64) * 64
    rows = torch.randn((k + 1, stride), device=dev) * 1e-2
    tab = torch.tensor([rows.data_ptr() + r * stride * 4 for r in range(k + 1)], dtype=torch.int64, device=dev)
    chunk = torch.from_numpy(np.asarray([[0, 0, stride, 0]], dtype=np.uint32).view(np.int32)).to(dev)
    h = torch.cuda.current_stream(dev).cuda_stream
    ref = None
    for v in range(_lib.tune().plato_agg_tune_num_entry_norms_variants()):
        out = torch.empty(k + 1, device=dev)

        def fn():
            _lib.tune_call("plato_agg_tune_entry_norms", v, tab.data_ptr(), None, k + 1, None, None, chunk.data_ptr(), 1,
                      None, 0, 1, stride, 0, out.data_ptr(), h)
        fn()
        torch.cuda.synchronize(dev)
        got = out.cpu().numpy().tobytes()
        ref = ref or got
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        med = statistics.median(ts)
        print(json.dumps({"port_norms_variant": v, "vectors": k + 1, "n": stride, "ms_median": round(med, 4),
                          "cycles_per_step_at_2.4GHz": round(med * 1e-3 * 2.4e9 / (stride // 8), 2),
                          "bitwise_equal_to_v0": got == ref}), flush=True)


def sdot_kernels(dev, k, n, reps):
    """plato_agg_sdot_pairs (one workgroup per pair) vs every plato_agg_sdot_shared variant, bitwise compared."""
    from plato_amd import _lib

    stride = -(-n // 64) * 64
    x = torch.randn(stride, device=dev)
    ys = torch.randn((k + 1, stride), device=dev) * 1e-2
    ys[k] = x  # the per-pair kernel gets g.g as a pair (x, x) after the clients
    py = torch.tensor([ys.data_ptr() + r * stride * 4 for r in range(k + 1)], dtype=torch.int64, device=dev)
    px = torch.full((k + 1,), x.data_ptr(), dtype=torch.int64, device=dev)
    ws = torch.empty(_lib.lib().plato_agg_sdot_shared_workspace(k, 1) // 4, device=dev)
    h = torch.cuda.current_stream(dev).cuda_stream
    runs = {"pairs": lambda o1, o2: _lib.call("plato_agg_sdot_pairs", px.data_ptr(), py.data_ptr(), k + 1, n,
                                              o1.data_ptr(), o2.data_ptr(), h),
            "shared_default": lambda o1, o2: _lib.call("plato_agg_sdot_shared", x.data_ptr(), py.data_ptr(), k, n, 1,
                                                       ws.data_ptr(), o1.data_ptr(), o2.data_ptr(), h)}
    for v in range(_lib.tune().plato_agg_tune_num_sdot_shared_variants()):
        runs[f"shared_v{v}"] = (lambda o1, o2, v=v: _lib.tune_call("plato_agg_tune_sdot_shared", v, x.data_ptr(),
                                                               py.data_ptr(), k, n, 1, ws.data_ptr(), o1.data_ptr(),
                                                               o2.data_ptr(), h))
    ref = None
    for name, fn in runs.items():
        o1 = torch.empty(k + 1, device=dev)
        o2 = torch.empty(k + 1, device=dev)
        fn(o1, o2)
        torch.cuda.synchronize(dev)
        got = (o1.cpu().numpy().tobytes(), o2.cpu().numpy().tobytes())
        ref = ref or got
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn(o1, o2)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        med = statistics.median(ts)
        uniq = (k + 1) * n * 4 + n * 4  # every y once + x once
        print(json.dumps({"sdot": name, "pairs": k + 1, "n": n, "ms_median": round(med, 4),
                          "ms_min": round(min(ts), 4), "GBps_unique_bytes": round(uniq / (med * 1e-3) / 1e9, 1),
                          "bitwise_equal_to_pairs": got == ref}), flush=True)


if __name__ == "__main__":
    main()
