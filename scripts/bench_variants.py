"""Timing of the variant kernels on C2-sized inputs (K ResNet-18 client updates in HBM).

One JSON line per kernel: median ms over R repetitions (HIP events on the
launch stream), algorithmic bytes, GB/s and fraction of the 8 TB/s peak.

* qsgd        plato_agg_fedavg_qsgd: K x 1 B codes + fp32 baseline read + result write
* entrywise   plato_agg_fedavg_entrywise (FedAtt's sum, noise + baseline): K x 4 B + 3 x 4 B
* stats       plato_agg_entry_stats with v (FedAdp): K x 4 B + 2 x 4 B
* norms       plato_agg_entry_norms_f32 (FedAtt, torch CPU order): K x 4 B + 4 B; a serial
              fma chain per (client, entry, lane) — latency-bound by the largest entry
* fedavg      the FedAvg kernel itself, for reference

Usage: python scripts/bench_variants.py [--clients 128] [--reps 10]
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default=None)
    ap.add_argument("--qsgd-codes", default="qsgd", choices=["qsgd", "uniform"])
    ap.add_argument("--norm-variants", action="store_true", help="also time each entry_norms kernel variant")
    ap.add_argument("--norm-list", default=None, help="comma-separated entry_norms variants to time (instead of all)")
    ap.add_argument("--qsgd-variants", action="store_true", help="also time each fedavg_qsgd kernel variant")
    ap.add_argument("--qsgd-list", default=None, help="comma-separated fedavg_qsgd variants to time (instead of all)")
    ap.add_argument("--interleave", type=int, default=0,
                    help="time the selected kernels round-robin this many rounds (A/B on one box: clock and "
                         "thermal drift hit every kernel alike); each round times each kernel --reps times")
    ap.add_argument("--ew-chunks", default=None,
                    help="comma-separated fedavg_entrywise chunk sizes to time besides the engine's (tuning)")
    ap.add_argument("--ew-shapes", default=None,
                    help="comma-separated chunk:threads pairs of fedavg_entrywise to time through the tuning "
                         "library (plato_agg_tune_set_entrywise_block), e.g. 2048:256,512:64")
    ap.add_argument("--sumsq-list", default=None, help="comma-separated np_sumsq variants to time")
    ap.add_argument("--deltas", action="store_true",
                    help="client arenas hold x - b (delta arenas): entry norms run with a null baseline")
    ap.add_argument("--norm-order", default="longest", choices=["longest", "layout"],
                    help="entry order of the norms launch (longest first = the engine's)")
    args = ap.parse_args()

    from plato_amd import _lib, workloads
    from plato_amd.arena import ArenaLayout
    from plato_amd.engine import ClientSlab, DeviceArena, FedAvgEngine, _ptr
    from plato_amd.synthetic import fill_baseline, fill_clients

    dev = torch.device("cuda", 0)
    k = args.clients
    layout = ArenaLayout.from_shapes(workloads.resnet(18, 10))
    engine = FedAvgEngine(dev)
    base = DeviceArena(layout, dev)
    slab = ClientSlab(layout, k, dev)
    fill_baseline(base, 0)
    fill_clients(slab, base, 0, k)
    stream = torch.cuda.current_stream(dev)
    h = stream.cuda_stream
    if args.deltas:  # every client row turned into its delta in place (FedAvgEngine.delta_arenas)
        for r in range(k):
            _lib.call("plato_agg_compute_deltas", _ptr(slab.f32[r]), _ptr(slab.i64[r]), _ptr(base.f32),
                      _ptr(base.i64), _ptr(slab.f32[r]), _ptr(slab.i64[r]), layout.n_f32, layout.n_i64, h)
        torch.cuda.synchronize(dev)
    nb_f = None if args.deltas else base.f32
    nb_i = None if args.deltas else base.i64
    pf, pi = slab.row_pointers(range(k))
    tf = torch.from_numpy(pf).to(dev)
    ti = torch.from_numpy(pi).to(dev)
    n_f, n_i, n_e = layout.n_f32, layout.n_i64, len(layout.entries)
    out_f = torch.empty(layout.row_f32, device=dev)
    out_i = torch.empty(layout.row_i64, device=dev)
    w = torch.full((k,), 1.0 / k, device=dev)
    w_ek = torch.full((n_e, k), -1.0 / k, device=dev)
    noise = torch.randn(layout.row_f32, device=dev)
    noise_i = torch.randn(layout.row_i64, device=dev)

    def chunks(cap):
        return engine._chunks(layout, cap)

    # QSGD codes, one max_v per (entry, client).  "qsgd": what the client quantizer
    # (model_quantize_qsgd.py) makes of normally distributed deltas at level 64,
    # |zeta| = floor(|x| / max_v * 63 + U[0,1)) with max_v ~ 5 sigma, random sign;
    # "uniform": every byte equally likely (worst case for the LDS decode tables).
    qslab = ClientSlab(layout, k, dev, codec="qsgd")

    def codes(shape, r):
        if args.qsgd_codes == "uniform":
            return torch.randint(0, 256, shape, dtype=torch.uint8, device=dev)
        g = torch.Generator(device=dev).manual_seed(1 + r)  # every client its own codes
        mag = torch.floor(torch.randn(shape, device=dev, generator=g).abs() * (63 / 5)
                          + torch.rand(shape, device=dev, generator=g)).clamp_(0, 127)
        sign = (torch.rand(shape, device=dev, generator=g) < 0.5).to(torch.float32) * 128
        return (mag + sign).to(torch.uint8)

    for r in range(k):
        qslab.f32[r].copy_(codes(qslab.f32[r].shape, r))
    qslab.i64.copy_(codes(qslab.i64.shape, k))
    qpf, qpi = qslab.row_pointers(range(k))
    qtf = torch.from_numpy(qpf).to(dev)
    qti = torch.from_numpy(qpi).to(dev)
    max_v = torch.rand((n_e, k), device=dev) * 0.1 + 0.01
    ws_stats = torch.empty((engine.lib.plato_agg_entry_stats_workspace(k, int(sum(t.shape[0] for t in chunks(4096))))
                            + 7) // 8, dtype=torch.float64, device=dev)
    stats_out = torch.empty((2 * k + 1) * n_e, dtype=torch.float64, device=dev)
    norms_out = torch.empty(k * n_e, dtype=torch.float32, device=dev)

    def run_qsgd(variant=None):
        if variant is None:
            cf, ci = chunks(engine.QSGD_CHUNK)
            _lib.call("plato_agg_fedavg_qsgd", _ptr(qtf), _ptr(qti), k, _ptr(max_v), n_e, 63.0, _ptr(w), None,
                      _ptr(cf), cf.shape[0], _ptr(ci), ci.shape[0], _ptr(base.f32), _ptr(base.i64), _ptr(out_f),
                      _ptr(out_i), n_f, n_i, h)
            return
        cf, ci = chunks(_lib.tune().plato_agg_tune_qsgd_chunk(variant))
        _lib.tune_call("plato_agg_tune_fedavg_qsgd", variant, _ptr(qtf), _ptr(qti), k, _ptr(max_v), n_e, 63.0, _ptr(w),
                  None, _ptr(cf), cf.shape[0], _ptr(ci), ci.shape[0], _ptr(base.f32), _ptr(base.i64), _ptr(out_f),
                  _ptr(out_i), n_f, n_i, h)

    def run_entrywise(cap=None, threads=None):
        cf, ci = chunks(cap or engine.ENTRYWISE_CHUNK)
        if threads is not None:  # the tuning library's copy of the entry point, at this workgroup size
            _lib.tune().plato_agg_tune_set_entrywise_block(threads)
            _lib.tune_call("plato_agg_fedavg_entrywise", _ptr(tf), _ptr(ti), k, _ptr(w_ek), n_e, _ptr(cf),
                           cf.shape[0], _ptr(ci), ci.shape[0], _ptr(base.f32), _ptr(base.i64), _ptr(noise),
                           _ptr(noise_i), -1.2, 0.001, _lib.PLATO_AGG_ADD_BASE, _ptr(out_f), _ptr(out_i), n_f, n_i, h)
            return
        _lib.call("plato_agg_fedavg_entrywise", _ptr(tf), _ptr(ti), k, _ptr(w_ek), n_e, _ptr(cf), cf.shape[0],
                  _ptr(ci), ci.shape[0], _ptr(base.f32), _ptr(base.i64), _ptr(noise), _ptr(noise_i), -1.2, 0.001,
                  _lib.PLATO_AGG_ADD_BASE, _ptr(out_f), _ptr(out_i), n_f, n_i, h)

    def run_stats():
        cf, ci = chunks(engine.STATS_CHUNK)
        _lib.call("plato_agg_entry_stats", _ptr(tf), _ptr(ti), k, _ptr(base.f32), _ptr(base.i64), _ptr(out_f),
                  _ptr(out_i), _ptr(cf), cf.shape[0], _ptr(ci), ci.shape[0], n_e, n_f, n_i, _ptr(ws_stats),
                  _ptr(stats_out), h)

    def run_norms(variant=None):
        ef, ei = engine._norm_tables(layout) if args.norm_order == "longest" else chunks(1 << 32)
        if variant is None:
            _lib.call("plato_agg_entry_norms_f32", _ptr(tf), _ptr(ti), k, _ptr(nb_f), _ptr(nb_i), _ptr(ef),
                      ef.shape[0], _ptr(ei), ei.shape[0], n_e, n_f, n_i, _ptr(norms_out), h)
        else:
            _lib.tune_call("plato_agg_tune_entry_norms", variant, _ptr(tf), _ptr(ti), k, _ptr(nb_f), _ptr(nb_i),
                      _ptr(ef), ef.shape[0], _ptr(ei), ei.shape[0], n_e, n_f, n_i, _ptr(norms_out), h)

    def run_fedavg():
        engine.launch_fedavg(layout, tf, ti, w, None, k, base.f32, base.i64, out_f, out_i, stream)

    # Polaris: numpy-order sums of squares per fp32 entry (plato_agg_np_sumsq, the product kernels)
    sq_rows, sq_first, sq_chunks = [], [], 0
    for idx, e in enumerate(layout.entries):
        if e.region == "f32" and e.numel:
            sq_rows.append((idx, e.offset, e.offset + e.numel, 0))
            sq_first.append(sq_chunks)
            sq_chunks += -(-e.numel // 8192)
    sq_pieces = torch.from_numpy(np.asarray(sq_rows, dtype=np.uint32).view(np.int32).copy()).to(dev)
    sq_firsts = torch.from_numpy(np.asarray(sq_first, dtype=np.uint32).view(np.int32)).to(dev)
    sq_ws = torch.empty(max(1, engine.lib.plato_agg_np_sumsq_workspace(k, sq_chunks) // 4), device=dev)
    sq_out = torch.empty((k, len(sq_rows)), device=dev)

    def run_sumsq(variant=None):
        if variant is None:
            _lib.call("plato_agg_np_sumsq", _ptr(tf), k, _ptr(nb_f), _ptr(sq_pieces), _ptr(sq_firsts), len(sq_rows),
                      sq_chunks, _ptr(sq_ws), _ptr(sq_out), h)
        else:
            _lib.tune_call("plato_agg_tune_np_sumsq", variant, _ptr(tf), k, _ptr(nb_f), _ptr(sq_pieces), _ptr(sq_firsts),
                           len(sq_rows), sq_chunks, _ptr(sq_ws), _ptr(sq_out), h)

    kernels = {
        "qsgd": (run_qsgd, k * (n_f + n_i) + n_f * 8 + n_i * 12),
        "entrywise": (run_entrywise, (k + 3) * n_f * 4 + (k + 2) * n_i * 8),
        "stats": (run_stats, (k + 2) * n_f * 4 + (k + 1) * n_i * 8),
        "norms": (run_norms, (k + 1) * n_f * 4 + (k + 1) * n_i * 8),
        "fedavg": (run_fedavg, layout.algorithmic_bytes(k)),
        "sumsq": (run_sumsq, (k + 1) * n_f * 4),
    }
    if args.qsgd_variants or args.qsgd_list:  # tuning: every (or the listed) plato_agg_tune_fedavg_qsgd variant
        vlist = ([int(x) for x in args.qsgd_list.split(",")] if args.qsgd_list
                 else range(_lib.tune().plato_agg_tune_num_qsgd_variants()))
        for v in vlist:
            kernels[f"qsgd_v{v}"] = ((lambda v=v: run_qsgd(v)), kernels["qsgd"][1])
    if args.ew_chunks:  # tuning: fedavg_entrywise at other chunk sizes
        for cap in [int(x) for x in args.ew_chunks.split(",")]:
            kernels[f"entrywise_v{cap}"] = ((lambda cap=cap: run_entrywise(cap)), kernels["entrywise"][1])
    if args.ew_shapes:  # tuning: fedavg_entrywise at other (chunk, workgroup size) pairs
        for pair in args.ew_shapes.split(","):
            cap, thr = (int(x) for x in pair.split(":"))
            kernels[f"entrywise_v{cap}x{thr}"] = ((lambda cap=cap, thr=thr: run_entrywise(cap, thr)),
                                                  kernels["entrywise"][1])
    if args.sumsq_list:  # tuning: the listed plato_agg_tune_np_sumsq variants
        for v in [int(x) for x in args.sumsq_list.split(",")]:
            kernels[f"sumsq_v{v}"] = ((lambda v=v: run_sumsq(v)), kernels["sumsq"][1])
    if args.norm_variants or args.norm_list:  # tuning: every (or the listed) plato_agg_tune_entry_norms variant
        for v in ([int(x) for x in args.norm_list.split(",")] if args.norm_list
                  else range(_lib.tune().plato_agg_tune_num_entry_norms_variants())):
            kernels[f"norms_v{v}"] = ((lambda v=v: run_norms(v)), kernels["norms"][1])
    selected = [(name, fn, nbytes) for name, (fn, nbytes) in kernels.items()
                if not args.only or name.split("_v")[0] in args.only.split(",")]

    def timed(fn):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1)

    times = {name: [] for name, _, _ in selected}
    for name, fn, _ in selected:  # warm every kernel first
        fn()
    torch.cuda.synchronize(dev)
    for _ in range(max(1, args.interleave)):
        for name, fn, _ in selected:
            times[name].extend(timed(fn) for _ in range(args.reps))
    for name, _, nbytes in selected:
        med = statistics.median(times[name])
        gbs = nbytes / (med * 1e-3) / 1e9
        print(json.dumps({"kernel": name, "clients": k, "ms_median": round(med, 4), "ms_min": round(min(times[name]), 4),
                          "algorithmic_bytes": int(nbytes), "GBps": round(gbs, 1),
                          "frac_of_8TBps": round(gbs / PEAK, 4), "samples": len(times[name])}), flush=True)


if __name__ == "__main__":
    main()
