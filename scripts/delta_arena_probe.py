#!/usr/bin/env python3
"""Delta arenas: what the variant reductions gain when each client's arena holds x - b.

Every FedAdp / FedAtt (entry norms) workgroup streams the baseline again beside its client
(L2-served re-reads that take a CU's read slots).  If the arenas hold deltas —
compute_weight_deltas (plato/algorithms/fedavg.py:13-27) done once per client when its payload is
staged — the kernels read no baseline.  This times, interleaved in one process on K ResNet-18 clients:
  * plato_agg_fedadp_dots on weight arenas (the default) and on delta arenas (null baseline),
    asserting the outputs are bitwise equal;
  * plato_agg_entry_norms_f32 with the baseline and on delta arenas (null baseline), bitwise;
  * plato_agg_compute_deltas in place, per client (the staging-time cost).
Usage: python scripts/delta_arena_probe.py [--clients 128] [--reps 10] [--rounds 3]
"""

import argparse
import json
import statistics
import sys
import os

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--adp-variants", default="0,9",
                    help="plato_agg_tune_fedadp_dots variants: weight-arena ones get the baseline, delta ones none")
    args = ap.parse_args()

    from plato_amd import _lib, workloads
    from plato_amd.arena import ArenaLayout
    from plato_amd.engine import ClientSlab, DeviceArena, FedAvgEngine, _ptr
    from plato_amd.synthetic import fill_baseline, fill_clients

    dev = torch.device("cuda", 0)
    k = args.clients
    spec = workloads.resnet(18, 10)
    lay = ArenaLayout.from_shapes(spec, align="fedadp")
    base = DeviceArena(lay, dev)
    slab = ClientSlab(lay, k, dev)
    fill_baseline(base, 0)
    fill_clients(slab, base, 0, k)
    dslab = ClientSlab(lay, k, dev)
    stream = torch.cuda.current_stream(dev)
    h = stream.cuda_stream
    n_f, n_i = lay.n_f32, lay.n_i64
    for r in range(k):
        _lib.call("plato_agg_compute_deltas", _ptr(slab.f32[r]), _ptr(slab.i64[r]), _ptr(base.f32), _ptr(base.i64),
                  _ptr(dslab.f32[r]), _ptr(dslab.i64[r]), n_f, n_i, h)
    torch.cuda.synchronize(dev)

    eng = FedAvgEngine(dev)
    eng.layout_align = "fedadp"
    baseline = lay.unpack(base.f32.cpu(), base.i64.cpu())
    rnd = eng.begin(baseline, k)
    rnd.put_baseline(baseline)
    torch.cuda.synchronize(dev)
    order = rnd._fedadp_order()
    segs, n_flat = rnd._flat_segments(order, True)
    g = torch.randn(lay.row_f32, device=dev) * 0.01
    gi = torch.zeros(max(1, lay.row_i64), device=dev)
    g_flat, _ = rnd._flatten(_lib.PLATO_AGG_FLAT_RAW, segs, len(order), n_flat, [g.data_ptr()], [gi.data_ptr()],
                             None, 0.01, stream)

    def ptrs_of(s):
        pf, pi = s.row_pointers(range(k))
        return torch.from_numpy(np.concatenate([pf, pi]).astype(np.int64)).to(dev)

    p_w, p_d = ptrs_of(slab), ptrs_of(dslab)
    ws = torch.empty(-(-_lib.lib().plato_agg_fedadp_dots_workspace(k, 1, n_i, n_flat, len(order)) // 4),
                     dtype=torch.float32, device=dev)
    outs = {}

    def adp(variant):
        delta = bool(_lib.tune().plato_agg_tune_fedadp_is_delta(variant))
        p = p_d if delta else p_w
        xy = torch.empty(k + 1, device=dev)
        yy = torch.empty(k + 1, device=dev)
        _lib.tune_call("plato_agg_tune_fedadp_dots", variant, g_flat.data_ptr(), p.data_ptr(), p.data_ptr() + 8 * k,
                       k, None if delta else _ptr(base.f32), None if delta else _ptr(base.i64), segs.data_ptr(),
                       len(order), n_flat, n_f, n_i, 0.01, 1, ws.data_ptr(), xy.data_ptr(), yy.data_ptr(), h)
        outs[f"adp_v{variant}"] = (xy, yy)

    ef, ei = eng._norm_tables(lay)
    n_e = len(lay.entries)
    tf_w = torch.from_numpy(slab.row_pointers(range(k))[0]).to(dev)
    ti_w = torch.from_numpy(slab.row_pointers(range(k))[1]).to(dev)
    tf_d = torch.from_numpy(dslab.row_pointers(range(k))[0]).to(dev)
    ti_d = torch.from_numpy(dslab.row_pointers(range(k))[1]).to(dev)

    def norms(delta):
        out = torch.empty(k * n_e, device=dev)
        tf, ti = (tf_d, ti_d) if delta else (tf_w, ti_w)
        _lib.call("plato_agg_entry_norms_f32", _ptr(tf), _ptr(ti), k, None if delta else _ptr(base.f32),
                  None if delta else _ptr(base.i64), _ptr(ef), ef.shape[0], _ptr(ei), ei.shape[0], n_e, n_f, n_i,
                  _ptr(out), h)
        outs["norms_delta" if delta else "norms_base"] = out

    scratch = ClientSlab(lay, 1, dev)

    def to_delta():  # the staging-time cost: one client's arena turned into its delta in place
        _lib.call("plato_agg_compute_deltas", _ptr(scratch.f32[0]), _ptr(scratch.i64[0]), _ptr(base.f32),
                  _ptr(base.i64), _ptr(scratch.f32[0]), _ptr(scratch.i64[0]), n_f, n_i, h)

    cases = {f"fedadp_dots_v{v}": (lambda v=v: adp(v)) for v in [int(x) for x in args.adp_variants.split(",")]}
    cases["entry_norms_base"] = lambda: norms(False)
    cases["entry_norms_delta"] = lambda: norms(True)
    cases["compute_deltas_in_place_1_client"] = to_delta
    for fn in cases.values():
        fn()
    torch.cuda.synchronize(dev)
    times = {name: [] for name in cases}
    for _ in range(args.rounds):
        for name, fn in cases.items():
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                fn()
                e1.record(stream)
                e1.synchronize()
                times[name].append(e0.elapsed_time(e1))
    torch.cuda.synchronize(dev)
    ref = outs[f"adp_v{args.adp_variants.split(',')[0]}"]
    for key, val in outs.items():
        if key.startswith("adp_"):
            xy, yy = val
            same = bool(torch.equal(xy.view(torch.int32), ref[0].view(torch.int32))
                        and torch.equal(yy.view(torch.int32), ref[1].view(torch.int32)))
            print(json.dumps({"check": key, "bitwise_equal_to": f"adp_v{args.adp_variants.split(',')[0]}",
                              "equal": same}), flush=True)
    same_n = bool(torch.equal(outs["norms_base"].view(torch.int32), outs["norms_delta"].view(torch.int32)))
    print(json.dumps({"check": "entry_norms delta vs base", "equal": same_n}), flush=True)
    for name in cases:
        print(json.dumps({"case": name, "clients": k, "ms_median": round(statistics.median(times[name]), 4),
                          "ms_min": round(min(times[name]), 4), "samples": len(times[name])}), flush=True)


if __name__ == "__main__":
    main()
