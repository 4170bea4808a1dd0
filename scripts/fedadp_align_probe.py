"""Does the arena-vs-flat alignment of FedAdp's 16-byte gathers cost time?

In name order (process_grad, fedadp_server.py:122-133) an entry's flat position and its arena
offset differ mod 4 for about half of ResNet-18's fp32 elements (the int64 counters take one flat
position each and are not in the fp32 arena), so the kernel's buffer_load_dwordx4 of b and of the
client arenas start 4, 8 or 12 bytes past a 16-byte boundary there.  This times
plato_agg_fedadp_dots (and the tuning variants named) on the same bytes with a synthetic
two-segment map whose arena offsets are shifted by 0..3 elements, next to the real layout.

Usage: python scripts/fedadp_align_probe.py [--clients 128] [--reps 10] [--variants 51,60]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="")
    args = ap.parse_args()

    from plato_amd import _lib, workloads
    from plato_amd.arena import ArenaLayout
    from plato_amd.engine import DeviceArena, FedAvgEngine
    from plato_amd.synthetic import fill_baseline, fill_clients

    dev = torch.device("cuda", 0)
    k = args.clients
    layout = ArenaLayout.from_shapes(workloads.resnet(18, 10))
    engine = FedAvgEngine(dev)
    base = DeviceArena(layout, dev)
    fill_baseline(base, 0)
    baseline = layout.unpack(base.f32[:layout.n_f32].cpu(), base.i64[:layout.n_i64].cpu())
    rnd = engine.begin(baseline, k)
    rnd.put_baseline(baseline)
    fill_clients(rnd.slab, base, 0, k)
    for s in range(k):
        pf, pi = rnd.slab.row_pointers([s])
        rnd._pf[s], rnd._pi[s] = int(pf[0]), int(pi[0])
        rnd.staged[s] = True
    torch.cuda.synchronize(dev)
    slots = list(range(k))
    n_e = len(layout.entries)
    grads = rnd.launch_entrywise(np.full((n_e, k), 1.0 / k), add_base=False, device=True)
    rnd.fedadp_dots(grads, slots, 0.01)
    g_flat, ptrs, ws = rnd._keep_flat
    order = rnd._fedadp_order()
    segs_real, n_flat_real = rnd._flat_segments(order, True)
    xy = torch.empty(k + 1, device=dev)
    yy = torch.empty(k + 1, device=dev)
    h = torch.cuda.current_stream(dev).cuda_stream
    base_f = rnd._base.f32.data_ptr()
    base_i = rnd._base.i64.data_ptr()
    n_f, n_i = layout.n_f32, layout.n_i64

    def seg_table(shift):
        # one fp32 entry of 64 elements, then one NEG_DIV entry: n_flat = n_f - 64 positions
        n = n_f - 64
        rows = np.asarray([[0, shift, 64, 0], [64, 64 + shift, n - 64, 1 << 32]], dtype=np.uint64)
        return torch.from_numpy(rows.view(np.int64).copy()).to(dev), n

    cases = {"real_layout": (segs_real, len(order), n_flat_real)}
    for sh in range(4):
        t, n = seg_table(sh)
        cases[f"one_entry_shift{sh}"] = (t, 2, n)
    variants = [None] + [int(v) for v in args.variants.split(",") if v]
    for cname, (segs, n_segs, n_flat) in cases.items():
        for v in variants:
            def fn():
                if v is None:
                    _lib.call("plato_agg_fedadp_dots", g_flat.data_ptr(), ptrs.data_ptr(), ptrs.data_ptr() + 8 * k, k,
                              base_f, base_i, segs.data_ptr(), n_segs, n_flat, n_f, n_i, 0.01, 1, ws.data_ptr(),
                              xy.data_ptr(), yy.data_ptr(), h)
                else:
                    _lib.tune_call("plato_agg_tune_fedadp_dots", v, g_flat.data_ptr(), ptrs.data_ptr(),
                                   ptrs.data_ptr() + 8 * k, k, base_f, base_i, segs.data_ptr(), n_segs, n_flat, n_f,
                                   n_i, 0.01, 1, ws.data_ptr(), xy.data_ptr(), yy.data_ptr(), h)
            fn()
            torch.cuda.synchronize(dev)
            ref = xy.cpu().numpy().tobytes() + yy.cpu().numpy().tobytes()
            ts = []
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            same = xy.cpu().numpy().tobytes() + yy.cpu().numpy().tobytes() == ref
            print(json.dumps({"case": cname, "variant": "default" if v is None else v, "n_flat": int(n_flat),
                              "ms_median": round(statistics.median(ts), 4), "ms_min": round(min(ts), 4),
                              "repeatable": same}), flush=True)


if __name__ == "__main__":
    main()
