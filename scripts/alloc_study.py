"""Does the C2 FedAvg kernel's rate depend on the client slab's allocation?  

bench.py --anchor timed the same C2 launch (128 x 11.18 M elements, the bench's row pitch) at
0.842 ms on a dense view of a 12.9 GB slab and at 0.901 ms on a slab of its own size, on one box
(profiles/r05d_anchor.log).  This allocates client slabs of several sizes in turn (freed and
released between them), times the same C2 launch on a dense view of each (HIP events, median of
--reps), and repeats the sequence, so that size effects and per-allocation placement can be told
apart.  One JSON line per (round, slab size).
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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--sizes-gb", default="5.73,12.9,5.73,8,5.73,24")
    args = ap.parse_args()

    from plato_amd import _lib, workloads
    from plato_amd.arena import ArenaLayout

    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    lay = ArenaLayout.from_shapes(workloads.resnet(18, 10))
    k, n, ni = 128, lay.n_f32, lay.n_i64
    pitch = -(-n // 64) * 64
    base = torch.empty(pitch, device=dev).uniform_(-1, 1)
    out = torch.empty(pitch, device=dev)
    base_i = torch.zeros(64, dtype=torch.int64, device=dev)
    out_i = torch.empty(64, device=dev)
    slab_i = torch.zeros((k, 64), dtype=torch.int64, device=dev)
    ti = torch.from_numpy(slab_i.data_ptr() + np.arange(k, dtype=np.int64) * 512).to(dev)
    w = torch.full((k,), 1.0 / k, device=dev)
    nbytes = (k + 2) * (n * 4 + ni * 8)
    for rnd in range(args.rounds):
        for gb in (float(x) for x in args.sizes_gb.split(",")):
            elems = max(k * pitch, int(gb * 1e9) // 4)
            slab = torch.empty(elems, dtype=torch.float32, device=dev)
            slab[: k * pitch].uniform_(-1, 1)
            tf = torch.from_numpy(slab.data_ptr() + np.arange(k, dtype=np.int64) * pitch * 4).to(dev)

            def launch():
                _lib.tune_call("plato_agg_tune_fedavg", 0, 1, tf.data_ptr(), ti.data_ptr(), w.data_ptr(), None, k,
                               base.data_ptr(), base_i.data_ptr(), out.data_ptr(), out_i.data_ptr(), n, ni,
                               stream.cuda_stream)

            for _ in range(3):
                launch()
            torch.cuda.synchronize(dev)
            ts = []
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                launch()
                e1.record(stream)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            med = statistics.median(ts)
            print(json.dumps({"round": rnd, "slab_GB": round(elems * 4 / 1e9, 2), "slab_va": hex(slab.data_ptr()),
                              "kernel_ms": round(med, 4), "kernel_ms_min": round(min(ts), 4),
                              "frac": round(nbytes / (med * 1e-3) / 8e12, 4)}), flush=True)
            del slab, tf
            torch.cuda.synchronize(dev)
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
