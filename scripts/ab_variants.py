"""Interleaved A/B timing of FedAvg kernel variants on the C2 workload.

Usage: python scripts/ab_variants.py 0 11 14 16 [--rounds 30 --launches 10]
Prints the median and quartiles of ms per launch and GB/s per variant.
"""

import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", type=int, nargs="+")
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--launches", type=int, default=10)
    args = ap.parse_args()
    from plato_amd import synthetic, workloads
    from plato_amd.arena import ArenaLayout
    from plato_amd.engine import ClientSlab, DeviceArena, FedAvgEngine, fp32_weights

    dev = torch.device("cuda", 0)
    layout = ArenaLayout.from_shapes(workloads.resnet(18, 10))
    k = 128
    base = DeviceArena(layout, dev)
    slab = ClientSlab(layout, k, dev)
    synthetic.fill_baseline(base, 0)
    synthetic.fill_clients(slab, base, 0, k)
    w = torch.from_numpy(fp32_weights(synthetic.fedavg_weights(synthetic.num_samples(k, 0))
                                      if hasattr(synthetic, "fedavg_weights") else
                                      [n / sum(synthetic.num_samples(k, 0)) for n in synthetic.num_samples(k, 0)])).to(dev)
    pf, pi = slab.row_pointers(range(k))
    tf, ti = torch.from_numpy(pf).to(dev), torch.from_numpy(pi).to(dev)
    out_f = torch.empty(layout.row_f32, device=dev)
    out_i = torch.empty(layout.row_i64, device=dev)
    eng = FedAvgEngine(dev)
    stream = torch.cuda.current_stream(dev)
    times = {v: [] for v in args.variants}
    for v in args.variants:
        eng.variant = v
        for _ in range(3):
            eng.launch_fedavg(layout, tf, ti, w, None, k, base.f32, base.i64, out_f, out_i, stream)
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for v in args.variants:
            eng.variant = v
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.launches):
                eng.launch_fedavg(layout, tf, ti, w, None, k, base.f32, base.i64, out_f, out_i, stream)
            e1.record(stream)
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) / args.launches)
    nbytes = layout.algorithmic_bytes(k)
    for v in args.variants:
        ts = sorted(times[v])
        med = statistics.median(ts)
        print(json.dumps({"variant": v, "ms_median": round(med, 4), "ms_q1": round(ts[len(ts) // 4], 4),
                          "ms_q3": round(ts[3 * len(ts) // 4], 4), "GBps": round(nbytes / med / 1e6, 1)}))


if __name__ == "__main__":
    main()
