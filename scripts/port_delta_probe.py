#!/usr/bin/env python3
"""Port's similarity reductions on weight arenas vs delta arenas (FedAvgEngine.delta_arenas), interleaved.

K ResNet-18 clients filled on the device (as bench.py's variant legs do), one round per arena kind; each
call is AggregationRound.model_similarities (port_norms + the cosine sums); prints the median HIP-event
times of both kernels per kind and whether the similarities are bitwise equal.
Usage: python scripts/port_delta_probe.py [--clients 128] [--reps 10] [--rounds 3]
"""

import argparse
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()

    from plato_amd import workloads
    from plato_amd.arena import ArenaLayout
    from plato_amd.engine import DeviceArena, FedAvgEngine
    from plato_amd.synthetic import fill_baseline, fill_clients

    dev = torch.device("cuda", 0)
    k = args.clients
    spec = workloads.resnet(18, 10)
    slots = list(range(k))

    def make_round(deltas):
        lay = ArenaLayout.from_shapes(spec)
        base = DeviceArena(lay, dev)
        fill_baseline(base, 0)
        baseline = lay.unpack(base.f32.cpu(), base.i64.cpu())
        eng = FedAvgEngine(dev)
        eng.delta_arenas = deltas
        rnd = eng.begin(baseline, k)
        rnd.put_baseline(baseline)
        torch.cuda.synchronize(dev)
        fill_clients(rnd.slab, eng._base, 0, k)
        for s in range(k):
            pf, pi = rnd.slab.row_pointers([s])
            rnd._pf[s], rnd._pi[s] = int(pf[0]), int(pi[0])
            rnd.staged[s] = True
            if deltas:
                rnd._to_delta(s)
        torch.cuda.synchronize(dev)
        prev = DeviceArena(lay, dev)
        fill_baseline(prev, 1)
        previous = lay.unpack(prev.f32.cpu(), prev.i64.cpu())
        return rnd, rnd.stage_reference(previous)

    rounds = {kind: make_round(kind == "deltas") for kind in ("weights", "deltas")}
    times = {kind: {"port_norms": [], "port_cosine": []} for kind in rounds}
    sims = {}
    for kind, (rnd, ref) in rounds.items():
        sims[kind] = rnd.model_similarities(ref, slots)
    for _ in range(args.rounds):
        for kind, (rnd, ref) in rounds.items():
            for _ in range(args.reps):
                rnd.model_similarities(ref, slots)
                for key in times[kind]:
                    times[kind][key].append(rnd.timings[key + "_ms"])
    same = bool(np.asarray(sims["weights"]).tobytes() == np.asarray(sims["deltas"]).tobytes())
    for kind in rounds:
        print(json.dumps({"arenas": kind, "clients": k,
                          **{f"{key}_ms_median": round(statistics.median(v), 4) for key, v in times[kind].items()},
                          "similarities_bitwise_equal": same}), flush=True)


if __name__ == "__main__":
    main()
