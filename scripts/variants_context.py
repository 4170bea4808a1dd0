"""Do the variant kernels time the same inside bench.py's round as in bench_variants.py's slab?  

Builds the round the way bench.py's `variants` leg does (FedAvgEngine.begin + fill_clients into the round's
slab) and times, interleaved with HIP events, the product FedAtt norms / Polaris sums through the round's own
methods (the bench's numbers) and the tuning library's one-client / two-client forms on the same pointers.
"""

from __future__ import annotations

import json
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from plato_amd import _lib, workloads
    from plato_amd.arena import ArenaLayout
    from plato_amd.engine import DeviceArena, FedAvgEngine, _ptr
    from plato_amd.synthetic import fill_baseline, fill_clients

    dev = torch.device("cuda", 0)
    k = 128
    lay = ArenaLayout.from_shapes(workloads.resnet(18, 10))
    base = DeviceArena(lay, dev)
    fill_baseline(base, 0)
    baseline = lay.unpack(base.f32.cpu(), base.i64.cpu())
    eng = FedAvgEngine(dev)
    rnd = eng.begin(baseline, k)
    rnd.put_baseline(baseline)
    torch.cuda.synchronize(dev)
    fill_clients(rnd.slab, eng._base, 0, k)
    for s in range(k):
        pf, pi = rnd.slab.row_pointers([s])
        rnd._pf[s], rnd._pi[s] = int(pf[0]), int(pi[0])
        rnd.staged[s] = True
    torch.cuda.synchronize(dev)
    slots = list(range(k))
    lay = rnd.layout  # the round's own layout object (its caches)
    stream = torch.cuda.current_stream(dev)
    h = stream.cuda_stream
    pf = np.asarray([rnd._pf[i] for i in slots], dtype=np.int64)
    pi = np.asarray([rnd._pi[i] for i in slots], dtype=np.int64)
    tf, ti = eng._pointer_tables(pf, pi)
    ef, ei = eng._norm_tables(lay)
    n_e = len(lay.entries)
    out = torch.empty(k * n_e, device=dev)
    rnd.np_sumsq(slots)
    pieces, first, entry_of, n_chunks = lay._cache[("np_sumsq_pieces", str(dev))]
    ws = torch.empty(max(1, eng.lib.plato_agg_np_sumsq_workspace(k, n_chunks) // 4), device=dev)
    sq_out = torch.empty((k, int(entry_of.size)), device=dev)

    def norms(v):
        _lib.tune_call("plato_agg_tune_entry_norms", v, _ptr(tf), _ptr(ti), k, _ptr(rnd._base.f32), _ptr(rnd._base.i64),
                       _ptr(ef), ef.shape[0], _ptr(ei), ei.shape[0], n_e, lay.n_f32, lay.n_i64, _ptr(out), h)

    def sumsq(v):
        _lib.tune_call("plato_agg_tune_np_sumsq", v, tf.data_ptr(), k, rnd._base.f32.data_ptr(), pieces.data_ptr(),
                       first.data_ptr(), int(entry_of.size), n_chunks, ws.data_ptr(), sq_out.data_ptr(), h)

    def events(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1)

    def round_method(name, fn):
        fn()
        return rnd.timings[name + "_ms"]

    cases = {
        "fedatt_round_method": lambda: round_method("entry_norms", lambda: rnd.entry_norms(slots)),
        "fedatt_one_client": lambda: events(lambda: norms(8)),
        "fedatt_two_clients": lambda: events(lambda: norms(9)),
        "fedatt_default": lambda: events(lambda: norms(0)),
        "polaris_round_method": lambda: round_method("np_sumsq", lambda: rnd.np_sumsq(slots)),
        "polaris_one_client": lambda: events(lambda: sumsq(6)),
        "polaris_two_clients": lambda: events(lambda: sumsq(0)),
    }
    def run_cases(tag):
        times = {n: [] for n in cases}
        for fn in cases.values():
            fn()
        for _ in range(5):
            for n, fn in cases.items():
                times[n].extend(fn() for _ in range(3))
        for n, ts in times.items():
            print(json.dumps({"pass": tag, "case": n, "ms_median": round(statistics.median(ts), 4),
                              "ms_min": round(min(ts), 4), "samples": len(ts)}), flush=True)

    run_cases("first round, fresh process")
    if "--with-bench-legs" in sys.argv:
        import bench

        legs = bench.variant_legs(dev, k, 5)
        print(json.dumps({"pass": "bench.variant_legs (its own rounds)",
                          **{n: v.get("kernel_ms") for n, v in legs.items() if isinstance(v, dict)}}), flush=True)
        run_cases("first round again, after bench.variant_legs")


if __name__ == "__main__":
    main()
