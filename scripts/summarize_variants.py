#!/usr/bin/env python3
"""Per-kernel summary of a scripts/profile_variants.sh run -> profiles/<tag>_summary.json.

HBM bytes per launch as MI355X_MICROARCH.md §HBM prescribes: read =
FETCH_SIZE (KiB) * 1024 * 2 (gfx950 half-count), write = WRITE_SIZE * 1024.
Algorithmic bytes come from the bench_variants log lines of the same run.
"""

import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"qsgd": "fedavg_qsgd_", "entrywise": "fedavg_entrywise_kernel",
           "stats": "entry_stats_partial", "norms": "entry_norms", "fedavg": "fedavg_kernel",
           "sumsq": "np_sumsq_half4"}


def per_kernel(path, name):
    """Median counter value per kernel name (the kernel trace's Name, e.g. one entry_norms instantiation)."""
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name:
            out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in out.items()}


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    alg = {}
    for line in open(os.path.join(src, "kt.log")):
        if line.startswith("{") and '"kernel"' in line:
            d = json.loads(line)
            alg[d["kernel"]] = d["algorithmic_bytes"]
    rows = list(csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))))
    fetch = per_kernel(os.path.join(src, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, "write", "write_counter_collection.csv"), "WRITE_SIZE")
    out = {"tag": tag, "workload": "ResNet-18 x 128 clients (scripts/bench_variants.py)", "kernels": {}}
    for key, sym in KERNELS.items():
        cand = [r for r in rows if sym in r["Name"]]
        if key == "fedavg":
            cand = [r for r in cand if "qsgd" not in r["Name"] and "entrywise" not in r["Name"]]
        if not cand or key not in alg:
            continue
        row = max(cand, key=lambda r: float(r["TotalDurationNs"]))  # the path's main kernel (norms, sumsq: 2 each)
        avg_ns = float(row["AverageNs"])
        rd = fetch.get(row["Name"], 0) * 1024 * 2
        wr = write.get(row["Name"], 0) * 1024
        out["kernels"][key] = {
            "kernel": row["Name"], "calls": int(row["Calls"]), "avg_duration_ms": avg_ns / 1e6,
            "algorithmic_bytes": alg[key], "achieved_GBps": alg[key] / avg_ns,
            "frac_of_8TBps": alg[key] / avg_ns / 8000.0,
            "hbm_read_bytes": rd, "hbm_write_bytes": wr,
            "traffic_over_algorithmic": (rd + wr) / alg[key] if alg[key] else None,
        }
    with open(os.path.join(dst, f"{tag}_summary.json"), "w") as f:
        json.dump(out, f, indent=2)
    print(json.dumps(out, indent=2))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01_variants")
