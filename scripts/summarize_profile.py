#!/usr/bin/env python3
"""Summarize a scripts/profile.sh run into profiles/<tag>_*.

Inputs (gpurun_out/prof_<tag>/): kernel-trace stats CSV and the two PMC
passes (FETCH_SIZE, WRITE_SIZE).  HBM bytes per launch follow
MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE counts half the bytes of a wide coalesced stream, so it
is doubled; WRITE_SIZE is exact for 16-byte-per-lane streaming stores.
"""

import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "fedavg_kernel"


def counter(path, name):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == name]
    return statistics.median(vals), len(vals)


def last_json(path):
    """The bench's one JSON result line in a log (None if the run printed none)."""
    try:
        lines = [ln for ln in open(path) if ln.startswith("{")]
    except OSError:
        return None
    return json.loads(lines[-1]) if lines else None


def main(tag, alg_bytes, label, steps=None):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats_csv = os.path.join(src, "kt", "kt_kernel_stats.csv")
    shutil.copy(stats_csv, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    row = next(r for r in csv.DictReader(open(stats_csv)) if KERNEL in r["Name"])
    fetch_kib, n_f = counter(os.path.join(src, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
    write_kib, n_w = counter(os.path.join(src, "write", "write_counter_collection.csv"), "WRITE_SIZE")
    read_bytes = fetch_kib * 1024 * 2
    write_bytes = write_kib * 1024
    avg_ns = float(row["AverageNs"])
    # the timed region's dispatches only (the bench's last `steps` launches; warm-up excluded)
    trace = [r for r in csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_trace.csv")))
             if r["Kernel_Name"] == row["Name"]]
    trace.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in trace]
    run = last_json(os.path.join(src, "bench.json"))
    prof_run = last_json(os.path.join(src, "kt.log"))
    if steps is None:  # the profiled bench's own timed-step count
        steps = (prof_run or run or {}).get("steps", 20)
    timed = durs[-steps:]
    sys.path.insert(0, ROOT)
    import bench  # noqa: E402  (source stamp of the profiled kernel)
    out = {
        "tag": tag,
        "workload": label,
        "kernel": row["Name"],
        "calls": int(row["Calls"]),
        # primary: the timed region's dispatches (the bench's last `steps` launches), the launches its
        # ms_per_step covers; the rocprof stats average over every call (warm-up included) beside it
        "avg_duration_ms": statistics.fmean(timed),
        "avg_duration_source": f"kernel trace, the {len(timed)} timed-region dispatches",
        "rocprof_stats_avg_ms": avg_ns / 1e6,
        "min_duration_ms": float(row["MinNs"]) / 1e6,
        "timed_avg_ms": statistics.fmean(timed),
        "timed_median_ms": statistics.median(timed),
        "timed_dispatches": len(timed),
        "source_sha16": bench.source_stamp(),
        # the same bench command unprofiled, in the same GPU lease (scripts/profile.sh step 0)
        "bench_same_lease": None if run is None else {
            "ms_per_step": run["ms_per_step"], "kernel_ms": run["roofline"]["kernel_ms"],
            "value": run["value"], "frac": run["roofline"]["frac"]},
        "bench_under_kernel_trace": None if prof_run is None else {
            "ms_per_step": prof_run["ms_per_step"], "kernel_ms": prof_run["roofline"]["kernel_ms"]},
        "algorithmic_bytes": alg_bytes,
        "achieved_GBps_timed_avg": alg_bytes / (statistics.fmean(timed) * 1e6),
        "achieved_GBps_rocprof_avg": alg_bytes / avg_ns,
        "pmc": {
            "FETCH_SIZE_KiB_median": fetch_kib,
            "WRITE_SIZE_KiB_median": write_kib,
            "dispatches": [n_f, n_w],
            "hbm_read_bytes": read_bytes,
            "hbm_write_bytes": write_bytes,
            "hbm_bytes": read_bytes + write_bytes,
            "traffic_over_algorithmic": (read_bytes + write_bytes) / alg_bytes,
            "correction": "read = FETCH_SIZE*1024*2 (gfx950 half-count), write = WRITE_SIZE*1024",
        },
    }
    with open(os.path.join(dst, f"{tag}_summary.json"), "w") as f:
        json.dump(out, f, indent=2)
    print(json.dumps(out, indent=2))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3] if len(sys.argv) > 3 else "C2 ResNet-18 x 128")
