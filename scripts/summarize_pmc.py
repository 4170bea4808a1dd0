"""Per-kernel medians of the SQ counters collected by scripts/pmc_sq.sh.

Usage: python scripts/summarize_pmc.py gpurun_out/pmc_<tag> [kernel-substring ...]
Prints one JSON line per kernel: the median of each counter over its dispatches,
plus derived ratios (cycles are quad-cycles for SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_*, MI355X_MICROARCH.md §Per-instruction cycle constants).
"""

from __future__ import annotations

import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    subs = sys.argv[2:]
    per = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                if subs and not any(s in name for s in subs):
                    continue
                per[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
                per[name]["_vgpr"] = [float(row["VGPR_Count"])]
                per[name]["_lds"] = [float(row["LDS_Block_Size"])]
    for name, ctr in per.items():
        med = {k: statistics.median(v) for k, v in ctr.items()}
        out = {"kernel": name[:160], **{k: round(v, 1) for k, v in sorted(med.items())}}
        wc = med.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VALU"):
                if k in med:
                    out[f"{k}/WAVE_CYCLES"] = round(med[k] / wc, 3)
        if med.get("SQ_INSTS_LDS"):
            out["bank_conflict_cycles_per_lds_inst"] = round(med.get("SQ_LDS_BANK_CONFLICT", 0) / med["SQ_INSTS_LDS"], 3)
        if med.get("SQ_BUSY_CYCLES") and wc:
            out["avg_waves_resident_per_busy_cycle"] = round(wc / med["SQ_BUSY_CYCLES"], 2)
        print(json.dumps(out))


if __name__ == "__main__":
    main()
