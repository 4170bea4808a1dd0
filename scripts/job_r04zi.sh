#!/bin/bash
# round 4: cosine kernel trace with the register-resident combine (and its parity tests)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04zi
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu $R/tests/test_flat_gpu.py $R/tests/test_golden_gpu.py -k "cosine or port or Port" > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/scripts/bench_variant_paths.py --cosine-variants --reps 3 --threads 16 > $OUT/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $R/scripts/bench_variant_paths.py --cosine-variants --reps 3 --threads 16 > $OUT/fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv, statistics, glob
out = "/root/repo/gpurun_out/r04zi"
rows = list(csv.DictReader(open(glob.glob(out + "/fetch/fetch_counter_collection.csv")[0])))
v = [float(r["Counter_Value"]) for r in rows if "cosine_chunks" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
print("cosine FETCH_SIZE KiB median", statistics.median(v), "-> read bytes x2", statistics.median(v) * 1024 * 2, "n", len(v))
st = list(csv.DictReader(open(glob.glob(out + "/kt/kt_kernel_stats.csv")[0])))
for r in st:
    if "cosine" in r["Name"] or "scale_by" in r["Name"] or "combine" in r["Name"]:
        print(r["Name"][:80], r["Calls"], r["AverageNs"])
PY
