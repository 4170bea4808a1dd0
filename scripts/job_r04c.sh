#!/bin/bash
# round 4: per-kernel durations of the FedAdp variants (kernel trace stats)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r04c
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04c/kt -o kt -- python3 $R/scripts/bench_variant_paths.py --fedadp-kernel --only none --reps 5 > $R/gpurun_out/r04c/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; tail -3 $R/gpurun_out/r04c/kt.log
f=$(find $R/gpurun_out/r04c/kt -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -30
exit $rc
