#!/bin/bash
# rocprofv3 evidence for the variant kernels (scripts/bench_variants.py): per-kernel
# durations, then HBM bytes from FETCH_SIZE / WRITE_SIZE in their own passes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01_variants}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
B="python3 $R/scripts/bench_variants.py --reps 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $B > $OUT/kt.log 2>&1
rc=$?; echo "kernel-trace rc=$rc"; tail -3 $OUT/kt.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $B > $OUT/fetch.log 2>&1
rc=$?; echo "pmc FETCH_SIZE rc=$rc"; tail -3 $OUT/fetch.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $B > $OUT/write.log 2>&1
rc=$?; echo "pmc WRITE_SIZE rc=$rc"; tail -3 $OUT/write.log
find $OUT -name "*.csv" | head -20
exit 0
