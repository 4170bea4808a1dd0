#!/bin/bash
# rocprofv3 evidence for the bench kernel, in ONE GPU lease (run on the GPU box).
#   0) bench.py unprofiled               -> the run's ms_per_step / HIP-event kernel_ms (bench.json)
#   1) --kernel-trace --stats            -> per-kernel durations (profiles/*kernel_stats.csv)
#   2) --pmc FETCH_SIZE  (own pass)      -> HBM read bytes (x2 on gfx950, MI355X_MICROARCH.md §HBM)
#   3) --pmc WRITE_SIZE  (own pass)      -> HBM write bytes
# Each pass runs bench.py directly under rocprofv3 (no launcher in between);
# scripts/summarize_profile.py puts the unprofiled run beside the profile.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03}
shift || true
EXTRA="$*"
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
B="python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-host-inclusive $EXTRA"
timeout -k 10 300 $B > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench (unprofiled) rc=$rc"; tail -c 400 $OUT/bench.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $B > $OUT/kt.log 2>&1
rc=$?; echo "kernel-trace rc=$rc"; tail -3 $OUT/kt.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $B > $OUT/fetch.log 2>&1
rc=$?; echo "pmc FETCH_SIZE rc=$rc"; tail -3 $OUT/fetch.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $B > $OUT/write.log 2>&1
rc=$?; echo "pmc WRITE_SIZE rc=$rc"; tail -3 $OUT/write.log
exit $rc
