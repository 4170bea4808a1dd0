#!/bin/bash
set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/bench_variant_paths.py --fedadp-only --reps 10 > gpurun_out/r03z_fedadp.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_sq.sh r03z python3 $R/scripts/bench_variant_paths.py --fedadp-only --reps 1
