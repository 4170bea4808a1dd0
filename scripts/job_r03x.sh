#!/bin/bash
# SQ counters (LDS bank conflicts, waits) of every kernel on the per-algorithm paths and the bench
set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
bash scripts/pmc_sq.sh r03x_paths python3 $R/scripts/bench_variant_paths.py --reps 1 || exit $?
bash scripts/pmc_sq.sh r03x_bench python3 $R/bench.py --steps 2 --warmup 1 || exit $?
