#!/bin/bash
set -u
mkdir -p gpurun_out
bash scripts/pmc_sq.sh r03v python3 $GRAFT_REPO_ROOT/scripts/bench_variant_paths.py --fedadp-only --reps 1
rc=$?; echo "pmc rc=$rc"
exit $rc
