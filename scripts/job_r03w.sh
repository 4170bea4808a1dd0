#!/bin/bash
set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_per_entry_gpu.py -k "tile_shapes or fedadp_server" > gpurun_out/r03w_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03w_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --fedadp-only --reps 10 > gpurun_out/r03w_fedadp.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_sq.sh r03w python3 $R/scripts/bench_variant_paths.py --fedadp-only --reps 1
