#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_per_entry_gpu.py -k "fedadp" > gpurun_out/r03b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r03b_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --fedadp-kernel --reps 5 > gpurun_out/r03b_paths.log 2>&1
rc=$?; echo "paths rc=$rc"; cat gpurun_out/r03b_paths.log
exit $rc
