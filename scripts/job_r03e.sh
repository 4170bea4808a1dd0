#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_per_entry_gpu.py tests/test_golden_gpu.py tests/test_server_loop_gpu.py > gpurun_out/r03e_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r03e_pytest.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --fedadp-only --reps 5 > gpurun_out/r03e_paths.log 2>&1
rc=$?; echo "paths rc=$rc"; cat gpurun_out/r03e_paths.log
exit $rc
