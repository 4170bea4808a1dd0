#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flat_gpu.py tests/test_per_entry_gpu.py tests/test_multi_gpu.py tests/test_golden_gpu.py -k "sumsq or polaris" > gpurun_out/r03p_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03p_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --polaris-variants --reps 7 > gpurun_out/r03p_polaris.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r03p_polaris.log | cut -c1-160
exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --reps 7 > gpurun_out/r03p_paths.log 2>&1; echo "paths rc=$?"; grep -v amdgpu.ids gpurun_out/r03p_paths.log | cut -c1-120
