#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_per_entry_gpu.py tests/test_golden_gpu.py tests/test_multi_gpu.py tests/test_hostorder_gpu.py -k "fedadp or probe" > gpurun_out/r03j_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03j_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --reps 7 > gpurun_out/r03j_paths.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r03j_paths.log | cut -c1-150
exit $rc
