#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 180 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_per_entry_gpu.py -k "fedadp" > gpurun_out/r03n_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03n_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/bench_variant_paths.py --fedadp-only --reps 7 > gpurun_out/r03n_fedadp.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r03n_fedadp.log | grep -E "\"(default|v23|v30|v4[89]|v50)\"" | cut -c1-110
[ $rc -ne 0 ] && exit $rc
true
rc=$?; echo "rc=$rc"; grep cycles gpurun_out/r03n_cycles.log | cut -c1-600
exit $rc
