#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_per_entry_gpu.py tests/test_multi_gpu.py tests/test_golden_gpu.py tests/test_server_loop_gpu.py -k "fedatt or entry_norm" > gpurun_out/r03t_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03t_pytest.log
[ $rc -ne 0 ] && exit $rc
for th in 0 131072 524288 1048576 32768; do
  timeout -k 10 120 python -u scripts/bench_variant_paths.py --only fedatt --reps 9 --norms-threshold $th >> gpurun_out/r03t_fedatt.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "paths rc=$rc"; exit $rc; }
done
grep -v amdgpu.ids gpurun_out/r03t_fedatt.log | cut -c1-150
