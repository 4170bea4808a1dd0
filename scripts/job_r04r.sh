#!/bin/bash
# round 4: Polaris np_sumsq without LDS staging for full chunks (direct kernel + tail kernel)
set -u
mkdir -p gpurun_out/r04r
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_flat_gpu.py tests/test_per_entry_gpu.py tests/test_golden_gpu.py -k "sumsq or polaris or Polaris" > gpurun_out/r04r/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04r/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --polaris-variants --reps 10 > gpurun_out/r04r/polaris.log 2>&1
rc=$?; echo "polaris rc=$rc"; grep np_sumsq gpurun_out/r04r/polaris.log; exit $rc
