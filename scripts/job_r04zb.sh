#!/bin/bash
# round 4: Polaris leaves staged transposed (4 ds_read_b128 + one wait per lane, variant 5) against the default
set -u
mkdir -p gpurun_out/r04zb
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_flat_gpu.py tests/test_golden_gpu.py -k "sumsq or polaris or Polaris" > gpurun_out/r04zb/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04zb/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --polaris-variants --reps 15 > gpurun_out/r04zb/polaris.log 2>&1
rc=$?; echo "polaris rc=$rc"; grep np_sumsq gpurun_out/r04zb/polaris.log | cut -c1-140; exit $rc
