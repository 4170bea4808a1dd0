#!/bin/bash
# round 4: FedAdp prep + boundary table fused into one launch (default) against two launches (variant 9)
# interleaved whole-call timing
set -u
mkdir -p gpurun_out/r04y
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_per_entry_gpu.py -k "fedadp" > gpurun_out/r04y/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04y/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --fedadp-kernel --only none --reps 15 > gpurun_out/r04y/fedadp.log 2>&1
rc=$?; echo "fedadp rc=$rc"; grep fedadp_dots gpurun_out/r04y/fedadp.log | cut -c1-150; exit $rc
