#!/bin/bash
# round 4: cosine sums with chunks grouped by XCD (variant 2)
set -u
mkdir -p gpurun_out/r04zm
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_flat_gpu.py tests/test_golden_gpu.py tests/test_hostorder_gpu.py tests/test_multi_gpu.py -k "cosine or port or Port or hostorder" > gpurun_out/r04zm/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04zm/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/bench_variant_paths.py --cosine-variants --reps 15 --threads 16 > gpurun_out/r04zm/cosine.log 2>&1
rc=$?; echo "cosine rc=$rc"; grep cosine_variant gpurun_out/r04zm/cosine.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --only port_staged --reps 7 > gpurun_out/r04zm/port_path.log 2>&1
rc=$?; echo "port path rc=$rc"; grep path gpurun_out/r04zm/port_path.log | cut -c1-120; exit $rc
