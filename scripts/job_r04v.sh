#!/bin/bash
# round 4: FedAdp dots without the chain-group-major x / b buffer (x from the flat gradient, b from the
# aligned baseline arena: no prep launch), interleaved whole-call timing against the default
set -u
mkdir -p gpurun_out/r04v
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_per_entry_gpu.py -k "fedadp" > gpurun_out/r04v/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04v/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --fedadp-kernel --only none --reps 15 > gpurun_out/r04v/fedadp.log 2>&1
rc=$?; echo "fedadp rc=$rc"; grep fedadp_dots gpurun_out/r04v/fedadp.log | cut -c1-150; exit $rc
