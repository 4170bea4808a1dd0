#!/bin/bash
# round 4: QSGD plain form with scalar max_v loads and the batch's codes issued before its table build
set -u
mkdir -p gpurun_out/r04q
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_qsgd_gpu.py > gpurun_out/r04q/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04q/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variants.py --only qsgd --qsgd-list 0,1,5,6 --clients 128 --reps 10 --interleave 5 > gpurun_out/r04q/qsgd.log 2>&1
rc=$?; echo "qsgd rc=$rc"; grep qsgd gpurun_out/r04q/qsgd.log | cut -c1-100; exit $rc
