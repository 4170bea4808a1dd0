#!/bin/bash
# round 4: QSGD-coded FedAvg at 384 / 640 threads (3,072 / 5,120-element chunks; variants 7, 8) against the default
set -u
mkdir -p gpurun_out/r04zo
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_qsgd_gpu.py > gpurun_out/r04zo/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04zo/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variants.py --only qsgd --qsgd-list 0,6,7,8 --reps 10 --interleave 4 > gpurun_out/r04zo/qsgd.log 2>&1
rc=$?; echo "qsgd rc=$rc"; grep qsgd gpurun_out/r04zo/qsgd.log | cut -c1-90; exit $rc
