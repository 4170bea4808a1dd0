#!/bin/bash
# round 4: FedAtt norms with the lookahead d ring (interleaved against the register-staged shapes)
set -u
mkdir -p gpurun_out/r04l
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_per_entry_gpu.py -k "norm or fedatt" > gpurun_out/r04l/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04l/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
for k in 128 64 4; do
  timeout -k 10 300 python -u scripts/bench_variants.py --only norms --norm-variants --clients $k --reps 4 --interleave 3 > gpurun_out/r04l/norms_k$k.log 2>&1
  rc=$?; echo "norms k=$k rc=$rc"; grep norms gpurun_out/r04l/norms_k$k.log | cut -c1-80; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_qsgd_gpu.py > gpurun_out/r04l/pytest_qsgd.log 2>&1
rc=$?; echo "pytest qsgd rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04l/pytest_qsgd.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variants.py --only qsgd --qsgd-list 0,12,13,14 --clients 128 --reps 10 --interleave 4 > gpurun_out/r04l/qsgd.log 2>&1
rc=$?; echo "qsgd rc=$rc"; grep qsgd gpurun_out/r04l/qsgd.log | cut -c1-100; exit $rc
