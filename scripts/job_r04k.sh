#!/bin/bash
# round 4: persistent long/short-split FedAtt norms; QSGD plain-form default and shapes (interleaved)
set -u
mkdir -p gpurun_out/r04k
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_qsgd_gpu.py tests/test_per_entry_gpu.py -k "qsgd or norm or fedatt" > gpurun_out/r04k/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04k/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variants.py --only qsgd --qsgd-list 0,1,8,9,10,11 --clients 128 --reps 10 --interleave 4 > gpurun_out/r04k/qsgd.log 2>&1
rc=$?; echo "qsgd rc=$rc"; grep qsgd gpurun_out/r04k/qsgd.log | cut -c1-100; [ $rc -eq 0 ] || exit $rc
for k in 128 64 32 4; do
  timeout -k 10 300 python -u scripts/bench_variants.py --only norms --norm-variants --clients $k --reps 4 --interleave 3 > gpurun_out/r04k/norms_k$k.log 2>&1
  rc=$?; echo "norms k=$k rc=$rc"; grep norms gpurun_out/r04k/norms_k$k.log | cut -c1-80; [ $rc -eq 0 ] || exit $rc
done
