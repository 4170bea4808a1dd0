#!/bin/bash
# round 4: FedAtt norms chain with two 16-step blocks in flight and one wait per block (variant 8, 64 VGPRs)
set -u
mkdir -p gpurun_out/r04zl
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_per_entry_gpu.py -k "norm" > gpurun_out/r04zl/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04zl/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
for k in 128 64 4; do
  timeout -k 10 300 python -u scripts/bench_variants.py --only norms --norm-variants --clients $k --reps 5 --interleave 4 > gpurun_out/r04zl/norms_k$k.log 2>&1
  rc=$?; echo "norms k=$k rc=$rc"; grep norms gpurun_out/r04zl/norms_k$k.log | cut -c1-80; [ $rc -eq 0 ] || exit $rc
done
