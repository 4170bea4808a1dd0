#!/bin/bash
# round 4: FedAtt norms with short entries on the per-wave launch (variants 8, 9)
set -u
mkdir -p gpurun_out/r04ze
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_per_entry_gpu.py -k "norm" > gpurun_out/r04ze/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04ze/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
for k in 128 32; do
  timeout -k 10 300 python -u scripts/bench_variants.py --only norms --norm-variants --clients $k --reps 5 --interleave 4 > gpurun_out/r04ze/norms_k$k.log 2>&1
  rc=$?; echo "norms k=$k rc=$rc"; grep norms gpurun_out/r04ze/norms_k$k.log | cut -c1-80; [ $rc -eq 0 ] || exit $rc
done
