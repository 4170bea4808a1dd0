#!/bin/bash
# round 4: 4,096-element tiles for the register-staged norms; np_sumsq at 512 / 1,024 threads
set -u
mkdir -p gpurun_out/r04n
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_per_entry_gpu.py tests/test_flat_gpu.py -k "norm or sumsq or polaris" > gpurun_out/r04n/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04n/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
for k in 128 4; do
  timeout -k 10 300 python -u scripts/bench_variants.py --only norms --norm-variants --clients $k --reps 4 --interleave 3 > gpurun_out/r04n/norms_k$k.log 2>&1
  rc=$?; echo "norms k=$k rc=$rc"; grep norms gpurun_out/r04n/norms_k$k.log | cut -c1-80; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u scripts/bench_variant_paths.py --polaris-variants --reps 10 > gpurun_out/r04n/polaris.log 2>&1
rc=$?; echo "polaris rc=$rc"; grep np_sumsq gpurun_out/r04n/polaris.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --port-gathered --reps 5 > gpurun_out/r04n/port.log 2>&1
rc=$?; echo "port rc=$rc"; grep port_norms gpurun_out/r04n/port.log | cut -c1-160; exit $rc
