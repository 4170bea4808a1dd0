#!/bin/bash
# round 4: FedAtt split shapes (variants 7-9 vs the default) and the 512-thread cosine cascade
set -u
mkdir -p gpurun_out/r04s
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_per_entry_gpu.py tests/test_flat_gpu.py tests/test_golden_gpu.py -k "norm or fedatt or sumsq or polaris or Polaris or cosine or port or Port" > gpurun_out/r04s/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04s/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --cosine-variants --reps 9 --threads 16 > gpurun_out/r04s/cosine.log 2>&1
rc=$?; echo "cosine rc=$rc"; grep cosine_variant gpurun_out/r04s/cosine.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc
for k in 128 64; do
  timeout -k 10 300 python -u scripts/bench_variants.py --only norms --norm-variants --clients $k --reps 4 --interleave 3 > gpurun_out/r04s/norms_k$k.log 2>&1
  rc=$?; echo "norms k=$k rc=$rc"; grep norms gpurun_out/r04s/norms_k$k.log | cut -c1-80; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python -u scripts/bench_variant_paths.py --only port,port_staged --reps 7 > gpurun_out/r04s/port.log 2>&1
rc=$?; echo "port rc=$rc"; cut -c1-100 gpurun_out/r04s/port.log | grep path; exit $rc
