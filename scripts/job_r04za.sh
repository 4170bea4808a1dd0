#!/bin/bash
# round 4: one s_waitcnt per chain block — FedAtt norms variants 6 / 7 against the default, and the Port
# default (one wait per 32 steps): parity and interleaved timing
set -u
mkdir -p gpurun_out/r04za
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_per_entry_gpu.py tests/test_golden_gpu.py tests/test_hostorder_gpu.py -k "norm or fedatt or port or Port or hostorder" > gpurun_out/r04za/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04za/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
for k in 128 4; do
  timeout -k 10 300 python -u scripts/bench_variants.py --only norms --norm-variants --clients $k --reps 5 --interleave 4 > gpurun_out/r04za/norms_k$k.log 2>&1
  rc=$?; echo "norms k=$k rc=$rc"; grep norms gpurun_out/r04za/norms_k$k.log | cut -c1-80; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u scripts/bench_variant_paths.py --only port_staged --reps 7 > gpurun_out/r04za/port_path.log 2>&1
rc=$?; echo "port path rc=$rc"; grep path gpurun_out/r04za/port_path.log | cut -c1-120; exit $rc
