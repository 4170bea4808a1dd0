#!/bin/bash
# round 4: register-staged FedAtt norms kernel shapes; QSGD software-pipelined / persistent shapes;
# FedAdp parallel boundary-row scan
set -u
mkdir -p gpurun_out/r04i
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_qsgd_gpu.py tests/test_per_entry_gpu.py tests/test_multi_gpu.py tests/test_flat_gpu.py > gpurun_out/r04i/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04i/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variants.py --only qsgd --qsgd-variants --clients 128 --reps 20 > gpurun_out/r04i/qsgd_k128.log 2>&1
rc=$?; echo "qsgd rc=$rc"; grep qsgd gpurun_out/r04i/qsgd_k128.log; [ $rc -eq 0 ] || exit $rc
for k in 128 32 4; do
  timeout -k 10 300 python -u scripts/bench_variants.py --only norms --norm-variants --clients $k --reps 10 > gpurun_out/r04i/norms_k$k.log 2>&1
  rc=$?; echo "norms k=$k rc=$rc"; grep norms gpurun_out/r04i/norms_k$k.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u scripts/bench_variant_paths.py --polaris-variants --reps 10 > gpurun_out/r04i/polaris.log 2>&1
rc=$?; echo "polaris rc=$rc"; tail -6 gpurun_out/r04i/polaris.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04i/prof -o adp -- python -u scripts/bench_variant_paths.py --only fedadp --reps 5 > gpurun_out/r04i/fedadp_paths.log 2>&1
rc=$?; echo "fedadp rc=$rc"; tail -5 gpurun_out/r04i/fedadp_paths.log; exit $rc
