#!/bin/bash
# round 4: more register-staged FedAtt norms shapes (K = 128 / 64 / 32 / 4, interleaved), QSGD A/B of
# the default against the round-1 shape, FedAdp overhead kernels under rocprof (csv)
set -u
mkdir -p gpurun_out/r04j
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_per_entry_gpu.py -k "norm or fedatt or fedadp" > gpurun_out/r04j/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04j/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
for k in 128 64 32 4; do
  timeout -k 10 300 python -u scripts/bench_variants.py --only norms --norm-variants --clients $k --reps 4 --interleave 3 > gpurun_out/r04j/norms_k$k.log 2>&1
  rc=$?; echo "norms k=$k rc=$rc"; grep norms gpurun_out/r04j/norms_k$k.log | cut -c1-110; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u scripts/bench_variants.py --only qsgd --qsgd-list 0,1,5,7 --clients 128 --reps 10 --interleave 5 > gpurun_out/r04j/qsgd_ab.log 2>&1
rc=$?; echo "qsgd rc=$rc"; grep qsgd gpurun_out/r04j/qsgd_ab.log | cut -c1-110; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04j/prof -o adp -- python3 -u scripts/bench_variant_paths.py --only fedadp --reps 5 > gpurun_out/r04j/fedadp_paths.log 2>&1
rc=$?; echo "fedadp rc=$rc"; grep '"path"' gpurun_out/r04j/fedadp_paths.log; exit $rc
