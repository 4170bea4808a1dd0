#!/bin/bash
# QSGD sign-rotated tables: parity, timing (two orders), SQ counters of default vs rotated
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_qsgd_gpu.py > gpurun_out/r03m_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03m_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_variants.py --only qsgd --qsgd-list 0,61,62,63,14,0,61 --reps 20 > gpurun_out/r03m_qsgd.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r03m_qsgd.log | cut -c1-160
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_variants.py --only qsgd --qsgd-list 0,61,62,63,14,0,61 --reps 20 --qsgd-codes uniform > gpurun_out/r03m_qsgd_uniform.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r03m_qsgd_uniform.log | cut -c1-160
[ $rc -ne 0 ] && exit $rc
bash scripts/pmc_sq.sh r03m python3 $GRAFT_REPO_ROOT/scripts/bench_variants.py --only qsgd --qsgd-list 0,61 --reps 3
rc=$?; echo "pmc rc=$rc"
exit $rc
