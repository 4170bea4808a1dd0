#!/bin/bash
# round 4: FedAdp v3 (descriptor table, boundary groups precomputed) — parity tests, timings, kernel trace
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r04f
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests -k "fedadp or sdot or hostorder or division or port" > gpurun_out/r04f/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04f/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --fedadp-kernel --only fedadp --reps 10 > gpurun_out/r04f/fedadp.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/r04f/fedadp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/fedadp_align_probe.py --reps 10 --variants 2 > gpurun_out/r04f/align.log 2>&1
rc=$?; echo "align rc=$rc"; grep -v amdgpu.ids gpurun_out/r04f/align.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04f/kt -o kt -- python3 $R/scripts/bench_variant_paths.py --fedadp-kernel --only none --reps 5 > $R/gpurun_out/r04f/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; exit $rc
