#!/bin/bash
# round 4: FedAdp v2 — parity tests, HIP-event timings of every variant, per-kernel durations
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r04d
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests -k "fedadp or sdot or hostorder or division" > gpurun_out/r04d/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r04d/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --fedadp-kernel --only fedadp --reps 10 > gpurun_out/r04d/fedadp.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/r04d/fedadp.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04d/kt -o kt -- python3 $R/scripts/bench_variant_paths.py --fedadp-kernel --only none --reps 5 > $R/gpurun_out/r04d/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; exit $rc
