#!/bin/bash
# round 4: FedAdp default nt + faster row scan; bench with the variants leg
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r04g
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests -k "fedadp or hostorder or port" > gpurun_out/r04g/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04g/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r04g/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/r04g/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --fedadp-kernel --only fedadp --reps 10 > gpurun_out/r04g/fedadp.log 2>&1
rc=$?; echo "paths rc=$rc"; grep -v amdgpu.ids gpurun_out/r04g/fedadp.log; exit $rc
