#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_golden_gpu.py tests/test_flat_gpu.py tests/test_per_entry_gpu.py -k "port or similarit or cosine or torch" > gpurun_out/r03q_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03q_pytest.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r03q -o kt -- python3 $GRAFT_REPO_ROOT/scripts/bench_variant_paths.py --port-only --reps 5 > $GRAFT_REPO_ROOT/gpurun_out/r03q_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; grep -v amdgpu.ids $GRAFT_REPO_ROOT/gpurun_out/r03q_kt.log | grep path | cut -c1-120
exit $rc
