#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_golden_gpu.py tests/test_per_entry_gpu.py tests/test_multi_gpu.py tests/test_hostorder_gpu.py tests/test_server_loop_gpu.py -k "port or similarit or probe" > gpurun_out/r03k_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/r03k_pytest.log
[ $rc -ne 0 ] && exit $rc
true
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r03k_port.log | cut -c1-180
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --reps 7 > gpurun_out/r03k_paths.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r03k_paths.log | cut -c1-150
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r03k -o kt -- python3 $GRAFT_REPO_ROOT/scripts/bench_variant_paths.py --port-only --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/r03k_kt.log 2>&1
rc=$?; echo "kt rc=$rc"
exit $rc
