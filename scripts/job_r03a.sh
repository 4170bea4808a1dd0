#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_server_loop_gpu.py tests/test_hostorder_gpu.py tests/test_golden_gpu.py tests/test_per_entry_gpu.py > gpurun_out/r03a_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r03a_pytest.log
[ $rc -ge 124 ] && exit $rc
bash scripts/profile.sh r03a
