#!/bin/bash
# round 4: the whole GPU suite, smoke and the default bench on one box
set -u
mkdir -p gpurun_out/r04t
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_full_size_gpu.py > gpurun_out/r04t/pytest_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04t/pytest_full.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04t/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/r04t/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r04t/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 2500 gpurun_out/r04t/bench.log; exit $rc
