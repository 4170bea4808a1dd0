#!/bin/bash
# round 4: client-split FedAdp / Port over aggregation_devices; FedAdp default nt; bench with the variants leg
set -u
mkdir -p gpurun_out/r04h
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_multi_gpu.py tests/test_per_entry_gpu.py tests/test_hostorder_gpu.py > gpurun_out/r04h/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04h/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r04h/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3500 gpurun_out/r04h/bench.log; exit $rc
