#!/bin/bash
# round 4: verify the new FedAtt-norms and QSGD defaults and the pruned tables; bench with variants leg
set -u
mkdir -p gpurun_out/r04m
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_per_entry_gpu.py tests/test_qsgd_gpu.py tests/test_golden_gpu.py tests/test_multi_gpu.py tests/test_flat_gpu.py > gpurun_out/r04m/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04m/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r04m/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/r04m/bench.log; exit $rc
