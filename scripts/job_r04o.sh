#!/bin/bash
# round 4: Port norms at 4,096-position tiles by default; every Port shape bit for bit
set -u
mkdir -p gpurun_out/r04o
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_golden_gpu.py tests/test_hostorder_gpu.py tests/test_multi_gpu.py -k "port or Port or hostorder or client_split" > gpurun_out/r04o/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04o/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --port-gathered --reps 5 > gpurun_out/r04o/port.log 2>&1
rc=$?; echo "port rc=$rc"; grep port_norms gpurun_out/r04o/port.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --only port,port_staged --reps 5 > gpurun_out/r04o/port_path.log 2>&1
rc=$?; echo "port path rc=$rc"; grep '"path"' gpurun_out/r04o/port_path.log | cut -c1-200; exit $rc
