#!/bin/bash
# round 4: Port norms: 4 producers or 3 tiles in flight with the one-wait chain (variants 8, 9)
# port_norms, the variant timings
set -u
mkdir -p gpurun_out/r04zz
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_golden_gpu.py tests/test_per_entry_gpu.py tests/test_hostorder_gpu.py tests/test_multi_gpu.py -k "port or Port or threshold or long or hostorder" > gpurun_out/r04zz/pytest4.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04zz/pytest4.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --port-gathered --only port,port_staged --reps 7 > gpurun_out/r04zz/port4.log 2>&1
rc=$?; echo "port rc=$rc"; grep "port" gpurun_out/r04zz/port4.log | cut -c1-120; exit $rc
