#!/bin/bash
# round 4: Port norms chain with one s_waitcnt per 16- or 32-step block (variants 6, 7): parity and timing
# port_norms, the variant timings
set -u
mkdir -p gpurun_out/r04zz
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_golden_gpu.py tests/test_per_entry_gpu.py tests/test_hostorder_gpu.py tests/test_multi_gpu.py -k "port or Port or threshold or long or hostorder" > gpurun_out/r04zz/pytest3.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04zz/pytest3.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --port-gathered --only port,port_staged --reps 7 > gpurun_out/r04zz/port3.log 2>&1
rc=$?; echo "port rc=$rc"; grep "port" gpurun_out/r04zz/port3.log | cut -c1-120; exit $rc
