#!/bin/bash
set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_golden_gpu.py tests/test_per_entry_gpu.py -k "port or entry_norms" > gpurun_out/r03y_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03y_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --port-gathered --only port_staged,port --reps 10 > gpurun_out/r03y_port.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_sq.sh r03y python3 $R/scripts/bench_variant_paths.py --port-only --reps 1
