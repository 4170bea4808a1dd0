#!/bin/bash
# round-3 HEAD check: full GPU suite, smoke, same-lease bench + rocprof passes
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r03r_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r03r_pytest_gpu.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03r_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/r03r_smoke.log
[ $rc -ne 0 ] && exit $rc
bash scripts/profile.sh r03r
rc=$?; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r03r_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/r03r_bench.log
exit $rc
