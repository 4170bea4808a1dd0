#!/bin/bash
# round 4 close: the whole GPU suite, smoke, the same-lease profile of the bench kernel, the default bench
set -u
mkdir -p gpurun_out/r04x
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/r04x/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04x/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04x/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r04x/smoke.log; [ $rc -eq 0 ] || exit $rc
bash scripts/profile.sh r04z
rc=$?; echo "profile rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py > gpurun_out/r04x/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 1200 gpurun_out/r04x/bench.log; exit $rc
