#!/bin/bash
# FedAdp default = variant 60: every FedAdp GPU test, the smoke, the variant timings
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests -k "fedadp or sdot or hostorder" > gpurun_out/r03zd_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03zd_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03zd_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r03zd_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --fedadp-kernel --only fedadp,fedadp_flat --reps 10 > gpurun_out/r03zd_fedadp.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
