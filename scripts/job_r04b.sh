#!/bin/bash
# round 4: FedAdp v2 (chain-group-major x/b, 256-step stages) — parity tests, then timings of every variant
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests -k "fedadp or sdot or hostorder or division" > gpurun_out/r04b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r04b_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_variant_paths.py --fedadp-kernel --only fedadp,fedadp_flat --reps 10 > gpurun_out/r04b_fedadp.log 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r04b_fedadp.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/fedadp_align_probe.py --reps 10 --variants 1,2,3 > gpurun_out/r04b_align.log 2>&1
rc=$?; echo "align rc=$rc"; cat gpurun_out/r04b_align.log | grep -v amdgpu.ids; exit $rc
