#!/bin/bash
# round 4: cosine cascade with double-buffered level-0 sums (A/B, parity), and FedAtt norms timed
# three ways on one box (kernel table, engine path, bench variants leg)
set -u
mkdir -p gpurun_out/r04u
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_flat_gpu.py tests/test_golden_gpu.py tests/test_hostorder_gpu.py -k "cosine or port or Port or hostorder" > gpurun_out/r04u/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04u/pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/bench_variant_paths.py --cosine-variants --reps 15 --threads 16 > gpurun_out/r04u/cosine.log 2>&1
rc=$?; echo "cosine rc=$rc"; grep cosine_variant gpurun_out/r04u/cosine.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/bench_variants.py --only norms --clients 128 --reps 5 --interleave 3 > gpurun_out/r04u/norms.log 2>&1
rc=$?; echo "norms rc=$rc"; cut -c1-90 gpurun_out/r04u/norms.log | grep norms; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/bench_variant_paths.py --only fedatt,polaris,port_staged --reps 9 > gpurun_out/r04u/paths.log 2>&1
rc=$?; echo "paths rc=$rc"; cut -c1-110 gpurun_out/r04u/paths.log | grep path; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-inclusive --steps 5 --warmup 2 --variant-reps 9 > gpurun_out/r04u/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; python3 -c "
import json,sys
l=[x for x in open('gpurun_out/r04u/bench.log') if x.startswith('{')][-1]
v=json.loads(l)['variants']
print({k:(d['kernel_ms'],d.get('path_ms')) for k,d in v.items() if isinstance(d,dict)})"; exit $rc
