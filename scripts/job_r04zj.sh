#!/bin/bash
# round 4: fedavg_entrywise (FedAdp global gradient, FedAtt sum) at chunk sizes 1,024 (the engine's) to 8,192
set -u
mkdir -p gpurun_out/r04zj
timeout -k 10 300 python -u scripts/bench_variants.py --only entrywise,fedavg --ew-chunks 2048,4096,8192 --reps 5 --interleave 4 > gpurun_out/r04zj/ew.log 2>&1
rc=$?; echo "ew rc=$rc"; grep kernel gpurun_out/r04zj/ew.log | cut -c1-100; exit $rc
