#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/ingest_probe.py > gpurun_out/r03s_ingest.log 2>&1
rc=$?; echo "probe rc=$rc"; grep -v amdgpu.ids gpurun_out/r03s_ingest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r03s_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"host_inclusive".*' gpurun_out/r03s_bench.log | cut -c1-700
exit $rc
