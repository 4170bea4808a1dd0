#!/bin/bash
# FedAdp fused-dots variants + probes, sdot_shared variants, and a kernel trace of the fedadp paths
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/bench_variant_paths.py --fedadp-kernel --sdot --reps 5 > gpurun_out/r03h_paths.log 2>&1
rc=$?; echo "paths rc=$rc"; cat gpurun_out/r03h_paths.log | grep -v amdgpu.ids
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r03h -o kt -- python3 $GRAFT_REPO_ROOT/scripts/bench_variant_paths.py --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/r03h_kt.log 2>&1
rc=$?; echo "kt rc=$rc"
exit $rc
