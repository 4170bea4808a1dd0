#!/bin/bash
# round 4, first lease: FedAdp gather alignment probe + variant 60 check
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/fedadp_align_probe.py --reps 10 --variants 51,60 > gpurun_out/r04a_align.log 2>&1
rc=$?; echo "probe rc=$rc"; cat gpurun_out/r04a_align.log | tail -20; [ $rc -eq 0 ] || exit $rc
