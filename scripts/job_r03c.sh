#!/bin/bash
# rocprofv3 of the fused FedAdp kernel: kernel trace, then PMC passes (each its own run)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_r03c
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/scripts/bench_variant_paths.py --fedadp-only --reps 3"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- $B > $O/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; tail -2 $O/kt.log; [ $rc -ne 0 ] && exit $rc
i=0
for P in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/pmc$i -o pmc -- $B > $O/pmc$i.log 2>&1
  rc=$?; echo "pmc$i ($P) rc=$rc"; tail -1 $O/pmc$i.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
