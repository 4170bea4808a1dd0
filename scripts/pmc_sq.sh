#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run per pass, each under its own time
# limit) over a benchmark command: where a kernel's wave-cycles go (waiting on
# memory/barriers, issue stalls, LDS bank conflicts, instruction mix).
# Usage: bash scripts/pmc_sq.sh <tag> <command...>   (results in gpurun_out/pmc_<tag>/)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d $OUT/p$i -o p$i -- "$@" > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
exit 0
