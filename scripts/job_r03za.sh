#!/bin/bash
# FedAdp: HBM read bytes and L2 hit rate per variant (own --pmc pass each)
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_r03za
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread $R/tests/test_per_entry_gpu.py -k "tile_shapes or fedadp_server" > $R/gpurun_out/r03za_pytest.log 2>&1 || exit $?
timeout -k 10 300 python3 -u $R/scripts/bench_variant_paths.py --fedadp-only --reps 10 > $R/gpurun_out/r03za_fedadp.log 2>&1 || exit $?
i=0
for p in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d $OUT/p$i -o p$i -- python3 $R/scripts/bench_variant_paths.py --fedadp-only --reps 1 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
