#!/bin/bash
# round-3 final check: full GPU suite, smoke, same-lease bench + rocprof passes, 2-rank gloo rehearsal of --gpus 2
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r03zb_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03zb_pytest_gpu.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03zb_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r03zb_smoke.log
[ $rc -ne 0 ] && exit $rc
bash scripts/profile.sh r03zb
rc=$?; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r03zb_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/r03zb_bench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 env PLATO_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/r03zb_bench_dist2_gloo.log 2>&1
rc=$?; echo "dist2 rc=$rc"; tail -c 400 gpurun_out/r03zb_bench_dist2_gloo.log
exit $rc
