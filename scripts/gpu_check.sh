#!/bin/bash
# GPU-box job: parity tests, kernel-variant sweep, bench line.
# Each GPU step has its own time limit; a fault / abort / timeout ends the job
# (exit codes >= 124), while an ordinary test failure (1) still lets the
# measurement steps run so the log shows both.
set -u
mkdir -p gpurun_out
run() {  # run <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $name; stopping"; exit $rc; fi
  return 0
}
# libraries are built in-tree before the call (never on the GPU box)
for f in plato_amd/libplato_agg.so plato_amd/libplato_ingest.so; do [ -f $f ] || { echo "missing $f"; exit 1; }; done
for step in "$@"; do
  case $step in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    sweep) run sweep 600 python bench.py --sweep --steps 10 --no-cpu-baseline --no-host-inclusive ;;
    bench) run bench 900 python bench.py ;;
    dist2) run bench_dist2 600 env PLATO_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 ;;
    dist2c3) run bench_dist2_c3 600 env PLATO_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --config C3 --clients 256 --steps 5 --warmup 2 ;;
    multi1) run bench_multi1 600 python bench.py --engine-devices 1 --steps 3 --warmup 1 ;;
    multi4) run bench_multi4 600 python bench.py --engine-devices 4 --steps 3 --warmup 1 ;;
    profile) run profile 900 bash scripts/profile.sh ${PROFILE_TAG:-r02} ;;
    bf16) run bench_bf16 600 python bench.py --codec bf16 --steps 20 ;;
    bf16sweep) run sweep_bf16 600 python bench.py --codec bf16 --sweep --steps 10 ;;
    variants) run bench_variants 600 python scripts/bench_variants.py ;;
    configs) for c in C1 C3 C4 C5 C5-gpt2; do run bench_$c 600 python bench.py --config $c --steps 10 --warmup 3; done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
