#!/bin/bash
# One GPU-box job (replaces the per-session job_r0*.sh files):
#   scripts/gpu_job.sh <tag> <step> [<step> ...]
# Logs go to gpurun_out/<tag>/<step>.log.  Every step runs under its own time limit and the job stops
# at the first failing step (never a retry, never another GPU step after a fault / abort / timeout).
# Steps:
#   pytest             the whole -m gpu suite
#   pytest=<expr>      the -m gpu tests matching -k <expr>
#   smoke              __graft_entry__.smoke()
#   bench              the driver's default bench line
#   bench=<args>       bench.py <args> (spaces as '+', e.g. bench=--config+C3+--steps+10)
#   anchor             bench.py --anchor (one rank's piece kernels at N = 1, 2, 4, 8; grid-tail shapes)
#   sweep              bench.py --sweep (headline kernel variants, interleaved)
#   variants           scripts/bench_variants.py (variant-server kernels)
#   profile            scripts/profile.sh <tag>: unprofiled bench + kernel trace + FETCH_SIZE + WRITE_SIZE passes
#   profile_variants   scripts/profile_variants.sh <tag>
#   pmc=<counters>@<script+args>   one rocprofv3 --pmc pass (comma-separated counters) over python3 <script> <args>
#                      (default script: scripts/bench_variants.py --reps 3)
#   kt=<script+args>   rocprofv3 --kernel-trace --stats over python3 <script> <args>
#   py=<script+args>   python <script> <args> (spaces as '+')
# Libraries are built in-tree before the call (never on the GPU box).
set -u
tag=$1
shift
out=gpurun_out/$tag
mkdir -p "$out"
for f in plato_amd/libplato_agg.so plato_amd/libplato_agg_tune.so plato_amd/libplato_ingest.so; do
  [ -f "$f" ] || { echo "missing $f (build first)"; exit 1; }
done

run() {  # run <log name> <timeout s> <cmd...>
  local name=$1 t=$2
  shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -4 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}

n=0
for step in "$@"; do
  n=$((n + 1))
  arg=${step#*=}
  args=${arg//+/ }
  case $step in
    pytest) run pytest 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ ;;
    pytest=*) run pytest_$n 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ -k "$args" ;;
    smoke) run smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 300 python -u bench.py ;;
    bench=*) run bench_$n 600 python -u bench.py $args ;;
    anchor) run anchor 600 python -u bench.py --anchor --steps 10 ;;
    sweep) run sweep 600 python -u bench.py --sweep --steps 10 --no-cpu-baseline --no-host-inclusive ;;
    variants) run variants 600 python -u scripts/bench_variants.py ;;
    profile) run profile 900 bash scripts/profile.sh "$tag" ;;
    profile_variants) run profile_variants 900 bash scripts/profile_variants.sh "$tag" ;;
    pmc=*) ctrs=${arg%%@*}
           prog="scripts/bench_variants.py --reps 3"
           [ "$ctrs" != "$arg" ] && prog=${arg#*@} && prog=${prog//+/ }
           set -- $prog
           script=$1; shift
           (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc ${ctrs//,/ } --output-format csv \
              -d "$GRAFT_REPO_ROOT/$out/pmc_$n" -o pmc -- python3 "$GRAFT_REPO_ROOT/$script" "$@") \
             > "$out/pmc_$n.log" 2>&1 || { rc=$?; echo "pmc pass $n rc=$rc"; tail -4 "$out/pmc_$n.log"; exit $rc; }
           echo "=== pmc_$n ok ($ctrs over $script $*)" ;;
    kt=*) set -- $args
          script=$1; shift
          (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$GRAFT_REPO_ROOT/$out/kt_$n" -o kt -- python3 "$GRAFT_REPO_ROOT/$script" "$@") \
            > "$out/kt_$n.log" 2>&1 || { rc=$?; echo "kernel trace $n rc=$rc"; tail -4 "$out/kt_$n.log"; exit $rc; }
          echo "=== kt_$n ok (kernel trace of $script $*)" ;;
    py=*) run py_$n 600 python -u $args ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
