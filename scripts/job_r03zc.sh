#!/bin/bash
# end of round 3: FedAdp variant timings + HBM/L2 counters, then the full GPU suite, smoke, bench
set -u
R=$GRAFT_REPO_ROOT
bash scripts/job_r03za.sh || exit $?
bash scripts/job_r03zb.sh
