#!/bin/bash
# round 4 close (final): the whole GPU suite, smoke and the default bench on the final build
set -u
mkdir -p gpurun_out/r04zn
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/r04zn/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r04zn/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04zn/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r04zn/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r04zn/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; python3 -c "
import json
l=[x for x in open('gpurun_out/r04zn/bench.log') if x.startswith('{')][-1]
b=json.loads(l)
print(b['value'], b['ms_per_step'], b['roofline']['frac'], b['roofline']['traffic_source'])
print({k:(d['kernel_ms'],d.get('path_ms'),d['frac_of_floor']) for k,d in b['variants'].items() if isinstance(d,dict)})"; exit $rc
