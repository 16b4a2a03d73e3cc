#!/bin/bash
# Round-5 final checks: the whole GPU suite in one process + smoke, then the default bench line.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=${TAG:-r05final}; mkdir -p gpurun_out/$T
TAG=$T bash tools/gpu_tests.sh
timeout -k 10 400 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
python3 -c "
import json; l=[json.loads(x) for x in open('gpurun_out/$T/bench.json') if x.startswith('{')][-1]
print('headline', l['value'], l['ms_per_step'], l['roofline']['avg_launch_ms'], l['roofline']['frac'], l['cpu_baseline']['value'])
for k,v in l['secondary'].items(): print(k, v.get('ms_per_step', v), v.get('docs_general'))"
