#!/bin/bash
# Rich-content V1 checks: parity selection, k_pw_small outcomes, timings.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=${TAG:-r05rich}; mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-golden or canon or rich or nested or workload}" > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
OP=diff WL=c2r_v1 timeout -k 10 120 python3 tools/pw_reasons.py 2>&1 | tail -1
OP=sv WL=c4r_v1 timeout -k 10 120 python3 tools/pw_reasons.py 2>&1 | tail -1
YM_SECONDARY=${SEC:-diff_c2r_v1,sv_c4r_v1,diff_c2_v1,sv_c2_v1,meta_c2_v1,diff_c3_v1,sv_c3_v1} timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
python3 -c "
import json; l=[json.loads(x) for x in open('gpurun_out/$T/bench.json') if x.startswith('{')][-1]
for k,v in l['secondary'].items(): print(k, v.get('ms_per_step', v), v.get('docs_general'))"
