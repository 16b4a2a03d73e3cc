#!/bin/bash
# Round-5 scratch run: a GPU test selection (PYTEST_K / PYTEST_FILES), then the secondary bench lines named
# in YM_SECONDARY (default: the small-document sync-server lines).
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=${TAG:-r05s}; mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
[ -n "$NO_BENCH" ] && exit 0
YM_SECONDARY=${YM_SECONDARY:-sv_c2_v2,diff_c2_v2,sv_c2_v1,diff_c2_v1} timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-baseline-seconds 0.5 > gpurun_out/$T/bench.log 2>&1 || { tail -20 gpurun_out/$T/bench.log; exit 1; }
python3 -c "
import json; l=[json.loads(x) for x in open('gpurun_out/$T/bench.log') if x.startswith('{')][-1]
print('headline', l['value'], l['roofline']['avg_launch_ms'])
for k,v in l['secondary'].items(): print(k, v.get('ms_per_step', v), v.get('docs_general'))"
