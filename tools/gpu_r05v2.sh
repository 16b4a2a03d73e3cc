#!/bin/bash
# V2 small-document checks: the V2 parity selection, decline outcomes, then timings.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=${TAG:-r05v2}; mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-v2 or diff or golden or async or sv}" > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
for w in c2_v2 c2r_v2 c4r_v2; do OP=diff WL=$w timeout -k 10 120 python3 tools/pv2_reasons.py 2>&1 | tail -1; done
YM_SECONDARY=${SEC:-diff_c2_v2,diff_c2r_v2,diff_c4r_v2,sv_c2_v2,diff_c3_v2,diff_c5_v2,meta_c3_v2,sv_c3_v2} timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
python3 -c "
import json; l=[json.loads(x) for x in open('gpurun_out/$T/bench.json') if x.startswith('{')][-1]
for k,v in l['secondary'].items(): print(k, v.get('ms_per_step', v), v.get('docs_general'))"
