set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r05s
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sv or golden or meta or v2" > gpurun_out/r05s/pytest.log 2>&1 || { tail -30 gpurun_out/r05s/pytest.log; exit 1; }
tail -2 gpurun_out/r05s/pytest.log
YM_SECONDARY=sv_c2_v2,sv_c3_v2,meta_c2_v2,meta_c3_v2,sv_c2_v1,diff_c2_v2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-baseline-seconds 0.5 > gpurun_out/r05s/bench.log 2>&1 || { tail -20 gpurun_out/r05s/bench.log; exit 1; }
python3 -c "
import json; l=[json.loads(x) for x in open('gpurun_out/r05s/bench.log') if x.startswith('{')][-1]
for k,v in l['secondary'].items(): print(k, v.get('ms_per_call', v))"
