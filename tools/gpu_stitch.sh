#!/bin/bash
# The V1 chunk walk / stitch: its parity tests, C5 diff / sv timings (tools/prof_c5.py), C3 / C5 bench lines.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-stitch}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_workloads.py tests/test_gpu_golden.py -x -v --timeout 300 --timeout-method thread -k "c3 or c5 or chunked or client_map or pref" > gpurun_out/$TAG/pytest.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/$TAG/pytest.log | head; tail -5 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
FMTS=1 timeout -k 10 300 python -u tools/prof_c5.py > gpurun_out/$TAG/c5_v1.log 2>&1
YMLIB=yjs_amd/libymerge_prof.so REPS=8 FMTS=1 timeout -k 10 300 python -u tools/prof_c5.py > gpurun_out/$TAG/c5_v1_ticks.log 2>&1
YM_SECONDARY=diff_c3_v1,sv_c3_v1,meta_c3_v1,diff_c5_v1 timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
echo done
