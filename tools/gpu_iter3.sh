#!/bin/bash
# Iteration run: chunk-walk / stitch parity (C3, C5, golden), rich-content parity, C5 V1 stitch phase ticks
# (prof build), bench lines of the touched paths.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-it3}
mkdir -p gpurun_out/$TAG
[ -n "$NOTEST" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_workloads.py tests/test_gpu_golden.py -x -v --timeout 300 --timeout-method thread -k "c3 or c5 or chunked or client_map or pref or rich or merge_workload" > gpurun_out/$TAG/pytest.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/$TAG/pytest.log | head; tail -5 gpurun_out/$TAG/pytest.log; exit 1; }
[ -n "$NOTEST" ] || tail -1 gpurun_out/$TAG/pytest.log
FMTS=1 timeout -k 10 300 python -u tools/prof_c5.py > gpurun_out/$TAG/c5_v1.log 2>&1
YMLIB=yjs_amd/libymerge_prof.so REPS=8 FMTS=1 timeout -k 10 300 python -u tools/prof_c5.py > gpurun_out/$TAG/c5_v1_ticks.log 2>&1
YM_SECONDARY=${SEC:-diff_c3_v1,sv_c3_v1,diff_c5_v1,merge_c2r_v1,merge_c4r_v1,merge_c5_v1,merge_c4_v1} timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
echo done
