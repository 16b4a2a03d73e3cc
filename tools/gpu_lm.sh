#!/bin/bash
# Large-document merge pipeline (ym_large.hip): its parity tests, the C5 / rich merge bench lines, and a
# rocprofv3 kernel trace of the C5 merges (the timeline shows the host round trips between kernels).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-lm}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_workloads.py tests/test_gpu_golden.py -x -v --timeout 300 --timeout-method thread -k "large or c5 or rich or merge" > gpurun_out/$TAG/pytest.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/$TAG/pytest.log | head; tail -5 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
YM_SECONDARY=${SEC:-merge_c5_v1,merge_c5_v2,merge_c2r_v1,merge_c4r_v2} timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
TAG=$TAG/prof CASES="merge_c5_v1 merge_c5_v2" bash tools/gpu_prof_pw.sh > gpurun_out/$TAG/prof.log 2>&1
echo done
