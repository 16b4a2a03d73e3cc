#!/bin/bash
# Rich-content workloads (C2R / C4R): parity of the merges against the oracle, then the bench lines.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-rich}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_gpu_workloads.py -x -q --timeout 300 --timeout-method thread -k "merge_workload or rich_content" > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
YM_SECONDARY=merge_c2r_v1,merge_c2r_v2,merge_c4r_v1,merge_c4r_v2,diff_c2r_v1,diff_c2r_v2,sv_c4r_v1,diff_c4r_v2,merge_c2_v2 timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
echo done
