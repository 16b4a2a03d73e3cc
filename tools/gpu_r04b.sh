#!/bin/bash
# Round-4 iteration: parity of the block-parallel rest walk (ym_pv2ms.hip) and the lane-per-document small-update
# kernel (ym_small.hip), then C5 V2 timings.  Every GPU step has its own limit; stops at the first failure.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r04b}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_workloads.py -x -v --timeout 200 --timeout-method thread -k "golden or c5_sv or sv_and_diff or meta or client_map or c3 or rich or state_does" > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest.log
FMTS=2 REPS=32 timeout -k 10 300 python -u tools/prof_c5.py > gpurun_out/$TAG/c5v2.log 2>&1 || { tail -20 gpurun_out/$TAG/c5v2.log; exit 1; }
grep -v Warn gpurun_out/$TAG/c5v2.log | head -20
