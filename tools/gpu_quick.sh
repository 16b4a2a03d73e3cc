#!/bin/bash
# Quick GPU iteration: merge parity on the workloads, then the phase ablation (stops at the first failure).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_workloads.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread -k "merge" > gpurun_out/pytest_quick.log 2>&1 || { tail -30 gpurun_out/pytest_quick.log; exit 1; }
tail -3 gpurun_out/pytest_quick.log
for wl in ${WLS:-c2_v1}; do
  WL=$wl timeout -k 10 240 python tools/ablate_fast.py > gpurun_out/ablate_$wl.txt 2>&1 || { cat gpurun_out/ablate_$wl.txt; exit 1; }
  echo "== $wl"; cat gpurun_out/ablate_$wl.txt
done
