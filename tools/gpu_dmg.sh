#!/bin/bash
# Damaged-update parity (truncations / byte flips of C3) in one process; NOPW=1 disables the chunk /
# column paths (the sequential walkers and the general path alone).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -n "$NOPW" ]; then export YMERGE_NO_PW=1; fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_workloads.py -x -v --timeout 200 --timeout-method thread \
  -k "damaged" > gpurun_out/pytest_dmg.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/pytest_dmg.log | tail -8
exit $rc
