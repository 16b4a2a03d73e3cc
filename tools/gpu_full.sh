#!/bin/bash
# Full GPU parity suite + smoke + selected bench lines (YM_SECONDARY) in one call.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-full}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/$TAG/pytest_gpu.log | head -20; tail -5 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1
tail -1 gpurun_out/$TAG/smoke.log
if [ -n "$SEC" ]; then
  YM_SECONDARY=$SEC timeout -k 10 500 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
fi
echo done
