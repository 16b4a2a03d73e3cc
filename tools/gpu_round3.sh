#!/bin/bash
# Round-3 GPU evidence in one call: full GPU parity, smoke, the default bench (headline + secondaries),
# rocprofv3 kernel stats + PMC passes of the headline kernel, kernel stats of the C3 diff / sv cases.
# Every GPU step has its own limit; the script stops at the first failure.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r03b}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1
tail -2 gpurun_out/$TAG/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1
tail -1 gpurun_out/$TAG/smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
TAG=$TAG/c2 bash tools/gpu_prof.sh > gpurun_out/$TAG/prof_c2.log 2>&1
[ -n "$DIFFPROF" ] && TAG=$TAG/diff CASES="$DIFFPROF" bash tools/gpu_prof_pw.sh > gpurun_out/$TAG/prof_diff.log 2>&1
echo done
