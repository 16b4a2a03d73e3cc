#!/bin/bash
# One box session for a round's record: the default bench line (with secondaries), the same command's
# headline under rocprofv3 --kernel-trace --stats, the PMC passes of the headline kernel, then the GPU
# parity suite and smoke().  Every GPU step under its own limit; the first failure ends the script.
# Usage: TAG=r06a [SKIP_TESTS=1] [SKIP_PMC=1] bash tools/gpu_round.sh
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${TAG:-round}
mkdir -p gpurun_out/$T
timeout -k 10 420 python3 -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
tail -c 600 gpurun_out/$T/bench.json; echo
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/trace -o run -- python3 bench.py --no-secondary --no-cpu-baseline > gpurun_out/$T/bench_prof.json 2> gpurun_out/$T/bench_prof.err || { echo "rocprof failed"; tail -5 gpurun_out/$T/bench_prof.err; exit 1; }
find gpurun_out/$T/trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/$T/c2_v1_bench_kernel_stats.csv \;
head -4 gpurun_out/$T/c2_v1_bench_kernel_stats.csv
if [ -z "$SKIP_PMC" ]; then TAG=$T/pmc bash tools/pmc_passes.sh > /dev/null || exit 1; cat gpurun_out/$T/pmc/summary.txt | head -30; fi
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$T/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/$T/pytest_gpu.log
  timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1
  tail -1 gpurun_out/$T/smoke.log
fi
