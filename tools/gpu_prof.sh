#!/bin/bash
# Profiles of the headline kernel (C2 V1, 10 k docs, tools/prof_run.py): rocprofv3 kernel trace + stats,
# the PMC passes (tools/pmc_passes.sh) and, with STOPS set, the per-phase ablation counters.
# Usage: TAG=r02a [STOPS="1 8 2 3 4 7 5 0"] bash tools/gpu_prof.sh
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-prof}
mkdir -p gpurun_out/$TAG
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/trace -o run -- python3 tools/prof_run.py 20 > gpurun_out/$TAG/trace.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/$TAG/trace.log; exit 1; }
find gpurun_out/$TAG/trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/$TAG/c2_v1_kernel_stats.csv \;
head -5 gpurun_out/$TAG/c2_v1_kernel_stats.csv
TAG=$TAG/pmc bash tools/pmc_passes.sh || exit 1
if [ -n "$STOPS" ]; then bash tools/pmc_stops.sh > gpurun_out/$TAG/stops.txt 2>&1 || exit 1; fi
