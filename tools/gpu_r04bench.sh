#!/bin/bash
# Round-4 final: the default bench line, and the rocprofv3 kernel statistics of the same command's
# headline (C2 V1, asynchronous submission) for the roofline's launch-duration check.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r04bench}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python3 bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o run -- python3 bench.py --no-secondary --no-cpu-baseline > gpurun_out/$TAG/prof_bench.json 2> gpurun_out/$TAG/prof.err
find gpurun_out/$TAG/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/$TAG/c2_v1_kernel_stats.csv \;
