#!/bin/bash
# rocprofv3 kernel averages of the V1 merge kernel on C2 / C4 (tools/prof_run.py), for A/B builds.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${TAG:-r04ab}
mkdir -p gpurun_out/$T
for wl in c2_v1 c4_v1; do
  WL=$wl timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/$wl -o run -- python3 tools/prof_run.py 30 > gpurun_out/$T/$wl.log 2>&1 || exit 1
done
