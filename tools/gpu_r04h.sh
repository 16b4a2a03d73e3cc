#!/bin/bash
# Round-4 kernel traces of the small-document V1 diff / sv / meta path (C2, 10 k merged documents).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r04h}
mkdir -p gpurun_out/$TAG
for op in ${OPS:-diff sv meta}; do
  OP=$op timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/$op -o run -- python3 tools/prof_run.py 10 > gpurun_out/$TAG/$op.log 2>&1 || { echo "$op failed"; tail -5 gpurun_out/$TAG/$op.log; exit 1; }
  find gpurun_out/$TAG/$op -name "*kernel_stats.csv" -exec cp {} gpurun_out/$TAG/c2_v1_${op}_kernel_stats.csv \;
  echo "== $op"; cut -d, -f1-8 gpurun_out/$TAG/c2_v1_${op}_kernel_stats.csv | head -8
done
