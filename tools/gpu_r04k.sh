#!/bin/bash
# Round-4: small-document V1 diff / sv (C2, 10 k merged documents): kernel traces and SQ counters of k_pw_small.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r04k}
mkdir -p gpurun_out/$TAG
for op in ${OPS:-diff sv}; do
  OP=$op timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/$op -o run -- python3 tools/prof_run.py 10 > gpurun_out/$TAG/$op.log 2>&1 || { echo "$op failed"; tail -5 gpurun_out/$TAG/$op.log; exit 1; }
  find gpurun_out/$TAG/$op -name "*kernel_stats.csv" -exec cp {} gpurun_out/$TAG/c2_v1_${op}_kernel_stats.csv \;
  echo "== $op"; cut -d, -f1-4 gpurun_out/$TAG/c2_v1_${op}_kernel_stats.csv | sed 's/(ymk::[^"]*//' | head -6
  OP=$op timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_INSTS_VMEM --output-format csv -d gpurun_out/$TAG/${op}pmc/p1 -o run -- python3 tools/prof_run.py 3 > gpurun_out/$TAG/${op}pmc.log 2>&1 || { echo "$op pmc failed"; tail -5 gpurun_out/$TAG/${op}pmc.log; exit 1; }
  KERNEL=k_pw_small python3 tools/summarize_pmc.py gpurun_out/$TAG/${op}pmc | tee gpurun_out/$TAG/${op}_pmc_summary.txt
done
