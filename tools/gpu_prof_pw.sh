#!/bin/bash
# rocprofv3 kernel stats of the chunk-parallel V1 walk (k_pw_walk, k_pw_stitch) on the bench's diff / sv
# secondary cases.  Usage: TAG=r02g [CASES="diff_c3_v1 sv_c3_v1 diff_c5_v1"] bash tools/gpu_prof_pw.sh
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-pw}
for CASE in ${CASES:-diff_c3_v1 sv_c3_v1 diff_c5_v1}; do
  D=gpurun_out/$TAG/$CASE
  mkdir -p $D
  CASE=$CASE timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 tools/prof_big.py > $D/trace.log 2>&1 || { echo "$CASE trace failed"; tail -5 $D/trace.log; exit 1; }
  find $D/trace -name "*kernel_stats.csv" -exec cp {} $D/kernel_stats.csv \;
  echo "== $CASE"; head -8 $D/kernel_stats.csv | cut -d, -f1-8
done
