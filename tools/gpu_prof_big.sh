#!/bin/bash
# rocprofv3 kernel stats + PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) of the diff / state-vector kernels on
# the bench's C3 / C5 secondary cases.  Usage: TAG=r02c [CASES="diff_c3_v1 diff_c3_v2 diff_c5_v1 diff_c5_v2"] bash tools/gpu_prof_big.sh
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-big}
for CASE in ${CASES:-diff_c3_v1 diff_c3_v2 diff_c5_v1 diff_c5_v2}; do
  D=gpurun_out/$TAG/$CASE
  mkdir -p $D
  case $CASE in *v2) K=k_big_v2;; *) K=k_big_v1;; esac
  CASE=$CASE timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 tools/prof_big.py > $D/trace.log 2>&1 || { echo "$CASE trace failed"; tail -5 $D/trace.log; exit 1; }
  find $D/trace -name "*kernel_stats.csv" -exec cp {} $D/kernel_stats.csv \;
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    CASE=$CASE timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $D/p$i -o run -- python3 tools/prof_big.py > $D/p$i.log 2>&1 || { echo "$CASE pass $i failed"; tail -5 $D/p$i.log; exit 1; }
  done
  KERNEL=$K python3 tools/summarize_pmc.py $D > $D/pmc_summary.txt
  echo "== $CASE ($K)"; head -3 $D/kernel_stats.csv | cut -c1-200; cat $D/pmc_summary.txt
done
