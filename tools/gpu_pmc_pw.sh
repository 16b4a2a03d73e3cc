#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) of the chunk-parallel walk kernels on one bench case.
# Usage: TAG=pw3 CASE=diff_c3_v1 [KERNELS="k_pw_walk k_pw_stitch"] bash tools/gpu_pmc_pw.sh
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-pwp}; CASE=${CASE:-diff_c3_v1}
D=gpurun_out/$TAG/$CASE
mkdir -p $D
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_INSTS_SMEM"; do
  i=$((i+1))
  CASE=$CASE timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $D/p$i -o run -- python3 tools/prof_big.py > $D/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $D/p$i.log; exit 1; }
done
for K in ${KERNELS:-k_pw_walk k_pw_stitch}; do echo "== $K"; KERNEL=$K python3 tools/summarize_pmc.py $D | tee $D/pmc_$K.txt; done
