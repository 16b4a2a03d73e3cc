#!/bin/bash
# Round-4: SQ counters of the C5 V1 chunk walk and stitch (diff, sv).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r04u}
mkdir -p gpurun_out/$TAG
FMTS=1 REPS=32 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_INSTS_VMEM --output-format csv -d gpurun_out/$TAG/pmc/p1 -o run -- python3 tools/prof_c5.py > gpurun_out/$TAG/pmc.log 2>&1 || { tail -20 gpurun_out/$TAG/pmc.log; exit 1; }
for k in "k_pw_stitch<1>" "k_pw_stitch<2>" k_pw_walk; do echo "== $k"; KERNEL="$k" python3 tools/summarize_pmc.py gpurun_out/$TAG/pmc; done | tee gpurun_out/$TAG/pmc_summary.txt
FMTS=1 REPS=32 timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/$TAG/pmc/p2 -o run -- python3 tools/prof_c5.py > gpurun_out/$TAG/pmc2.log 2>&1 || { tail -20 gpurun_out/$TAG/pmc2.log; exit 1; }
for k in "k_pw_stitch<1>" "k_pw_stitch<2>" k_pw_walk; do echo "== $k"; KERNEL="$k" python3 tools/summarize_pmc.py gpurun_out/$TAG/pmc; done | tee gpurun_out/$TAG/pmc_summary.txt
