#!/bin/bash
# PMC passes over tools/prof_run.py (one rocprofv3 --pmc run per counter group).  Usage:
#   TAG=name [YMERGE_FAST_STOP=n] bash tools/pmc_passes.sh
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-pmc}
mkdir -p gpurun_out/$TAG
i=0
# PMC_GROUPS (optional): ';'-separated counter groups replacing the default passes below
if [ -n "$PMC_GROUPS" ]; then IFS=';' read -ra GRPS <<< "$PMC_GROUPS"; else GRPS=(); fi
[ ${#GRPS[@]} -gt 0 ] || GRPS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH" \
           "SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_IFETCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_PMC})
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/$TAG/p$i -o run -- python3 ${RUNNER:-tools/prof_run.py} 5 > gpurun_out/$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/$TAG/p$i.log; exit 1; }
done
python3 tools/summarize_pmc.py gpurun_out/$TAG > gpurun_out/$TAG/summary.txt && cat gpurun_out/$TAG/summary.txt
