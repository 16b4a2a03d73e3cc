#!/bin/bash
# SQ / SQC counters of the streamed diff walkers (tools/prof_diff.py), one rocprofv3 --pmc pass each.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-pmc_diff}
mkdir -p gpurun_out/$TAG
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQC_DCACHE_HITS SQC_DCACHE_MISSES" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/$TAG/p$i -o run -- python3 tools/prof_diff.py 2 > gpurun_out/$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/$TAG/p$i.log; exit 1; }
done
python3 tools/summarize_pmc.py gpurun_out/$TAG > gpurun_out/$TAG/summary.txt && cat gpurun_out/$TAG/summary.txt
