#!/bin/bash
# Round-4: the V2 merge kernel (C2 V2, 10 k documents): kernel trace and SQ counters.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r04o}
mkdir -p gpurun_out/$TAG
WL=c2_v2 timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/tr -o run -- python3 tools/prof_run.py 10 > gpurun_out/$TAG/tr.log 2>&1 || { tail -5 gpurun_out/$TAG/tr.log; exit 1; }
find gpurun_out/$TAG/tr -name "*kernel_stats.csv" -exec cp {} gpurun_out/$TAG/c2_v2_kernel_stats.csv \;
awk -F'"' 'NR>1{print $2, $NF}' gpurun_out/$TAG/c2_v2_kernel_stats.csv | sed 's/(ymk::GeneralJob[^)]*)//' | cut -c1-150 | head -6
WL=c2_v2 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_INSTS_VMEM --output-format csv -d gpurun_out/$TAG/pmc/p1 -o run -- python3 tools/prof_run.py 3 > gpurun_out/$TAG/pmc.log 2>&1 || { tail -5 gpurun_out/$TAG/pmc.log; exit 1; }
KERNEL=k_fast_merge_v2 python3 tools/summarize_pmc.py gpurun_out/$TAG/pmc | tee gpurun_out/$TAG/pmc_summary.txt
