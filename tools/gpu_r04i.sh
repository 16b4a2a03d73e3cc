#!/bin/bash
# Round-4: C5 diff / sv kernel traces and SQ counters of the multi-section walks, then the small-document
# traces (tools/gpu_r04h.sh).  Each GPU step has its own limit; stops at the first failure.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r04i}
mkdir -p gpurun_out/$TAG
FMTS=${FMTS:-2,1} REPS=32 timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/c5 -o run -- python3 tools/prof_c5.py > gpurun_out/$TAG/c5.log 2>&1 || { tail -20 gpurun_out/$TAG/c5.log; exit 1; }
grep -v -i warn gpurun_out/$TAG/c5.log | grep -v "ga = torch" | head -30
find gpurun_out/$TAG/c5 -name "*kernel_stats.csv" -exec cp {} gpurun_out/$TAG/c5_kernel_stats.csv \;
cut -d, -f1-4 gpurun_out/$TAG/c5_kernel_stats.csv | head -14
FMTS=${FMTS:-2,1} REPS=32 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_INSTS_SMEM --output-format csv -d gpurun_out/$TAG/c5pmc/p1 -o run -- python3 tools/prof_c5.py > gpurun_out/$TAG/c5pmc.log 2>&1 || { tail -20 gpurun_out/$TAG/c5pmc.log; exit 1; }
for k in k_ms_walk k_ms_rest k_pw_ms k_ms_out; do echo "== $k"; KERNEL=$k python3 tools/summarize_pmc.py gpurun_out/$TAG/c5pmc; done > gpurun_out/$TAG/c5pmc_summary.txt 2>&1 || true
cat gpurun_out/$TAG/c5pmc_summary.txt
if [ -n "$SMALL" ]; then TAG=$TAG/small bash tools/gpu_r04h.sh; fi
