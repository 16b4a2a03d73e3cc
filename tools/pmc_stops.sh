#!/bin/bash
# SQ instruction counters of the fast-path kernel per ablation stop (where the VALU/SALU go).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_stops
for stop in ${STOPS:-1 2 3 4 5 0}; do
  YMERGE_FAST_STOP=$stop timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_stops/s$stop -o run -- python3 tools/prof_run.py 3 > gpurun_out/pmc_stops/s$stop.log 2>&1 || { echo "stop $stop failed"; tail -5 gpurun_out/pmc_stops/s$stop.log; exit 1; }
  echo "== stop $stop"; mkdir -p gpurun_out/pmc_stops/t$stop; mv gpurun_out/pmc_stops/s$stop gpurun_out/pmc_stops/t$stop/p1
  python3 tools/summarize_pmc.py gpurun_out/pmc_stops/t$stop
done
