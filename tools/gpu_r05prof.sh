#!/bin/bash
# Round-5 profile set of the headline kernel (C2 V1 merge, 10 k documents): the default bench line and its
# rocprofv3 kernel statistics, the PMC passes, the per-phase instruction counts (ablation stops) and the
# per-wave timeline (YM_FAST_TIMELINE build).  Every GPU step under its own limit; the first failure ends it.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=${TAG:-r05prof}; mkdir -p gpurun_out/$T
TAG=$T/bench bash tools/gpu_r04bench.sh
echo bench done
TAG=$T/pmc bash tools/pmc_passes.sh > gpurun_out/$T/pmc.txt 2>&1 || { tail -5 gpurun_out/$T/pmc.txt; exit 1; }
echo pmc done
STOPS="${STOPS:-1 8 3 4 7 2 5 0}" bash tools/pmc_stops.sh > gpurun_out/$T/stops.txt 2>&1 || { tail -5 gpurun_out/$T/stops.txt; exit 1; }
echo stops done
YMERGE_LIB=$PWD/yjs_amd/libymerge_tl.so timeout -k 10 120 python3 tools/fast_timeline.py > gpurun_out/$T/timeline.txt 2>&1 || { tail -5 gpurun_out/$T/timeline.txt; exit 1; }
head -3 gpurun_out/$T/timeline.txt
