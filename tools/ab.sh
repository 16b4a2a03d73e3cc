#!/bin/bash
# A/B of library builds in one box session: rocprofv3 kernel averages of the workloads in $WLS (default
# c2_v1 c4_v1; tools/prof_run.py, OP=merge) for each library in $LIBS (paths relative to the repo), then
# one line per (library, workload, kernel) from tools/ab_summary.py.  Optional: PYTEST_K runs that
# selection of the GPU suite first (with the default library).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${TAG:-ab}
LIBS=${LIBS:-yjs_amd/libymerge.so}
WLS=${WLS:-c2_v1 c4_v1}
mkdir -p gpurun_out/$T
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$PYTEST_K" > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
  tail -2 gpurun_out/$T/pytest.log
fi
for lib in $LIBS; do
  b=$(basename $lib .so)
  for wl in $WLS; do
    YMERGE_LIB=$PWD/$lib WL=$wl timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/$b/$wl -o run -- python3 tools/prof_run.py ${STEPS:-30} > gpurun_out/$T/$b.$wl.log 2>&1 || { tail -20 gpurun_out/$T/$b.$wl.log; exit 1; }
  done
done
python3 tools/ab_summary.py gpurun_out/$T
