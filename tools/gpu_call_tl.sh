#!/bin/bash
# One call's kernel timeline (tools/call_timeline.py) of OP over WL (tools/prof_run.py), rocprofv3 kernel trace.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${TAG:-ctl}
mkdir -p gpurun_out/$T
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/$OP.$WL -o run -- python3 tools/prof_run.py ${STEPS:-3} > gpurun_out/$T/$OP.$WL.log 2>&1 || { tail -5 gpurun_out/$T/$OP.$WL.log; exit 1; }
python3 tools/call_timeline.py $(find gpurun_out/$T/$OP.$WL -name "*kernel_trace.csv") ${K:-16}
