#!/bin/bash
# rocprofv3 kernel averages of $KERNEL over tools/prof_run.py (WL / OP from the environment) under each value
# of the environment variable $VAR in $VALS.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=${TAG:-ksweep}; mkdir -p gpurun_out/$T
for v in $VALS; do
  env $VAR=$v timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/$v -o run -- python3 tools/prof_run.py ${STEPS:-5} > gpurun_out/$T/$v.log 2>&1 || { tail -5 gpurun_out/$T/$v.log; exit 1; }
  python3 - gpurun_out/$T/$v "$VAR=$v" "$KERNEL" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if sys.argv[3] in r["Name"]:
        print(sys.argv[2], f"{float(r['AverageNs'])/1e3:9.1f} us  x{r['Calls']}  {r['Name'][:90]}")
PY
done
