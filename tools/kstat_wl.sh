#!/bin/bash
# rocprofv3 kernel statistics (top kernels) of tools/prof_run.py for each workload in $WLS (OP from the env).
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=${TAG:-kwl}; mkdir -p gpurun_out/$T
for w in $WLS; do
  WL=$w timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/$w -o run -- python3 tools/prof_run.py ${STEPS:-5} > gpurun_out/$T/$w.log 2>&1 || { tail -5 gpurun_out/$T/$w.log; exit 1; }
  python3 - gpurun_out/$T/$w "$w" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:int(__import__("os").environ.get("TOPK", "8"))]:
    if "ymk" in r["Name"] or "anonymous" in r["Name"]:
        print(sys.argv[2], f"{float(r['AverageNs'])/1e3:9.1f} us  x{r['Calls']}  {r['Name'][:100]}")
PY
done
