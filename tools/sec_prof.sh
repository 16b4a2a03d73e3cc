#!/bin/bash
# Secondary bench lines ($SEC, comma-separated case names of bench.py secondary()) with the library
# $LIB (default: the in-tree one), then the same command under rocprofv3 --kernel-trace --stats.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${TAG:-sec}
mkdir -p gpurun_out/$T
[ -n "$LIB" ] && export YMERGE_LIB=$PWD/$LIB
YM_SECONDARY="$SEC" timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
python3 - gpurun_out/$T/bench.json <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k, v in r.get("secondary", {}).items():
    print(f"{k:22s} " + json.dumps({x: v[x] for x in v if x in ('ms_per_step', 'kernel_ms', 'docs_fast', 'docs_large', 'docs_general', 'error')} if isinstance(v, dict) else v))
PY
if [ -n "$PROF" ]; then
  YM_SECONDARY="$SEC" timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  python3 - gpurun_out/$T/prof <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms  x{int(r['Calls']):5d}  {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:110]}")
PY
fi
