#!/bin/bash
# Round-4: kernel stats of the C5 V2 diff / sv (block-parallel rest walk) and the secondary lines of the
# small-document kernel and compaction.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r04c}
mkdir -p gpurun_out/$TAG
FMTS=2 REPS=32 timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/c5 -o run -- python3 tools/prof_c5.py > gpurun_out/$TAG/c5.log 2>&1 || { tail -5 gpurun_out/$TAG/c5.log; exit 1; }
find gpurun_out/$TAG/c5 -name "*kernel_stats.csv" -exec cp {} gpurun_out/$TAG/c5_v2_kernel_stats.csv \;
head -12 gpurun_out/$TAG/c5_v2_kernel_stats.csv | cut -c1-160
YM_SECONDARY=diff_c2r_v1,sv_c4r_v1,meta_c2_v1,diff_c5_v2,compact_c2_v1 timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
python3 - <<'PY'
import json
b = json.loads(open("gpurun_out/r04c/bench.json").read().strip().splitlines()[-1])
for k, v in b["secondary"].items():
    print(k, {x: v.get(x) for x in ("ms_per_step", "kernel_ms", "kernel_in_plus_out_gbs", "roofline_frac", "docs_general", "errors", "error")})
    if "cpu_baseline" in v: print("   cpu", v["cpu_baseline"])
PY
