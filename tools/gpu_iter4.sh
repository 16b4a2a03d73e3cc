#!/bin/bash
# Round-4 iteration: a GPU test subset (TESTK, a pytest -k expression; TESTF: files), the C5 profile (FMTS),
# and bench secondary lines (SEC, comma-separated).  Every GPU step has its own limit; stops at the first failure.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r04x}
mkdir -p gpurun_out/$TAG
if [ -n "$TESTK" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTF:-tests/test_gpu_golden.py tests/test_gpu_workloads.py} -x -v --timeout 200 --timeout-method thread -k "$TESTK" > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
  tail -2 gpurun_out/$TAG/pytest.log
fi
if [ -n "$FMTS" ]; then
  FMTS=$FMTS REPS=32 timeout -k 10 300 python -u tools/prof_c5.py > gpurun_out/$TAG/c5.log 2>&1 || { tail -20 gpurun_out/$TAG/c5.log; exit 1; }
  grep -v -i warn gpurun_out/$TAG/c5.log | grep -v "ga = torch" | head -30
fi
if [ -n "$SEC" ]; then
  YM_SECONDARY=$SEC timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
  TAG=$TAG python3 - <<'PY'
import json, os
b = json.loads(open(f"gpurun_out/{os.environ['TAG']}/bench.json").read().strip().splitlines()[-1])
print("headline", b["value"], b["ms_per_step"], b["roofline"]["avg_launch_ms"], b["roofline"]["frac"])
for k, v in b["secondary"].items():
    print(k, {x: v.get(x) for x in ("ms_per_step", "kernel_ms", "kernel_in_plus_out_gbs", "roofline_frac", "docs_general", "errors", "error")})
    if "cpu_baseline" in v: print("   cpu", v["cpu_baseline"]["docs_per_s"], v["cpu_baseline"]["all_host_cores_estimate"])
PY
fi
