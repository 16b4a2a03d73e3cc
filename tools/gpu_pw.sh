#!/bin/bash
# GPU iteration for the chunk-parallel V1 diff / sv walk: parity (golden through the walk, C3 / C5
# workloads, damaged updates), then the diff / sv bench lines.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_workloads.py -x -v --timeout 200 --timeout-method thread \
  -k "${PWK:-diff or sv or chunked}" > gpurun_out/pytest_pw.log 2>&1 || { tail -40 gpurun_out/pytest_pw.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_pw.log | tail -3
YM_SECONDARY=${SEC:-diff_c3_v1,sv_c3_v1,diff_c5_v1,meta_c3_v1} timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_pw.json 2> gpurun_out/bench_pw.err || { tail -20 gpurun_out/bench_pw.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_pw.json').read().strip().splitlines()[-1])
for k,v in d.get('secondary',{}).items(): print(k, v)
"
if [ -n "$PROF" ]; then TAG=${PROF} bash tools/gpu_prof_pw.sh; fi
