#!/bin/bash
# One iteration of the headline-kernel / compaction work: merge parity (golden + workloads), the stop
# ablation of k_fast_merge_v1, the default bench's headline line, the compaction lanes sweep.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-iter}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_workloads.py -x -q --timeout 300 --timeout-method thread -k "merge or golden or pref or ds_merge" > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
STOPS="${STOPS:-2 3 0}" bash tools/pmc_stops.sh > gpurun_out/$TAG/stops.txt 2>&1
timeout -k 10 200 python -u bench.py --no-secondary --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
for L in ${LANES:-}; do
  YMERGE_COMPACT_LANES=$L YM_SECONDARY=compact_c2_v1,compact_c4_v1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/bench_l$L.json 2> gpurun_out/$TAG/bench_l$L.err
done
echo done
