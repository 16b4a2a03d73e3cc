#!/bin/bash
# Compaction: GPU parity, then the bench lines at several documents-per-wave settings.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-cpt2}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_gpu_compact.py -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_compact.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_compact.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest_compact.log
for L in ${LANES:-16 4 64}; do
  YMERGE_COMPACT_LANES=$L YM_SECONDARY=compact_c2_v1,compact_c2_v2,compact_c4_v1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/bench_l$L.json 2> gpurun_out/$TAG/bench_l$L.err
done
echo done
