#!/bin/bash
# Compaction: bench lines over documents-per-wave (LANES) x register-occupancy target (OCCS) settings.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-cpts}
mkdir -p gpurun_out/$TAG
for O in ${OCCS:-1 2}; do
  for L in ${LANES:-8 10 16}; do
    YMERGE_COMPACT_OCC=$O YMERGE_COMPACT_LANES=$L YM_SECONDARY=compact_c2_v1,compact_c2_v2,compact_c4_v1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/bench_o${O}_l$L.json 2> gpurun_out/$TAG/bench_o${O}_l$L.err
  done
done
echo done
