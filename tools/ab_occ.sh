#!/bin/bash
# A/B of k_fast_merge_v1's launch bound (YMERGE_FAST_OCC: waves per SIMD the register allocation targets) through the
# default bench line: for each value in $OCCS (REPS passes, interleaved) one bench.py --no-secondary --no-cpu-baseline
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/occ
for rep in $(seq ${REPS:-2}); do
  for o in ${OCCS:-8 7 6}; do
    YMERGE_FAST_OCC=$o timeout -k 10 120 python3 bench.py --no-secondary --no-cpu-baseline --steps ${STEPS:-200} --workload ${WL:-c2} > gpurun_out/occ/$o.$rep.json 2> gpurun_out/occ/$o.$rep.err || { tail -5 gpurun_out/occ/$o.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('occ %s rep %s  %.4f ms/step  %.1f GB/s  kernel %.4f ms' % (sys.argv[2], sys.argv[3], d['ms_per_step'], d['value'], d['roofline']['avg_launch_ms']))" gpurun_out/occ/$o.$rep.json $o $rep
  done
done
