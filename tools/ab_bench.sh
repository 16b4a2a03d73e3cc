#!/bin/bash
# A/B of library builds through the default bench line (C2 V1 unless WL is set: rotated buffer sets, data
# from HBM, asynchronous submission): for each library in $LIBS (REPS passes, interleaved) one
# `bench.py --no-secondary --no-cpu-baseline` run; prints library, ms per step and the kernel's average launch.
set -e
cd "$GRAFT_REPO_ROOT"
T=${TAG:-abb}
LIBS=${LIBS:-yjs_amd/libymerge.so}
mkdir -p gpurun_out/$T
for rep in $(seq ${REPS:-2}); do
  for lib in $LIBS; do
    b=$(basename $lib .so)
    YMERGE_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --no-secondary --no-cpu-baseline --steps ${STEPS:-200} --workload ${WL:-c2} > gpurun_out/$T/$b.$rep.json 2> gpurun_out/$T/$b.$rep.err || { tail -20 gpurun_out/$T/$b.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('%-22s rep %s  %.4f ms/step  %.1f GB/s  kernel %s' % (sys.argv[2], sys.argv[3], d['ms_per_step'], d['value'], r.get('avg_launch_ms', r.get('achieved'))))" gpurun_out/$T/$b.$rep.json $b $rep
  done
done
