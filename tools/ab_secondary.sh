#!/bin/bash
# A/B of library builds over a subset of bench.py's secondary lines: for each library in $LIBS (REPS passes,
# interleaved) one tools/secondary_only.py run with YM_SECONDARY=$CASES; prints library, case and ms per call.
set -e
cd "$GRAFT_REPO_ROOT"
T=${TAG:-abs}
mkdir -p gpurun_out/$T
for rep in $(seq ${REPS:-2}); do
  for lib in $LIBS; do
    b=$(basename $lib .so)
    YMERGE_LIB=$PWD/$lib YM_SECONDARY=$CASES timeout -k 10 300 python3 tools/secondary_only.py > gpurun_out/$T/$b.$rep.jsonl 2> gpurun_out/$T/$b.$rep.err || { tail -20 gpurun_out/$T/$b.$rep.err; exit 1; }
    python3 -c "
import json,sys
for l in open(sys.argv[1]):
    for k, v in json.loads(l).items():
        print('%-22s rep %s %-16s %s' % (sys.argv[2], sys.argv[3], k, {x: v[x] for x in v if x in ('ms_per_step', 'kernel_ms', 'docs_general', 'error')}))
" gpurun_out/$T/$b.$rep.jsonl $b $rep
  done
done
