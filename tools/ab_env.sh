#!/bin/bash
# A/B of environment settings over a subset of bench.py's secondary lines: for each setting in $ENVS
# (';'-separated "VAR=value VAR2=value" groups, REPS passes, interleaved) one tools/secondary_only.py run with
# YM_SECONDARY=$CASES; prints the setting, case and ms per call.
set -e
cd "$GRAFT_REPO_ROOT"
T=${TAG:-abe}
mkdir -p gpurun_out/$T
IFS=';' read -ra SETS <<< "$ENVS"
for rep in $(seq ${REPS:-2}); do
  i=0
  for e in "${SETS[@]}"; do
    i=$((i+1))
    env $e YM_SECONDARY=$CASES timeout -k 10 300 python3 tools/secondary_only.py > gpurun_out/$T/s$i.$rep.jsonl 2> gpurun_out/$T/s$i.$rep.err || { tail -20 gpurun_out/$T/s$i.$rep.err; exit 1; }
    python3 -c "
import json,sys
for l in open(sys.argv[1]):
    for k, v in json.loads(l).items():
        print('%-28s rep %s %-14s %s' % (sys.argv[2], sys.argv[3], k, {x: v[x] for x in v if x in ('ms_per_step', 'kernel_ms', 'docs_general', 'error')}))
" gpurun_out/$T/s$i.$rep.jsonl "$e" $rep
  done
done
