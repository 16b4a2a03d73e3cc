#!/bin/bash
# Secondary bench lines ($SEC) under each value of the environment variable $VAR in $VALS: one line per value.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=${TAG:-sweep}; mkdir -p gpurun_out/$T
for v in $VALS; do
  env $VAR=$v YM_SECONDARY="$SEC" timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$T/b_$v.json 2> gpurun_out/$T/b_$v.err || { tail -5 gpurun_out/$T/b_$v.err; exit 1; }
  python3 -c "
import json; l=[json.loads(x) for x in open('gpurun_out/$T/b_$v.json') if x.startswith('{')][-1]
print('$VAR=$v', ' '.join(f'{k}={v.get(\"ms_per_step\", v)}' for k,v in l['secondary'].items()))"
done
