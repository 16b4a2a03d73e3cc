#!/bin/bash
# The host-resident path: its GPU tests (pipelined merges, the Node addon), then REPS default bench lines
# without secondaries, printing the headline and the pcie_inclusive object of each.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_host_pipe.py tests/test_gpu_js.py -x -q --timeout 300 --timeout-method thread > gpurun_out/hp/pytest.log 2>&1 || { tail -20 gpurun_out/hp/pytest.log; exit 1; }
tail -1 gpurun_out/hp/pytest.log
for i in $(seq ${REPS:-2}); do
  timeout -k 10 120 python3 bench.py --no-secondary --no-cpu-baseline > gpurun_out/hp/b$i.json 2> gpurun_out/hp/b$i.err || { tail -5 gpurun_out/hp/b$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], json.dumps(d['pcie_inclusive']))" gpurun_out/hp/b$i.json
done
