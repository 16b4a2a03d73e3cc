#!/bin/bash
# One GPU call: parity tests, smoke, bench (with secondary lines), rocprof kernel stats of the C2 and
# C5 benches, PMC passes of the headline kernel.  Every GPU step has its own limit; stops at a failure.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01c}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_c5 -o run -- python -u bench.py --workload c5v2 --docs-per-gpu 256 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/bench_prof_c5.json 2> gpurun_out/bench_prof_c5.err
TAG=pmc_$TAG bash tools/pmc_passes.sh > gpurun_out/pmc_passes.log 2>&1
echo done
