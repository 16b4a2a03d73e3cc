set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
WL=c2_v2 timeout -k 10 300 python tools/ablate_fast.py > gpurun_out/abl2.log 2>&1
