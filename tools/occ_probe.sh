cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_workloads.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread -k "merge" > gpurun_out/pytest_quick.log 2>&1 || { tail -30 gpurun_out/pytest_quick.log; exit 1; }
tail -2 gpurun_out/pytest_quick.log
for wl in c2_v1 c4_v1; do for occ in 4 5 6; do
  echo "$wl occ $occ"; WL=$wl YMERGE_FAST_OCC=$occ YMERGE_FAST_STOP=0 timeout -k 10 120 python tools/ablate_fast.py 2>&1 | tail -1
done; done
