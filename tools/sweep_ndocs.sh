cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r06d
for n in 1024 2048 4096 8192 10000 16384 32768; do
  NDOCS=$n WL=c2_v1 timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06d/n$n -o run -- python3 tools/prof_run.py 20 > gpurun_out/r06d/n$n.log 2>&1 || exit 1
  echo n=$n $(grep k_fast_merge gpurun_out/r06d/n$n/run_kernel_stats.csv 2>/dev/null | head -1 | cut -d, -f4,6,7)
done
