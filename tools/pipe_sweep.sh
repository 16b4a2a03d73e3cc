# host-merge pipeline settings (tools/host_pipe_prof.py over the C2 V1 batch): copy kernels (pool-resident
# batch) against DMA copies, by chunk size and copy-queue priority
cd $GRAFT_REPO_ROOT
for kb in 4096 6144 9216; do
  r=$( YMERGE_PIPE_CHUNK_KB=$kb timeout -k 10 60 python3 tools/host_pipe_prof.py 16 | tail -1 ); echo "copykernel prio kb=$kb $r"
  r=$( YMERGE_PIPE_NOPRIO=1 YMERGE_PIPE_CHUNK_KB=$kb timeout -k 10 60 python3 tools/host_pipe_prof.py 16 | tail -1 ); echo "copykernel noprio kb=$kb $r"
done
r=$( YMERGE_PIPE_NOZC=1 YMERGE_PIPE_ALT=0 timeout -k 10 60 python3 tools/host_pipe_prof.py 16 | tail -1 ); echo "dma kb=6144 $r"
