#!/bin/bash
# host-merge pipeline: k_pack_docs grid per chunk (YMERGE_PACK_GRID) x chunk size x copy-queue priority
# (tools/host_pipe_prof.py over the C2 V1 batch, pool-resident batch and outputs)
cd $GRAFT_REPO_ROOT
for e in "YMERGE_PACK_GRID=0" "YMERGE_PACK_GRID=32" "YMERGE_PACK_GRID=64" "YMERGE_PACK_GRID=128" "YMERGE_PACK_GRID=256" \
         "YMERGE_PACK_GRID=64 YMERGE_PIPE_CHUNK_KB=3072" "YMERGE_PACK_GRID=64 YMERGE_PIPE_NOPRIO=1" "YMERGE_PACK_GRID=0 YMERGE_PIPE_CHUNK_KB=3072"; do
  r=$(env $e timeout -k 10 60 python3 tools/host_pipe_prof.py 16 | tail -1 | sed 's/.*GB\/s/GB\/s/'); echo "$e $r"
done
