"""Host-batch merges (the Node addon's path) of the C2 V1 batch, pipelined: u32 offsets, reused page-locked
outputs.  Run under rocprofv3 --kernel-trace --memory-copy-trace to see the copies and kernels overlap.
Usage: python tools/host_pipe_prof.py [calls]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from yjs_amd import Engine  # noqa: E402
from yjs_amd.workloads import load_ymb, replicate  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 10
a, o, d = replicate(*load_ymb(os.environ.get("WL", "c2_v1")), int(os.environ.get("NDOCS", "10000")))
e = Engine(0)
o32 = o.astype(np.uint32)
if os.environ.get("PINNED", "1") == "1":  # the batch in page-locked pool memory (as the Node addon packs it)
    pa = e.host_array(len(a)); pa[:] = a; a = pa
    po = e.host_array(len(o32), np.uint32); po[:] = o32; o32 = po
    pd = e.host_array(len(d), np.uint32); pd[:] = d; d = pd
hout = e.host_out(len(d) - 1, 2 * int(o[-1]) + 64 * (len(d) - 1) + 8192)
e.run_host("merge", 1, a, o32, d, out=hout)
ts = []
for _ in range(calls):
    t = time.perf_counter()
    e.run_host("merge", 1, a, o32, d, out=hout)
    ts.append(time.perf_counter() - t)
print("ms per call", [round(x * 1e3, 3) for x in ts], "GB/s", round(int(o[-1]) / np.median(ts) / 1e9, 2))
