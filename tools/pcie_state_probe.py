"""Probe: the pipelined host merge's time per call (C2 V1, pool-resident batch and outputs) in a fresh engine,
then after the bench's other steps (an unpipelined u64 host call; device-resident async merges over rotated
buffer sets), to find what makes it slower inside bench.py.  Usage: python tools/pcie_state_probe.py"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from yjs_amd import Engine  # noqa: E402
from yjs_amd.workloads import load_ymb, replicate  # noqa: E402

if os.environ.get("BENCH_DATA"):  # the bench's own batch (distinct copies, hash-partitioned over one rank)
    from yjs_amd.distributed import weak_scaling_shard
    a, o, d, _ = weak_scaling_shard(*load_ymb("c2_v1"), 10000, 1, 0, "hash")
else:
    a, o, d = replicate(*load_ymb("c2_v1"), 10000)
e = Engine(0)
o32 = o.astype(np.uint32)
pa = e.host_array(len(a)); pa[:] = a
po = e.host_array(len(o32), np.uint32); po[:] = o32
pd = e.host_array(len(d), np.uint32); pd[:] = d
hout = e.host_out(len(d) - 1, 2 * int(o[-1]) + 64 * (len(d) - 1) + 8192)


def timed(tag, n=12):
    e.run_host("merge", 1, pa, po, pd, out=hout)
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        e.run_host("merge", 1, pa, po, pd, out=hout)
        ts.append(time.perf_counter() - t)
    print(f"{tag:40s} median {np.median(ts) * 1e3:.3f} ms  min {min(ts) * 1e3:.3f}", flush=True)


timed("fresh")
e.run_host("merge", 1, a, o, d)
timed("after an unpipelined u64 call")
dev = torch.device("cuda", 0)
ga = torch.from_numpy(a).to(dev)
go = torch.from_numpy(o32.view(np.int32)).to(dev)
gd = torch.from_numpy(d.view(np.int32)).to(dev)
timed("after torch device copies")
big = [torch.empty(90 << 20, dtype=torch.uint8, device=dev) for _ in range(12)]
timed("after 1 GB of torch allocations")
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    x = torch.ones(1 << 20, device=dev)
    for _ in range(50):
        x = x * 1.0001
torch.cuda.synchronize()
timed("after work on a torch side stream")
cap = 2 * int(o[-1]) + 64 * (len(d) - 1) + 8192
oa = torch.empty(cap, dtype=torch.uint8, device=dev)
oo = torch.empty(len(d) - 1, dtype=torch.int64, device=dev)
ol = torch.empty(len(d) - 1, dtype=torch.int64, device=dev)
ost = torch.empty(len(d) - 1, dtype=torch.int32, device=dev)
call = e.prepare_device("merge", 1, ga, go, gd, oa, oo, ol, ost, stream=s)
for _ in range(5):
    call()
torch.cuda.synchronize()
timed("after device-resident ym_merge calls")
pending = torch.zeros(1, dtype=torch.int32, device=dev)
acall = e.prepare_merge_async(1, ga, go, gd, oa, oo, ol, ost, pending=pending, stream=s)
for _ in range(20):
    acall()
torch.cuda.synchronize()
timed("after ym_merge_async calls")
