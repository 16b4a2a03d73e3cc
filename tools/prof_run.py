"""Runs the C2 batched merge (OP: or diff / sv / meta over the merged documents) on cuda:0 (device-resident) a few times: the workload profiled by
rocprofv3 (kernel trace / PMC counters).  Usage: rocprofv3 ... -- python tools/prof_run.py [steps]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from yjs_amd import Engine  # noqa: E402
from yjs_amd.workloads import load_ymb, replicate  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
wl = os.environ.get("WL", "c2_v1")
fmt = 2 if wl.endswith("v2") else 1
a, o, d = replicate(*load_ymb(wl), int(os.environ.get("NDOCS", "10000")))
dev = torch.device("cuda", 0)
ga = torch.from_numpy(a).to(dev)
go = torch.from_numpy(o.astype(np.uint32).view(np.int32) if os.environ.get("OFF64") is None else o.view(np.int64)).to(dev)  # u32 offsets (YM_OFF32), as bench.py
gd = torch.from_numpy(d.view(np.int32)).to(dev)
n = len(d) - 1
oa = torch.empty(4 * len(a) + 128 * n + 8192, dtype=torch.uint8, device=dev)
oo = torch.empty(n, dtype=torch.int64, device=dev)
ol = torch.empty(n, dtype=torch.int64, device=dev)
st = torch.empty(n, dtype=torch.int32, device=dev)
e = Engine(0)
op = os.environ.get("OP", "merge")  # diff / sv / meta: over the merged documents (the engine's own merge)
gsa = gso = None
if op != "merge":
    from yjs_amd import pack_docs  # noqa: E402
    from yjs_amd.workloads import random_state_vectors  # noqa: E402
    ma, mo, ml, ms = e.run_host("merge", fmt, a, o, d)
    merged = [ma[int(mo[i]):int(mo[i]) + int(ml[i])].tobytes() for i in range(n)]
    a, o, d = pack_docs([[m] for m in merged])
    ga = torch.from_numpy(a).to(dev)
    go = torch.from_numpy(o.view(np.int64)).to(dev)
    gd = torch.from_numpy(d.view(np.int32)).to(dev)
    if op == "diff":
        sa, so, sl, _ = e.run_host("sv", fmt, a, o, d)
        svs = []
        for i in range(n):
            svs.extend(random_state_vectors(sa[int(so[i]):int(so[i]) + int(sl[i])].tobytes(), 1, seed=i))
        sva, svo, _ = pack_docs([[x] for x in svs])
        gsa = torch.from_numpy(sva).to(dev)
        gso = torch.from_numpy(svo.view(np.int64)).to(dev)
for i in range(steps):
    rc, used = e.run_device(op, fmt, ga, go, gd, oa, oo, ol, st, gsa, gso)
    assert rc == 0, rc
torch.cuda.synchronize()
print("in_bytes", len(a), "out_bytes", int(ol.sum().item()), "docs", n, e.stats)
