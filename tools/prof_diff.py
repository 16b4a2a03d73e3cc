"""Runs a batched diffUpdate / encodeStateVectorFromUpdate over replicated single-update documents on
cuda:0 (device-resident): the workload profiled by rocprofv3 for the streamed walkers (ym_big*.hip).
Usage: WL=c3_v1 OP=diff NDOCS=256 rocprofv3 ... -- python tools/prof_diff.py [steps]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from yjs_amd import Engine, pack_docs  # noqa: E402
from yjs_amd.workloads import load_ymb, replicate, random_state_vectors  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
wl = os.environ.get("WL", "c3_v1")
op = os.environ.get("OP", "diff")
n = int(os.environ.get("NDOCS", "256"))
fmt = 2 if wl.endswith("v2") else 1
a, o, d = load_ymb(wl)
e = Engine(0)
if len(d) - 1 > 1 or d[1] - d[0] > 1:  # multi-update templates (C5): merge them first
    ma, mo, ml, _ = e.run_host("merge", fmt, a, o, d)
    ups = [ma[int(mo[i]):int(mo[i]) + int(ml[i])].tobytes() for i in range(len(d) - 1)]
else:
    ups = [a.tobytes()]
sa, so_, sl, _ = e.run_host("sv", fmt, *pack_docs([[u] for u in ups]))
fulls = [sa[int(so_[i]):int(so_[i]) + int(sl[i])].tobytes() for i in range(len(ups))]
svs = [random_state_vectors(fulls[i % len(ups)], 1, seed=i)[0] for i in range(n)]
a, o, d = pack_docs([[ups[i % len(ups)]] for i in range(n)])
sva, svo, _ = pack_docs([[x] for x in svs])
dev = torch.device("cuda", 0)
ga = torch.from_numpy(a).to(dev)
go = torch.from_numpy(o.view(np.int64)).to(dev)
gd = torch.from_numpy(d.view(np.int32)).to(dev)
gsa = torch.from_numpy(sva).to(dev)
gso = torch.from_numpy(svo.view(np.int64)).to(dev)
oa = torch.empty(4 * len(a) + 128 * n + 8192 + 2 * len(sva), dtype=torch.uint8, device=dev)
oo = torch.empty(n, dtype=torch.int64, device=dev)
ol = torch.empty(n, dtype=torch.int64, device=dev)
st = torch.empty(n, dtype=torch.int32, device=dev)
for i in range(steps):
    if op == "diff":
        rc, used = e.run_device("diff", fmt, ga, go, gd, oa, oo, ol, st, gsa, gso)
    else:
        rc, used = e.run_device("sv", fmt, ga, go, gd, oa, oo, ol, st)
    assert rc == 0, rc
torch.cuda.synchronize()
print("op", op, "wl", wl, "in_bytes", len(a), "out_bytes", int(ol.sum().item()), "docs", n, e.stats,
      "ms", e.last_stats.fast_ms)
