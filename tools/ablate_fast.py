"""Times the fast-path kernel with phases ablated (YMERGE_FAST_STOP=n ends each doc after phase n).
Each variant runs in its own process (the stop level is read once).  Usage: python tools/ablate_fast.py"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json, numpy as np, torch
sys.path.insert(0, %r)
from yjs_amd import Engine
from yjs_amd.workloads import load_ymb, replicate
a, o, d = replicate(*load_ymb(os.environ.get("WL", "c2_v1")), int(os.environ.get("NDOCS", "10000")))
dev = torch.device("cuda", 0)
ga = torch.from_numpy(a).to(dev); go = torch.from_numpy(o.view(np.int64)).to(dev); gd = torch.from_numpy(d.view(np.int32)).to(dev)
n = len(d) - 1
oa = torch.empty(4 * len(a) + 128 * n + 8192, dtype=torch.uint8, device=dev)
oo = torch.empty(n, dtype=torch.int64, device=dev); ol = torch.empty(n, dtype=torch.int64, device=dev); st = torch.empty(n, dtype=torch.int32, device=dev)
e = Engine(0)
ms = []
for i in range(25):
    rc, used = e.run_device("merge", 2 if os.environ.get("WL", "c2_v1").endswith("v2") else 1, ga, go, gd, oa, oo, ol, st)
    if i >= 5: ms.append(e.last_stats.fast_ms)
print(json.dumps({"stop": int(os.environ.get("YMERGE_FAST_STOP", "0")), "fast_ms_mean": float(np.mean(ms)), "fast_ms_min": float(np.min(ms))}))
''' % ROOT

for stop in ([1, 2, 3, 4, 5, 6, 7, 0] if os.environ.get("WL", "").endswith("v2") else [int(x) for x in os.environ.get('STOPS', '1 2 3 4 5 6 0').split()]):
    env = dict(os.environ, YMERGE_FAST_STOP=str(stop))
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    print(line[0] if line else ("FAILED", stop, r.stderr[-2000:]), flush=True)
