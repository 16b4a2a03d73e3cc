"""Histogram of the V1 diff / sv decline reasons of the chunk walk and k_pw_small (ym__pw_reasons: done[d] per
document: 1 = completed, >= 2 = why) on merged workload documents.  Usage: OP=diff WL=c2r_v1 python tools/pw_reasons.py"""
import collections
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from yjs_amd import Engine, pack_docs  # noqa: E402
from yjs_amd.workloads import load_ymb, random_state_vectors  # noqa: E402

op, wl = os.environ.get("OP", "diff"), os.environ.get("WL", "c2r_v1")
e = Engine(0)
a, o, d = load_ymb(wl)
n = min(len(d) - 1, int(os.environ.get("NDOCS", "1024")))
ma, mo, ml, _ = e.run_host("merge", 1, a, o, d[:n + 1])
ups = [ma[int(mo[i]):int(mo[i]) + int(ml[i])].tobytes() for i in range(n)]
pa, po, pd = pack_docs([[u] for u in ups])
sva = svo = None
if op == "diff":
    sa, so, sl, _ = e.run_host("sv", 1, pa, po, pd)
    svs = [random_state_vectors(sa[int(so[i]):int(so[i]) + int(sl[i])].tobytes(), 1, seed=i)[0] for i in range(n)]
    sva, svo, _ = pack_docs([[x] for x in svs])
e.run_host(op, 1, pa, po, pd, sva, svo)
buf = np.zeros(n, np.uint8)
e.lib.ym__pw_reasons(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), ctypes.c_uint32(n))
print(op, wl, n, "docs; reasons:", sorted(collections.Counter(buf.tolist()).items()), "sizes p50", int(np.median([len(u) for u in ups])))
