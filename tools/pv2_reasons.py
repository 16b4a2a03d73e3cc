"""Histogram of the V2 diff / sv per-document outcomes of the specialised kernels (ym__pv2_done: done[d] = 1
completed by the column path or a small-document kernel, >= 2 = k_diff_small_v2's decline reason, 0 = left to
k_big_v2) on merged workload documents.  Usage: OP=diff WL=c2r_v2 python tools/pv2_reasons.py"""
import collections
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from yjs_amd import Engine, pack_docs  # noqa: E402
from yjs_amd.workloads import load_ymb, random_state_vectors, replicate  # noqa: E402

op, wl = os.environ.get("OP", "diff"), os.environ.get("WL", "c2r_v2")
e = Engine(0)
a, o, d = load_ymb(wl)
n = int(os.environ.get("NDOCS", "2048"))
if n > len(d) - 1:  # (batches above 4,096 documents run the V2 diff's lane kernel)
    a, o, d = replicate(a, o, d, n)
ma, mo, ml, _ = e.run_host("merge", 2, a, o, d[:n + 1])
ups = [ma[int(mo[i]):int(mo[i]) + int(ml[i])].tobytes() for i in range(n)]
pa, po, pd = pack_docs([[u] for u in ups])
sva = svo = None
if op == "diff":
    sa, so, sl, _ = e.run_host("sv", 2, pa, po, pd)
    svs = [random_state_vectors(sa[int(so[i]):int(so[i]) + int(sl[i])].tobytes(), 1, seed=i)[0] for i in range(n)]
    sva, svo, _ = pack_docs([[x] for x in svs])
e.run_host(op, 2, pa, po, pd, sva, svo)
buf = np.zeros(n, np.uint8)
e.lib.ym__pv2_done(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), ctypes.c_uint32(n))
sizes = np.array([len(u) for u in ups])
print(op, wl, n, "docs; outcomes:", sorted(collections.Counter(buf.tolist()).items()), "sizes p50", int(np.median(sizes)),
      "p90", int(np.percentile(sizes, 90)), "max", int(sizes.max()))
