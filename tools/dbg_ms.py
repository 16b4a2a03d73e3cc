"""Debug aid for the multi-section V2 column path (ym_pv2ms.hip): golden V2 diff / sv / meta vectors with the
path's threshold at 1 byte, and merged C5 V2 documents against random state vectors; prints mismatches with
the path's per-document decline codes (ym__pv2_why) and how many documents it took."""
import collections
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import golden_io  # noqa: E402
import oracle_ref as O  # noqa: E402
from yjs_amd import Engine, pack_docs  # noqa: E402
from yjs_amd.workloads import load_ymb, random_state_vectors  # noqa: E402

eng = Engine(0)


def why(n):
    w = np.zeros(n, np.uint32)
    eng.lib.ym__pv2_why(w.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(n))
    return w


def compare(res, outs, st):
    oa, oo, ol, s = res
    bad = []
    for i in range(len(s)):
        if int(s[i]) & 0xff != int(st[i]):
            bad.append((i, "status", int(s[i]), int(st[i])))
        elif s[i] == 0 and oa[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() != outs[i]:
            bad.append((i, "bytes", int(ol[i]), len(outs[i])))
    return bad


os.environ["YMERGE_PW_MIN"] = "1"
os.environ["YMERGE_PWMS_MIN"] = "2"
cases = golden_io.load_cases()
for op, fmt in [(o, f) for f in (1, 2) for o in ("diff", "sv", "meta")]:
    cs = [c for c in cases if c["op"] == op and c["fmt"] == fmt]
    a, o, d = pack_docs([[c["inputs"][0]] for c in cs])
    extra = ()
    if op == "diff":
        sva, svo, _ = pack_docs([[c["sv"]] for c in cs])
        extra = (sva, svo)
    res = eng.run_host(op, fmt, a, o, d, *extra)
    if fmt == 2:
        w = why(len(cs))
    else:
        w = np.zeros(len(cs), np.uint8)
        eng.lib.ym__pw_reasons(w.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(len(cs)))
    outs, st, _ = O.batch(op, fmt, a, o, d, *extra)
    bad = compare(res, outs, st)
    print(f"golden {op} v{fmt}: {len(cs)} cases, chunked {eng.stats['docs_chunked']}, why {dict(collections.Counter(w.tolist()))}")
    for b in bad[:10]:
        print("   BAD", b, cs[b[0]]["id"], "why", int(w[b[0]]))
    sys.stdout.flush()
del os.environ["YMERGE_PW_MIN"]
del os.environ["YMERGE_PWMS_MIN"]

arena, upd_off, doc_upd = load_ymb("c5_v2")
merged, status, _ = O.batch("merge", 2, arena, upd_off, doc_upd, nthreads=8)
a2, o2, d2 = pack_docs([[m] for m in merged])
for op in ("sv", "meta", "diff"):
    extra = ()
    if op == "diff":
        svs = []
        sv_outs, _, _ = O.batch("sv", 2, a2, o2, d2)
        for i in range(len(merged)):
            svs.extend(random_state_vectors(sv_outs[i], 1, seed=100 + i))
        sva, svo, _ = pack_docs([[s] for s in svs])
        extra = (sva, svo)
    t0 = time.time()
    res = eng.run_host(op, 2, a2, o2, d2, *extra)
    dt = time.time() - t0
    w = why(len(merged))
    outs, st, _ = O.batch(op, 2, a2, o2, d2, *extra, nthreads=8)
    bad = compare(res, outs, st)
    print(f"c5 {op} v2: chunked {eng.stats['docs_chunked']}/{len(merged)} why {dict(collections.Counter(w.tolist()))} "
          f"device_ms {eng.last_stats.device_ms:.2f} wall {dt * 1e3:.1f} ms bad {bad[:5]}")
    sys.stdout.flush()
