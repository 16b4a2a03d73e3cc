"""C5 (configs[4]) diff / sv of the merged documents in V1 and V2, device-resident, for rocprofv3 kernel
traces of the multi-section paths (ym_pv2ms.hip, ym_pwalk.hip k_pw_ms): prints per-call times and checks
the bytes against the oracle once."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_ref as O  # noqa: E402
from yjs_amd import Engine, pack_docs  # noqa: E402
from yjs_amd.workloads import load_ymb, random_state_vectors  # noqa: E402

eng = Engine(0, path=os.environ["YMLIB"]) if os.environ.get("YMLIB") else Engine(0)  # YMLIB: e.g. the prof build
dev = torch.device("cuda", 0)
reps = int(os.environ.get("REPS", "32"))  # documents = 8 templates x reps (bench: 256)
for fmt in [int(x) for x in os.environ.get("FMTS", "2,1").split(",")]:
    arena, upd_off, doc_upd = load_ymb(f"c5_v{fmt}")
    merged, status, _ = O.batch("merge", fmt, arena, upd_off, doc_upd, nthreads=8)
    svo, _, _ = O.batch("sv", fmt, *pack_docs([[m] for m in merged]))
    docs = [merged[i % len(merged)] for i in range(8 * reps)]
    svs = []
    for i in range(len(docs)):
        svs.extend(random_state_vectors(svo[i % len(merged)], 1, seed=100 + i))
    a, o, d = pack_docs([[m] for m in docs])
    sva, svoff, _ = pack_docs([[s] for s in svs])
    for op in ("diff", "sv"):
        extra = (sva, svoff) if op == "diff" else ()
        outs, st, _ = O.batch(op, fmt, *pack_docs([[m] for m in docs[:8]]), *([pack_docs([[s] for s in svs[:8]])[0], pack_docs([[s] for s in svs[:8]])[1]] if op == "diff" else []))
        res = eng.run_host(op, fmt, a, o, d, *extra)
        bad = [i for i in range(8) if res[3][i] != st[i] or res[0][int(res[1][i]):int(res[1][i]) + int(res[2][i])].tobytes() != outs[i]]
        ga = torch.from_numpy(a).to(dev)
        go = torch.from_numpy(o.view(np.int64)).to(dev)
        gd = torch.from_numpy(d.view(np.int32)).to(dev)
        gsa = torch.from_numpy(sva).to(dev)
        gso = torch.from_numpy(svoff.view(np.int64)).to(dev)
        toa = torch.empty(2 * len(a) + 8192 * len(docs), dtype=torch.uint8, device=dev)
        too = torch.empty(len(docs), dtype=torch.int64, device=dev)
        tol = torch.empty(len(docs), dtype=torch.int64, device=dev)
        tst = torch.empty(len(docs), dtype=torch.int32, device=dev)
        ts = []
        for it in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rc, _ = eng.run_device(op, fmt, ga, go, gd, toa, too, tol, tst, gsa if op == "diff" else None,
                                   gso if op == "diff" else None)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        print(f"c5 v{fmt} {op}: {len(docs)} docs, rc {rc}, ms {['%.2f' % x for x in ts]}, chunked {eng.stats['docs_chunked']}, "
              f"fast {eng.stats['docs_fast']}, bad(first 8) {bad}", flush=True)
        import ctypes
        pr = (ctypes.c_ulonglong * 16)()
        eng.lib.ym__pw_prof(pr, 1)
        if pr[10]:
            print("   k_pw_ms (ticks of 10 ns, summed): tables %d, serial walk %d, windows %d, structs %d" % (pr[8], pr[9], pr[10], pr[11]))
        print("   pw_prof: k_pw_ms phase ticks A %d B %d C %d patches %d | stitch counters: whole %d, entry not whole %d, "
              "entry not in first %d, record batches %d, re-parsed structs %d, search loads %d" % (tuple(pr[:4]) + tuple(pr[:6])))
        if hasattr(eng.lib, "ym__pw_ticks"):
            tk = (ctypes.c_ulonglong * 16)()
            eng.lib.ym__pw_ticks(tk, 1)
            if any(tk):
                names = "sv hdr desc stage search consume cut ds alloc write patch".split()
                per = 1e-2 / (len(docs) * 6)  # us per document per call (6 calls incl. the checked one)
                print("   k_pw_stitch us/doc: " + " ".join("%s %.0f" % (n, tk[i] * per) for i, n in enumerate(names)), flush=True)
        pm = (ctypes.c_ulonglong * 16)()
        eng.lib.ym__ms_prof(pm, 1)
        print("   k_ms_rest/k_ms_walk (ticks of 10 ns, summed over documents and calls): columns %d, walk kernel %d (serial %d, "
              "tables %d), windows %d, tokens %d (walker-parsed %d), headers %d (global %d), final-run structs %d, len cursor "
              "moves %d" % (pm[0], pm[1], pm[2], pm[7], pm[3], pm[4], pm[5], pm[6], pm[9], pm[8], pm[10]))
        for i in bad[:2]:
            got = res[0][int(res[1][i]):int(res[1][i]) + int(res[2][i])].tobytes()
            want = outs[i]
            k = next((q for q in range(min(len(got), len(want))) if got[q] != want[q]), None)
            print(f"   doc {i}: status {res[3][i]} vs {st[i]}, len {len(got)} vs {len(want)}, first diff at {k}: "
                  f"{got[k - 8:k + 8].hex() if k is not None else ''} vs {want[k - 8:k + 8].hex() if k is not None else ''}")
