"""Times the engine's ops on device-resident batches of the benchmark workloads (general and fast
paths): merge V1/V2 over C2/C4, diff/sv V1/V2 over C3 (replicated, random state vectors).
Usage: python tools/time_ops.py [case ...]   cases: merge:c2_v1 merge:c2_v2 diff:c3_v1 sv:c3_v2 ..."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from yjs_amd import Engine, pack_docs  # noqa: E402
from yjs_amd.workloads import load_ymb, replicate, random_state_vectors  # noqa: E402

dev = torch.device("cuda", 0)
eng = Engine(0)
cases = sys.argv[1:] or ["merge:c2_v1", "merge:c2_v2", "merge:c4_v2", "diff:c3_v1", "diff:c3_v2", "sv:c3_v1"]
for case in cases:
    op, wl = case.split(":")
    fmt = 2 if wl.endswith("v2") else 1
    a, o, d = load_ymb(wl)
    sva = svo = None
    if op == "merge":
        a, o, d = replicate(a, o, d, int(os.environ.get("NDOCS", "256" if wl.startswith("c5") else "10000")))
    elif wl.startswith("c5"):
        # diff / sv over merged C5 documents (1,024 clients each), random per-client state vectors
        n = int(os.environ.get("NDOCS_BIG", "256"))
        ma, mo, ml, mst = eng.run_host("merge", fmt, a, o, d)
        ups = [ma[int(mo[i]):int(mo[i]) + int(ml[i])].tobytes() for i in range(len(d) - 1)]
        svfn = eng.run_host
        sa, so_, sl, _ = svfn("sv", fmt, *pack_docs([[u] for u in ups]))
        fulls = [sa[int(so_[i]):int(so_[i]) + int(sl[i])].tobytes() for i in range(len(ups))]
        svs = [random_state_vectors(fulls[i % len(ups)], 1, seed=i)[0] for i in range(n)]
        a, o, d = pack_docs([[ups[i % len(ups)]] for i in range(n)])
        sva, svo, _ = pack_docs([[s] for s in svs])
    else:
        n = int(os.environ.get("NDOCS_BIG", "256"))
        upd = a.tobytes()
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ref as O
        full = O.sv_from_update(upd, fmt)[1]
        svs = random_state_vectors(full, n, seed=5)
        a, o, d = pack_docs([[upd] for _ in range(n)])
        sva, svo, _ = pack_docs([[s] for s in svs])
    nd = len(d) - 1
    ga = torch.from_numpy(a).to(dev)
    go = torch.from_numpy(o.view(np.int64)).to(dev)
    gd = torch.from_numpy(d.view(np.int32)).to(dev)
    gsa = torch.from_numpy(sva).to(dev) if sva is not None else None
    gso = torch.from_numpy(svo.view(np.int64)).to(dev) if svo is not None else None
    cap = 4 * len(a) + 128 * nd + 8192 + (2 * len(sva) if sva is not None else 0)
    oa = torch.empty(cap, dtype=torch.uint8, device=dev)
    oo = torch.empty(nd, dtype=torch.int64, device=dev)
    ol = torch.empty(nd, dtype=torch.int64, device=dev)
    st = torch.empty(nd, dtype=torch.int32, device=dev)
    times = []
    for i in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc, used = eng.run_device(op, fmt, ga, go, gd, oa, oo, ol, st, gsa, gso)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        assert rc == 0, rc
    t = min(times[1:])
    print(f"{case:14s} docs {nd:6d} in {len(a)/1e6:8.1f} MB  {t*1e3:9.3f} ms  {len(a)/t/1e9:8.2f} GB/s  "
          f"errors {int((st != 0).sum())}  {eng.stats}", flush=True)
