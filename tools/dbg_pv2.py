"""Debug aid for the column-parallel V2 path: C3 V2 diff over n replicated documents with random state
vectors (the bench's secondary case), device-resident and host-staged; prints how many documents the
path took (docs_chunked) and the per-document statuses that differ between the two."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from yjs_amd import Engine, pack_docs  # noqa: E402
from yjs_amd.workloads import load_ymb, replicate, random_state_vectors  # noqa: E402
import bench  # noqa: E402

eng = Engine(0)
dev = torch.device("cuda", 0)
a0, o0, d0 = load_ymb("c3_v2")
upd = a0.tobytes()
full = bench._sv_of_single_client_update(upd, 2)
for n in (8, 64, 512, 4096):
    a, o, d = replicate(a0, o0, d0, n)
    svs = random_state_vectors(full, n, seed=7)
    sva, svo, _ = pack_docs([[x] for x in svs])
    oa, oo, ol, st = eng.run_host("diff", 2, a, o, d, sva, svo)
    hs = dict(eng.stats)
    ga = torch.from_numpy(a).to(dev)
    go = torch.from_numpy(o.view(np.int64)).to(dev)
    gd = torch.from_numpy(d.view(np.int32)).to(dev)
    gsa = torch.from_numpy(sva).to(dev)
    gso = torch.from_numpy(svo.view(np.int64)).to(dev)
    cap = 4 * len(a) + 128 * n + 8192 + 2 * len(sva)
    toa = torch.empty(cap, dtype=torch.uint8, device=dev)
    too = torch.empty(n, dtype=torch.int64, device=dev)
    tol = torch.empty(n, dtype=torch.int64, device=dev)
    tst = torch.empty(n, dtype=torch.int32, device=dev)
    rc, used = eng.run_device("diff", 2, ga, go, gd, toa, too, tol, tst, gsa, gso)
    torch.cuda.synchronize()
    ds = dict(eng.stats)
    same = 0
    tl = tol.cpu().numpy(); to = too.cpu().numpy(); ta = None
    for i in range(min(n, 64)):
        if tl[i] == ol[i]:
            same += 1
    import collections, ctypes
    why = np.zeros(n, np.uint32)
    eng.lib.ym__pv2_why(why.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(n))
    print("   why", dict(collections.Counter(why.tolist())), "first declined", [i for i in range(n) if why[i]][:5])
    print(n, "host chunked", hs["docs_chunked"], "fast", hs["docs_fast"], "| device rc", rc, "chunked", ds["docs_chunked"],
          "fast", ds["docs_fast"], "ms", round(eng.last_stats.device_ms, 2), "len-equal(first64)", same, flush=True)
    del ga, go, gd, gsa, gso, toa, too, tol, tst
    torch.cuda.empty_cache()
