"""Host<->device copy rates on the box: pageable vs pinned, H2D / D2H / both directions at once
(two streams).  Usage: python tools/pcie_probe.py"""
import time

import torch

dev = torch.device("cuda", 0)
torch.ones(1, device=dev)
for mb in (4, 16, 64):
    n = mb << 20
    pg = torch.empty(n, dtype=torch.uint8)
    pg.fill_(1)
    pn = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    pn.fill_(1)
    pn2 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    d2 = torch.empty(n, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def t(fn, reps=10):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    r = {}
    r["h2d_pageable"] = n / t(lambda: d.copy_(pg)) / 1e9
    r["h2d_pinned"] = n / t(lambda: d.copy_(pn, non_blocking=True)) / 1e9
    r["d2h_pageable"] = n / t(lambda: pg.copy_(d)) / 1e9
    r["d2h_pinned"] = n / t(lambda: pn.copy_(d, non_blocking=True)) / 1e9

    def both():
        with torch.cuda.stream(s1):
            d.copy_(pn, non_blocking=True)
        with torch.cuda.stream(s2):
            pn2.copy_(d2, non_blocking=True)
    r["duplex_pinned_each"] = n / t(both) / 1e9
    print(mb, "MiB", {k: round(v, 1) for k, v in r.items()}, flush=True)
