"""Host round-trip cost of one device-resident ym_merge call (C2 V1, 10 k docs): wall time per call with
and without the stats struct, against the fast kernel's own time.  Usage: python tools/call_overhead.py"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from yjs_amd import Engine  # noqa: E402
from yjs_amd.engine import _Batch, _Out  # noqa: E402
from yjs_amd.workloads import load_ymb, replicate  # noqa: E402

dev = torch.device("cuda", 0)
eng = Engine(0)
a, o, d = replicate(*load_ymb(os.environ.get("WL", "c2_v1")), 10000)
fmt = 2 if os.environ.get("WL", "c2_v1").endswith("v2") else 1
g_a = torch.from_numpy(a).to(dev)
g_o = torch.from_numpy(o.view(np.int64)).to(dev)
g_d = torch.from_numpy(d.view(np.int32)).to(dev)
n = len(d) - 1
cap = 4 * int(o[-1]) + 128 * n + 8192
oa = torch.empty(cap, dtype=torch.uint8, device=dev)
oo = torch.empty(n, dtype=torch.int64, device=dev)
ol = torch.empty(n, dtype=torch.int64, device=dev)
os_ = torch.empty(n, dtype=torch.int32, device=dev)
stream = torch.cuda.current_stream(dev)
call = eng.prepare_device("merge", fmt, g_a, g_o, g_d, oa, oo, ol, os_, stream=stream)
b = _Batch(g_a.data_ptr(), g_o.data_ptr(), g_d.data_ptr(), n, len(o) - 1, fmt, 1, None, None)
out = _Out(oa.data_ptr(), cap, oo.data_ptr(), ol.data_ptr(), os_.data_ptr(), 0)
fn = eng.lib.ym_merge
s = ctypes.c_void_p(stream.cuda_stream)


def bare():
    return fn(ctypes.byref(b), ctypes.byref(out), s, None)


for name, f in (("stats", call), ("no-stats", bare), ("stats", call), ("no-stats", bare)):
    for _ in range(20):
        f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(300):
        f()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t) / 300 * 1e6
    print(f"{name:9s} {us:8.1f} us/call   fast kernel (events) {eng.last_stats.fast_ms * 1e3:7.1f} us", flush=True)
# baseline: a tiny torch op + synchronize (host <-> GPU round trip floor)
x = torch.zeros(16, device=dev)
for _ in range(20):
    x.add_(1)
    torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(300):
    x.add_(1)
    torch.cuda.synchronize()
print(f"torch tiny op + sync {(time.perf_counter() - t) / 300 * 1e6:8.1f} us", flush=True)
# PCIe-inclusive rate: the same batch from host memory (ym_merge with YM_MEM_HOST: H2D of the arena and
# offsets, the kernels, D2H of the outputs) through Engine.run_host
for _ in range(3):
    eng.run_host("merge", fmt, a, o, d)
t = time.perf_counter()
for _ in range(20):
    eng.run_host("merge", fmt, a, o, d)
el = (time.perf_counter() - t) / 20
print(f"host batch (PCIe-inclusive) {el * 1e3:8.3f} ms/call = {int(o[-1]) / el / 1e9:6.2f} GB/s of input", flush=True)
