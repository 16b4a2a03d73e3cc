"""Per-wave timeline of one k_fast_merge_v1 launch (the YM_FAST_TIMELINE diagnostics build,
tools/build_variant.sh tl ym_fast.hip <src> -DYM_FAST_TIMELINE): wave durations, how many waves run at once
over the launch, and how long the tail is.  Usage: YMERGE_LIB=.../libymerge_tl.so python tools/fast_timeline.py"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from yjs_amd import Engine  # noqa: E402
from yjs_amd.workloads import load_ymb, replicate  # noqa: E402

wl = os.environ.get("WL", "c2_v1")
a, o, d = replicate(*load_ymb(wl), int(os.environ.get("NDOCS", "10000")))
dev = torch.device("cuda", 0)
ga = torch.from_numpy(a).to(dev)
go = torch.from_numpy(o.astype(np.uint32).view(np.int32)).to(dev)
gd = torch.from_numpy(d.view(np.int32)).to(dev)
n = len(d) - 1
oa = torch.empty(4 * len(a) + 128 * n + 8192, dtype=torch.uint8, device=dev)
oo = torch.empty(n, dtype=torch.int64, device=dev)
ol = torch.empty(n, dtype=torch.int64, device=dev)
st = torch.empty(n, dtype=torch.int32, device=dev)
e = Engine(0)
for _ in range(5):
    rc, _ = e.run_device("merge", 1, ga, go, gd, oa, oo, ol, st)
    assert rc == 0, rc
torch.cuda.synchronize()
grid = (n + 7) & ~7
buf = np.zeros((grid, 4), np.uint64)
e.lib.ym__fast_timeline(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), ctypes.c_int(grid))
t0, t1 = buf[:, 0].astype(np.int64), buf[:, 1].astype(np.int64)
live = t1 > 0
t0, t1 = t0[live], t1[live]
base = t0.min()
s, f = (t0 - base) / 100.0, (t1 - base) / 100.0  # us (100 MHz)
dur = f - s
hw = buf[live, 2]
hwid = (hw & 0xffffffff).astype(np.int64)
simd = (hwid >> 4) & 3
cu = (hwid >> 8) & 15
se = (hwid >> 13) & 7
xcc = (hw >> 32).astype(np.int64) & 15
unit = ((xcc * 8 + se) * 16 + cu) * 4 + simd
print(f"{wl}: {live.sum()} waves, span {f.max():.1f} us, units {len(np.unique(unit))}")
print("wave duration us: p10 %.1f p50 %.1f p90 %.1f max %.1f mean %.1f" % tuple(np.percentile(dur, [10, 50, 90, 100]).tolist() + [dur.mean()]))
print("start us: p50 %.1f p90 %.1f p99 %.1f max %.1f" % tuple(np.percentile(s, [50, 90, 99, 100])))
ts = np.linspace(0, f.max(), 41)
conc = [int(((s <= t) & (f > t)).sum()) for t in ts]
print("waves running at t (us):")
for t, c in zip(ts, conc):
    print(f"  {t:7.1f} {c:6d} " + "#" * (c // 200))
per_unit = np.bincount(unit, minlength=unit.max() + 1)
per_unit = per_unit[per_unit > 0]
print("waves per SIMD: min %d max %d mean %.2f" % (per_unit.min(), per_unit.max(), per_unit.mean()))
busy_end = np.zeros(unit.max() + 1)
np.maximum.at(busy_end, unit, f)
be = busy_end[busy_end > 0]
print("SIMD last-wave end us: p10 %.1f p50 %.1f p90 %.1f" % tuple(np.percentile(be, [10, 50, 90])))
k = np.diff(d.astype(np.int64))
ob = o.astype(np.int64)
db = ob[d[1:].astype(np.int64)] - ob[d[:-1].astype(np.int64)]
docs_ = buf[live, 3].astype(np.int64)
bb = db[np.minimum(docs_, n - 1)]
q = np.percentile(bb, [25, 50, 75])
gen2 = s > 5.0
print("first generation: %d waves, mean duration %.1f us; later: %d waves, mean %.1f us, mean start %.1f" %
      ((~gen2).sum(), dur[~gen2].mean(), gen2.sum(), dur[gen2].mean(), s[gen2].mean()))
for lo, hi in ((0, q[0]), (q[0], q[1]), (q[1], q[2]), (q[2], 1e9)):
    m = (bb > lo) & (bb <= hi)
    print(f"doc bytes ({lo:.0f},{hi:.0f}]: gen1 mean {dur[m & ~gen2].mean():.1f} us, later mean {dur[m & gen2].mean():.1f} us")
np.save(os.path.join(ROOT, "gpurun_out", "fast_tl_%s.npy" % wl), np.stack([s, f, unit, docs_, bb]).T)
docs = buf[live, 3].astype(np.int64)
kk = k[np.minimum(docs, n - 1)]
for lo, hi in ((0, 64), (64, 96), (96, 129)):
    m = (kk > lo) & (kk <= hi)
    if m.any():
        print(f"updates in ({lo},{hi}]: {m.sum()} waves, mean duration {dur[m].mean():.1f} us")

if hasattr(e.lib, "ym__fast_phases"):
    ph = np.zeros((grid, 8), np.uint32)
    e.lib.ym__fast_phases(ph.ctypes.data_as(ctypes.POINTER(ctypes.c_uint)), ctypes.c_int(grid))
    ph = ph[live].astype(np.int64)
    st0 = (buf[live, 0] & 0xffffffff).astype(np.int64)
    en = (buf[live, 1] & 0xffffffff).astype(np.int64)
    pts = np.concatenate([st0[:, None], ph[:, :7], en[:, None]], axis=1)
    pts = np.maximum.accumulate(pts, axis=1)  # a phase a document skipped takes no time
    dt = np.diff(pts, axis=1) / 100.0
    names = ["stage", "W1", "sort", "layout", "emit", "W2", "ds merge", "ds emit"]
    for nm, g1, g2 in zip(names, dt[~gen2].mean(0), dt[gen2].mean(0)):
        print(f"  {nm:9s} gen1 {g1:6.2f} us   later {g2:6.2f} us")
