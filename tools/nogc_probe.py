"""Probe: ym_compact (YM_NO_GC) over every gc: false fixture with inputs, as js/test/golden.js calls it (one host
batch per format, the C5 workload documents included): call return code, bytes used, per-status counts, time."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import compact_cases  # noqa: E402
from yjs_amd import Engine, pack_docs  # noqa: E402

eng = Engine(0)
for fmt in (1, 2):
    cs = [c for c in compact_cases.load(nogc=True) if c["fmt"] == fmt and c.get("inputs")]
    a, o, d = pack_docs([c["inputs"] for c in cs])
    t = time.time()
    try:
        oa, oo, ol, st = eng.run_host("compact_nogc", fmt, a, o.astype(np.uint32) if os.environ.get("OFF32") else o, d)
        bad = [c["id"] for i, c in enumerate(cs) if compact_cases.mismatch(c, st[i], oa[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() if st[i] == 0 else None)]
        print(fmt, len(cs), "ok", "%.1fs" % (time.time() - t), dict(zip(*np.unique(st, return_counts=True))), "bad", bad[:5], flush=True)
    except Exception as e:
        print(fmt, len(cs), "raised", repr(e), "%.1fs" % (time.time() - t), flush=True)
