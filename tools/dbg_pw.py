"""Debug aid for the chunk-parallel V1 walk: runs the golden diff / sv V1 vectors with the walk's size
threshold at 1 byte and prints, per decline reason (ym_pwalk.hip `why`), how many documents and a few
case ids, next to the sequential walker's acceptance of the same documents."""
import collections
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import golden_io  # noqa: E402
from yjs_amd import Engine, pack_docs  # noqa: E402

eng = Engine(0)
cases = golden_io.load_cases()
for op in ("diff", "sv"):
    sel = [c for c in cases if c["op"] == op and c["fmt"] == 1]
    a, o, d = pack_docs([[c["inputs"][0]] for c in sel])
    extra = ()
    if op == "diff":
        sva, svo, _ = pack_docs([[c["sv"]] for c in sel])
        extra = (sva, svo)
    os.environ.pop("YMERGE_PW_MIN", None)
    eng.run_host(op, 1, a, o, d, *extra)
    base = dict(eng.stats)
    os.environ["YMERGE_PW_MIN"] = "1"
    eng.run_host(op, 1, a, o, d, *extra)
    st = dict(eng.stats)
    r = np.zeros(len(sel), dtype=np.uint8)
    eng.lib.ym__pw_reasons(r.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(len(sel)))
    print(op, "docs", len(sel), "normal fast", base["docs_fast"], "general", base["docs_general"],
          "| pw mode fast", st["docs_fast"], "chunked", st["docs_chunked"])
    byr = collections.defaultdict(list)
    for i, c in enumerate(sel):
        byr[int(r[i])].append(c["id"])
    for k in sorted(byr):
        print("  reason", k, len(byr[k]), byr[k][:6])
