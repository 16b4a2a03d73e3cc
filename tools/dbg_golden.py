"""Debug helper: runs named golden cases on the GPU and prints where the bytes differ."""
import sys
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from golden_io import load_cases  # noqa: E402
from yjs_amd import Engine, pack_docs  # noqa: E402

eng = Engine(0)
for cid in sys.argv[1:]:
    c = [x for x in load_cases() if x["id"] == cid][0]
    a, o, d = pack_docs([c["inputs"]])
    extra = ()
    if c["op"] == "diff":
        sa, so, _ = pack_docs([[c["sv"]]])
        extra = (sa, so)
    oa, oo, ol, st = eng.run_host(c["op"], c["fmt"], a, o, d, *extra)
    got = oa[int(oo[0]):int(oo[0]) + int(ol[0])].tobytes()
    exp = c["expect"]
    diffs = [i for i in range(min(len(got), len(exp))) if got[i] != exp[i]]
    print(cid, "status", int(st[0]), "len", len(got), len(exp), "ndiff", len(diffs), diffs[:20], eng.stats)
    for i in diffs[:5]:
        print("  at", i, "got", got[max(0, i - 8):i + 8].hex(), "exp", exp[max(0, i - 8):i + 8].hex())
