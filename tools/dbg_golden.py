"""Debug helper: runs golden cases on the GPU (by id, or all of an op/format: `diff:2`) and prints
where the bytes differ."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from golden_io import load_cases  # noqa: E402
from yjs_amd import Engine, pack_docs  # noqa: E402

eng = Engine(0)
cases = []
for sel in sys.argv[1:]:
    if ":" in sel and "/" not in sel:
        op, fmt = sel.split(":")
        cases += [x for x in load_cases() if x["op"] == op and x["fmt"] == int(fmt) and "expect" in x]
    else:
        cases += [x for x in load_cases() if x["id"] == sel]
shown = 0
for c in cases:
    a, o, d = pack_docs([c["inputs"]])
    extra = ()
    if c["op"] == "diff":
        sa, so, _ = pack_docs([[c["sv"]]])
        extra = (sa, so)
    oa, oo, ol, st = eng.run_host(c["op"], c["fmt"], a, o, d, *extra)
    got = oa[int(oo[0]):int(oo[0]) + int(ol[0])].tobytes()
    exp = c["expect"]
    if got == exp:
        continue
    diffs = [i for i in range(min(len(got), len(exp))) if got[i] != exp[i]]
    print(c["id"], "status", int(st[0]), "len", len(got), len(exp), "ndiff", len(diffs), diffs[:12], eng.stats["docs_fast"])
    print("  got", got[:120].hex())
    print("  exp", exp[:120].hex())
    print("  in ", c["inputs"][0][:120].hex(), "sv", c["sv"].hex() if "sv" in c else "")
    shown += 1
    if shown >= 4:
        break
print("checked", len(cases))
