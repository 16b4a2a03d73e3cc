"""Runs the compaction fixtures (tests/golden/compact.json) through the host build of ym_compact.h
(tests/native/core_host.cpp, op 7) and prints per-group pass counts and the first failures."""
import collections
import sys

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import compact_cases  # noqa: E402
import core_host  # noqa: E402
from yjs_amd import pack_docs  # noqa: E402

cases = compact_cases.load()
only = sys.argv[1] if len(sys.argv) > 1 else None
res = collections.defaultdict(lambda: [0, 0])
bad = []
for fmt in (1, 2):
    cs = [c for c in cases if c["fmt"] == fmt and (not only or c["group"].startswith(only))]
    if not cs:
        continue
    a, o, d = pack_docs([c["inputs"] for c in cs])
    outs, st = core_host.run("compact", fmt, a, o, d, san="san" in sys.argv)
    for c, out, s in zip(cs, outs, st):
        ok = s == 0 and compact_cases.matches(c, out)
        res[c["group"]][0 if ok else 1] += 1
        if not ok:
            bad.append((c["id"], int(s), len(out) if out else None, c["elen"] or (len(c["expect"]) if c["expect"] else None)))
for g, (p, f) in sorted(res.items()):
    print(f"{g:12s} pass {p:4d} fail {f:4d}")
for b in bad[:25]:
    print(b)
