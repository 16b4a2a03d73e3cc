"""Doc round-trip compaction fixtures (tests/golden/compact.json, oracle/gen/make_compact_fixtures.cjs):
gaberogan/yjs@v0 (yjs 13.4.9) new Doc() (gc: true), applyUpdate[V2] of every input in order,
encodeStateAsUpdate[V2].  Workload documents name their bench_data source and carry the expected output's
SHA-256 instead of its bytes."""
import base64
import functools
import hashlib
import json
import os

from yjs_amd.workloads import load_ymb

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "compact.json")


@functools.lru_cache(maxsize=None)
def _ymb(name):
    return load_ymb(name)


@functools.lru_cache(maxsize=1)
def load():
    with open(PATH) as f:
        d = json.load(f)
    out = []
    for c in d["cases"]:
        if "src" in c:
            arena, upd_off, doc_upd = _ymb(c["src"]["ymb"])
            k = c["src"]["doc"]
            ins = [arena[int(upd_off[u]):int(upd_off[u + 1])].tobytes() for u in range(int(doc_upd[k]), int(doc_upd[k + 1]))]
            exp = None
        else:
            ins = [base64.b64decode(x) for x in c["inputs"]]
            exp = base64.b64decode(c["expect"])
        out.append(dict(id=c["id"], group=c["group"], fmt=c["fmt"], inputs=ins, expect=exp,
                        sha=c.get("expect_sha256"), elen=c.get("expect_len")))
    return out


def matches(case, got):
    if got is None:
        return False
    if case["expect"] is not None:
        return got == case["expect"]
    return len(got) == case["elen"] and hashlib.sha256(got).hexdigest() == case["sha"]
