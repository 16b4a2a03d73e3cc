"""Doc round-trip compaction fixtures (tests/golden/compact.json, oracle/gen/make_compact_fixtures.cjs):
gaberogan/yjs@v0 (yjs 13.4.9) new Doc() (gc: true), applyUpdate[V2] of every input in order,
encodeStateAsUpdate[V2].  Workload documents name their bench_data source (`drop`: every drop-th update
left out, a gapped history) and carry the expected output's SHA-256 instead of its bytes.  Cases on which the
reference throws carry the exception (`error`: class and message) instead of bytes; `pending` records what the
reference's store still held pending after the last input (such documents compact to the integrated store
only)."""
import base64
import functools
import hashlib
import json
import os

from yjs_amd.workloads import load_ymb

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "compact.json")
# new Y.Doc({ gc: false }) over the same inputs (oracle/gen/make_compact_nogc_fixtures.cjs; ym_compact with YM_NO_GC)
PATH_NOGC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "compact_nogc.json")


# encodeStateAsUpdate[V2](doc, targetStateVector) (oracle/gen/make_compact_sv_fixtures.cjs; ym_compact with
# ym_batch.sv_arena)
PATH_SV = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "compact_sv.json")


@functools.lru_cache(maxsize=None)
def _ymb(name):
    return load_ymb(name)


@functools.lru_cache(maxsize=2)
def load(nogc=False):
    with open(PATH_NOGC if nogc else PATH) as f:
        d = json.load(f)
    out = []
    for c in d["cases"]:
        if "src" in c:
            arena, upd_off, doc_upd = _ymb(c["src"]["ymb"])
            k = c["src"]["doc"]
            ins = [arena[int(upd_off[u]):int(upd_off[u + 1])].tobytes() for u in range(int(doc_upd[k]), int(doc_upd[k + 1]))]
            drop = c["src"].get("drop")
            if drop:
                ins = [u for i, u in enumerate(ins) if i % drop != drop - 1]
            exp = None
        else:
            ins = [base64.b64decode(x) for x in c["inputs"]]
            exp = base64.b64decode(c["expect"]) if "expect" in c else None
        out.append(dict(id=c["id"], group=c["group"], fmt=c["fmt"], inputs=ins, expect=exp,
                        sha=c.get("expect_sha256"), elen=c.get("expect_len"), error=c.get("error"),
                        pending=c.get("pending"), differs=c.get("differs_from_gc"),
                        docsv=base64.b64decode(c["sv"]) if "sv" in c else None))
    return out


def matches(case, got):
    if got is None or case["error"]:
        return False
    if case["expect"] is not None:
        return got == case["expect"]
    return len(got) == case["elen"] and hashlib.sha256(got).hexdigest() == case["sha"]


def mismatch_sv_first(case, status, got):
    """mismatch() of a YM_SV_FIRST output: the reference's encodeStateVector(doc), then its update bytes."""
    if case["error"] or int(status) != 0 or got is None:
        return mismatch(case, status, got)
    from yjs_amd.engine import split_state_vector
    sv, rest = split_state_vector(got)
    if sv != case["docsv"]:
        return "state vector differs"
    return mismatch(case, status, rest)


def mismatch(case, status, got, message=True):
    """None if (status, bytes) is the reference's result for `case`, else the reason.  Error cases: the
    status word's class is the exception's class and (message=True: the engine, whose status word carries
    which message) ym_strerror's text is the exception's message."""
    import oracle_ref
    st = int(status)
    if case["error"]:
        e = case["error"]
        if st == 0:
            return "no error, reference threw " + e["name"]
        if message:
            return oracle_ref.js_error_mismatch(st, e["name"], e["message"])
        want = oracle_ref.js_error_status(e["name"], e["message"])
        return None if st & 0xff == want else f"class {st & 0xff} != {want}"
    if st != 0:
        return f"status {st:#x}"
    return None if matches(case, got) else "bytes differ"


@functools.lru_cache(maxsize=1)
def load_sv():
    """Target-state-vector fixtures, one entry per (document, target): the document's inputs (an inline
    case of compact.json named by `ref`, a workload document, or the generator's own "slice" documents),
    gc, the encoded target state vector and the reference's output (bytes or SHA-256) or exception."""
    base = {c["id"]: c for c in load()}
    with open(PATH_SV) as f:
        d = json.load(f)
    out = []
    for c in d["cases"]:
        if "ref" in c:
            ins = base[c["ref"]]["inputs"]
            cid = c["ref"]
        else:
            ins = [base64.b64decode(x) for x in c["inputs"]]
            cid = c["id"]
        for i, t in enumerate(c["targets"]):
            out.append(dict(id=f"{cid}/{t['kind']}{i}", group=c["group"], fmt=c["fmt"], gc=c["gc"], inputs=ins,
                            sv=base64.b64decode(t["sv"]), kind=t["kind"],
                            expect=base64.b64decode(t["expect"]) if "expect" in t else None,
                            sha=t.get("expect_sha256"), elen=t.get("expect_len"), error=t.get("error"),
                            pending=None, differs=None))
    return out
