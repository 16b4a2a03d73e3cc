"""GPU parity: every golden vector through libymerge.so (C ABI) on the MI355X, batched per
(op, format) group so one launch covers hundreds of documents.  Expected bytes / errors come from
yjs 13.5.16 itself (tests/golden, recipes oracle/gen/make_*fixtures.cjs), with no exceptions: every
vector must come out byte-identical (or with the same error), including the payload re-encodings of
tests/golden/canon.json."""
import collections

import numpy as np
import pytest

import golden_io
import oracle_ref as O

pytestmark = pytest.mark.gpu

CASES = [c for c in golden_io.load_cases() if not (c["op"] == "merge" and len(c["inputs"]) == 0)]


@pytest.fixture(scope="module")
def engine():
    from yjs_amd import Engine
    return Engine(0)


def _groups():
    g = collections.defaultdict(list)
    for c in CASES:
        g[(c["op"], c["fmt"])].append(c)
    return g


@pytest.mark.parametrize("key", sorted(_groups().keys()), ids=lambda k: f"{k[0]}-v{k[1]}")
def test_golden_batched_on_gpu(engine, key):
    _check_group(engine, key)


@pytest.mark.parametrize("ms", ["", "2"], ids=["stitch", "ms-stitch"])
@pytest.mark.parametrize("key", [("diff", 1), ("sv", 1), ("meta", 1), ("diff", 2), ("sv", 2), ("meta", 2)],
                         ids=lambda k: f"{k[0]}-v{k[1]}")
def test_golden_through_chunked_walk(engine, key, ms, monkeypatch):
    """The chunk-parallel V1 walk (ym_pwalk.hip) and the column-parallel V2 paths (ym_pv2.hip single section,
    ym_pv2ms.hip several sections) normally take updates of >= 32 KB only; with their threshold at 1 byte every
    golden diff / state-vector / meta vector goes through them (fallback to the sequential walkers on a decline)
    and must still come out byte-identical.  ms-stitch: the V1 documents of >= 2 sections through the
    section-parallel stitch (k_pw_ms, off by default)."""
    if ms and key[1] == 2:
        pytest.skip("the section-parallel stitch is V1 only")
    monkeypatch.setenv("YMERGE_PW_MIN", "1")
    if ms:
        monkeypatch.setenv("YMERGE_PWMS_MIN", ms)
    _check_group(engine, key)
    if key[1] == 1:  # the V1 walk accepts what the sequential walker accepts, except nested payloads (objects /
        # arrays in ContentAny, integer / object JSON formats: checked out of line by the sequential walker only)
        assert 0 < engine.stats["docs_chunked"] <= engine.stats["docs_fast"], engine.stats
    else:  # the V2 paths (one section: String / Deleted / GC; several: XML / format / any content too)
        assert engine.stats["docs_chunked"] > 0, engine.stats


def test_golden_v2_diff_through_lane_kernel(engine, monkeypatch):
    """k_diff_small_v2 (one update per lane, ym_fast2.hip) runs on batches of more than 8,192 documents only;
    with YMERGE_DF2_MIN=0 every golden V2 diff goes through it first (declines fall back to k_big_v2) and must
    come out byte-identical.  (Many vectors are outside its acceptance on purpose: non-ASCII strings, Skip / GC /
    JSON content, repeated clients; those decline and take the walker.)"""
    import ctypes
    monkeypatch.setenv("YMERGE_DF2_MIN", "0")
    _check_group(engine, ("diff", 2))
    n = len(_groups()[("diff", 2)])
    done = np.zeros(n, np.uint8)
    assert engine.lib.ym__pv2_done(done.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), ctypes.c_uint32(n)) == 0
    assert (done == 1).sum() >= n // 8, np.unique(done, return_counts=True)


def _check_group(engine, key):
    from yjs_amd import pack_docs
    cases = _groups()[key]
    op, fmt = key
    if op in ("merge", "dsmerge", "dsmerge_ref"):  # k inputs per document
        arena, upd_off, doc_upd = pack_docs([c["inputs"] for c in cases])
        res = engine.run_host(op, fmt, arena, upd_off, doc_upd)
    elif op == "diff":
        arena, upd_off, doc_upd = pack_docs([[c["inputs"][0]] for c in cases])
        sva, svo, _ = pack_docs([[c["sv"]] for c in cases])
        res = engine.run_host("diff", fmt, arena, upd_off, doc_upd, sva, svo)
    else:  # sv, conv, meta: one update per document
        arena, upd_off, doc_upd = pack_docs([[c["inputs"][0]] for c in cases])
        res = engine.run_host(op, fmt, arena, upd_off, doc_upd)
    out_arena, out_off, out_len, status = res
    bad = []
    for i, c in enumerate(cases):
        st = int(status[i])
        if "error" in c:
            why = O.js_error_mismatch(st, c["error"], c["message"])
            if why:
                bad.append((c["id"], "error", why))
            continue
        got = out_arena[int(out_off[i]):int(out_off[i]) + int(out_len[i])].tobytes() if st == 0 else None
        if st != 0 or got != c["expect"]:
            bad.append((c["id"], "bytes", st, len(got or b""), len(c["expect"])))
    assert not bad, bad[:20]


def test_pref_bytes_on_gpu(engine):
    """The engine's bytes are the ones gaberogan/yjs@v0 itself was checked against (P-ref, tests/pref)."""
    import hashlib
    import json
    import os
    from yjs_amd import pack_docs
    pref = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "pref", "pref.json")))
    gold = {c["id"]: c for c in CASES}  # (zero-input merges are answered by the host layer, not a kernel)
    for op in ("merge", "sv", "diff"):
        for fmt in (1, 2):
            sel = [c for c in pref["cases"] if c["op"] == op and c["fmt"] == fmt and c.get("applicable") and c["id"] in gold]
            docs = [gold[c["id"]]["inputs"] if op == "merge" else [gold[c["id"]]["inputs"][0]] for c in sel]
            extra = pack_docs([[gold[c["id"]]["sv"]] for c in sel])[:2] if op == "diff" else ()
            oa, oo, ol, st = engine.run_host(op, fmt, *pack_docs(docs), *extra)
            for i, c in enumerate(sel):
                got = oa[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes()
                assert st[i] == 0 and hashlib.sha256(got).hexdigest() == c["checked_sha256"], c["id"]


@pytest.mark.parametrize("fmt", [1, 2])
def test_golden_meta_update_log_shape(engine, fmt):
    """parseUpdateMeta[V2] of an update log (> 65,536 single-update documents: the lane-per-update kernels,
    ym_small.hip / ym_fast2.hip k_meta_v2, with their declines on the general path): every golden meta
    vector, repeated to that batch size, byte-identical (or the same error) in every copy."""
    from yjs_amd import pack_docs
    cases = _groups()[("meta", fmt)]
    reps = 65536 // len(cases) + 2
    arena, upd_off, doc_upd = pack_docs([[c["inputs"][0]] for c in cases] * reps)
    out_arena, out_off, out_len, status = engine.run_host("meta", fmt, arena, upd_off, doc_upd)
    bad = []
    for i in range(len(status)):
        c = cases[i % len(cases)]
        st = int(status[i])
        if "error" in c:
            why = O.js_error_mismatch(st, c["error"], c["message"])
            if why:
                bad.append((i, c["id"], why))
            continue
        got = out_arena[int(out_off[i]):int(out_off[i]) + int(out_len[i])].tobytes() if st == 0 else None
        if st != 0 or got != c["expect"]:
            bad.append((i, c["id"], st))
    assert not bad, bad[:20]
    assert engine.stats["docs_fast"] > 0, engine.stats


def test_tiny_inputs_one_document_per_call(engine):
    """Every golden merge / delete-set merge with at most 16 input bytes as a call of its own (the Node API's
    shape: each document alone, its bytes at offset 0 of the arena), with u64 and u32 offsets.  A document of no
    bytes at all (one empty delete set, empty updates) once made k_fast_merge_v1's staging load a vector at index
    2^32 - 1 (an illegal address that ended the process's GPU context)."""
    from yjs_amd import pack_docs
    cases = [c for c in CASES if c["op"] in ("merge", "dsmerge", "dsmerge_ref") and len(c["inputs"]) > 0
             and sum(len(x) for x in c["inputs"]) <= 16]
    assert any(sum(len(x) for x in c["inputs"]) == 0 for c in cases)
    bad = []
    for c in cases:
        for off32 in (False, True):
            arena, upd_off, doc_upd = pack_docs([c["inputs"]])
            if off32:
                upd_off = upd_off.astype(np.uint32)
            out_arena, out_off, out_len, status = engine.run_host(c["op"], c["fmt"], arena, upd_off, doc_upd)
            st = int(status[0])
            if "error" in c:
                why = O.js_error_mismatch(st, c["error"], c["message"])
                if why:
                    bad.append((c["id"], off32, why))
                continue
            got = out_arena[int(out_off[0]):int(out_off[0]) + int(out_len[0])].tobytes() if st == 0 else None
            if got != c["expect"]:
                bad.append((c["id"], off32, st))
    assert not bad, bad[:20]
