"""GPU parity of Doc round-trip compaction (ym_compact): the HIP kernel
(ym_compact.hip, one document per lane) against the reference's own outputs (tests/golden/compact.json,
oracle/gen/make_compact_fixtures.cjs: gaberogan/yjs@v0 applyUpdate x N + encodeStateAsUpdate on a gc=true
Doc) and, at workload scale, against the oracle's restatement (oracle/ymerge_oracle.c compact_impl)."""
import numpy as np
import pytest

import compact_cases
import oracle_ref as O
from yjs_amd.workloads import load_ymb

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from yjs_amd import Engine
    return Engine(0)


@pytest.mark.parametrize("lanes", ["1", "16", "64"])
@pytest.mark.parametrize("fmt", [1, 2])
def test_compact_fixtures_on_gpu(engine, fmt, lanes, monkeypatch):
    """Every fixture of the reference, including the histories it leaves pending (gapped workload documents,
    lost / late messages: only the integrated store is written) and the inputs on which it throws (class and
    message), at 1, 16 (the default) and 64 documents per wave (the library reads YMERGE_COMPACT_LANES on
    every call)."""
    from yjs_amd import pack_docs
    monkeypatch.setenv("YMERGE_COMPACT_LANES", lanes)
    # (the C5 workload documents, ~45 s per format at one lane each, run once in test_compact_c5_documents)
    cs = [c for c in compact_cases.load() if c["fmt"] == fmt and c["group"] not in ("gap_c5", "wl_c5")]
    a, o, d = pack_docs([c["inputs"] for c in cs])
    oa, oo, ol, st = engine.run_host("compact", fmt, a, o, d)
    bad = []
    for i, c in enumerate(cs):
        got = oa[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() if st[i] == 0 else None
        why = compact_cases.mismatch(c, st[i], got)
        if why:
            bad.append((c["id"], why))
    assert not bad, f"{len(bad)}/{len(cs)} differ: {bad[:8]}"
    assert sum(1 for c in cs if c["pending"]) > 60 and sum(1 for c in cs if c["error"]) > 0


@pytest.mark.parametrize("fmt", [1, 2])
def test_compact_nogc_fixtures_on_gpu(engine, fmt):
    """YM_NO_GC: every gc: false fixture of the reference (new Y.Doc({ gc: false }), deleted content kept).
    (Its C5 workload document is pinned through the host build, tests/test_compact.py: one lane each.)"""
    from yjs_amd import pack_docs
    cs = [c for c in compact_cases.load(nogc=True) if c["fmt"] == fmt and c["group"] != "wl_c5"]
    a, o, d = pack_docs([c["inputs"] for c in cs])
    oa, oo, ol, st = engine.run_host("compact_nogc", fmt, a, o, d)
    bad = []
    for i, c in enumerate(cs):
        got = oa[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() if st[i] == 0 else None
        why = compact_cases.mismatch(c, st[i], got)
        if why:
            bad.append((c["id"], why))
    assert not bad, f"{len(bad)}/{len(cs)} differ: {bad[:8]}"
    assert sum(1 for c in cs if c["differs"]) > 200


@pytest.mark.parametrize("gc", [True, False], ids=["gc", "nogc"])
@pytest.mark.parametrize("fmt", [1, 2])
def test_compact_target_sv_fixtures_on_gpu(engine, fmt, gc):
    """ym_compact with a target state vector per document (encodeStateAsUpdate[V2](doc, sv)): every target
    fixture of the reference -- empty / full / prefix / random / repeated / past-the-state vectors, each
    clock of the slice documents (surrogate pairs cut by str.slice), malformed vectors.  (The C5 workload
    document's targets, one lane each at HBM latency, are pinned through the host build of the same device
    code, tests/test_compact.py.)"""
    from yjs_amd import pack_docs
    cs = [c for c in compact_cases.load_sv() if c["fmt"] == fmt and c["gc"] == gc and c["group"] != "wl_c5"]
    a, o, d = pack_docs([c["inputs"] for c in cs])
    sa, so, _ = pack_docs([[c["sv"]] for c in cs])
    oa, oo, ol, st = engine.run_host("compact" if gc else "compact_nogc", fmt, a, o, d, sa, so)
    bad = []
    for i, c in enumerate(cs):
        got = oa[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() if st[i] == 0 else None
        why = compact_cases.mismatch(c, st[i], got)
        if why:
            bad.append((c["id"], why))
    assert not bad, f"{len(bad)}/{len(cs)} differ: {bad[:8]}"
    assert len(cs) > 400


@pytest.mark.parametrize("name", ["c2_v1", "c2_v2", "c4_v1"])
def test_compact_workload_matches_oracle(engine, name):
    """Every template document of the C2 / C4 workloads (bench_data/) compacted on the GPU equals the
    oracle's restatement byte for byte, and its state vector equals the merged update's."""
    from yjs_amd import pack_docs
    fmt = 2 if name.endswith("v2") else 1
    arena, upd_off, doc_upd = load_ymb(name)
    n = min(len(doc_upd) - 1, 200)
    docs = [[arena[int(upd_off[u]):int(upd_off[u + 1])].tobytes() for u in range(int(doc_upd[i]), int(doc_upd[i + 1]))]
            for i in range(n)]
    a, o, d = pack_docs(docs)
    oa, oo, ol, st = engine.run_host("compact", fmt, a, o, d)
    assert (st == 0).all(), np.unique(st)
    for i in range(n):
        s, want = O.compact(docs[i], fmt)
        assert s == 0
        assert oa[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() == want, i
    assert engine.stats["docs_general"] == n  # one kernel (ym_compact.hip) took every document


def test_compact_c5_documents(engine):
    """The large C5 documents (1,024 clients, ~16 k updates, nested XML types): workspace growth on the device
    (ST_RETRY rounds) and the fixture hashes of the reference; and the gapped C5 documents (every 5th update
    dropped: ~1,000 clients' structs and ~1,500 delete readers left pending, re-examined by the reference on
    every update -- on the device only the readers a client's new state can wake, ym_compact.h pdel_watch)."""
    from yjs_amd import pack_docs
    # (documents above YMERGE_COMPACT_BIG input bytes get a wave each: the four run side by side)
    cs = [c for c in compact_cases.load() if c["group"] in ("wl_c5", "gap_c5")]
    assert sum(c["group"] == "gap_c5" for c in cs) >= 4
    for fmt in (1, 2):
        sub = [c for c in cs if c["fmt"] == fmt]
        a, o, d = pack_docs([c["inputs"] for c in sub])
        oa, oo, ol, st = engine.run_host("compact", fmt, a, o, d)
        for i, c in enumerate(sub):
            assert compact_cases.mismatch(c, st[i], oa[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes()) is None, c["id"]


def test_compact_workspace_budget_chunks(engine, monkeypatch):
    """A batch whose workspaces exceed the device-memory budget runs in chunks (YMERGE_COMPACT_WS_GB, read
    on every call) with the same bytes as one launch; a document whose workspace alone exceeds the budget
    reports YM_ERR_CAPACITY without affecting the others."""
    from yjs_amd import pack_docs
    arena, upd_off, doc_upd = load_ymb("c2_v1")
    n = 300
    docs = [[arena[int(upd_off[u]):int(upd_off[u + 1])].tobytes() for u in range(int(doc_upd[i]), int(doc_upd[i + 1]))]
            for i in range(n)]
    a, o, d = pack_docs(docs)
    oa, oo, ol, st = engine.run_host("compact", 1, a, o, d)
    assert (st == 0).all()
    want = [oa[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() for i in range(n)]
    monkeypatch.setenv("YMERGE_COMPACT_WS_GB", "0.01")  # ~10 MB: ~27 documents per chunk
    oa, oo, ol, st = engine.run_host("compact", 1, a, o, d)
    assert (st == 0).all()
    assert [oa[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() for i in range(n)] == want
    # one C5 document (0.7 MB of updates: a workspace of tens of MB) between small ones
    big = [c for c in compact_cases.load() if c["group"] == "wl_c5" and c["fmt"] == 1][0]
    a, o, d = pack_docs([docs[0], big["inputs"], docs[1]])
    oa, oo, ol, st = engine.run_host("compact", 1, a, o, d)
    assert int(st[1]) == 9 and int(st[0]) == 0 and int(st[2]) == 0  # YM_ERR_CAPACITY
    assert oa[int(oo[0]):int(oo[0]) + int(ol[0])].tobytes() == want[0]
    assert oa[int(oo[2]):int(oo[2]) + int(ol[2])].tobytes() == want[1]


@pytest.mark.parametrize("gc", [True, False], ids=["gc", "nogc"])
@pytest.mark.parametrize("fmt", [1, 2])
def test_compact_doc_state_vector_on_gpu(engine, fmt, gc):
    """YM_SV_FIRST on the GPU: the compacted Doc's encodeStateVector (StructStore insertion order) before the
    update, against the reference's bytes for every fixture of compact.json / compact_nogc.json, the gapped C5
    documents included (gc=True: compact.json's gap_c5 group); the wl_c5 group's state vectors (~45 s per
    format on one lane per document) are checked through the host build of the same device code only
    (tests/test_compact.py)."""
    from yjs_amd import pack_docs
    cs = [c for c in compact_cases.load(nogc=not gc) if c["fmt"] == fmt and c["group"] != "wl_c5"]
    a, o, d = pack_docs([c["inputs"] for c in cs])
    oa, oo, ol, st = engine.run_host("compact_sv" if gc else "compact_nogc_sv", fmt, a, o, d)
    bad = []
    for i, c in enumerate(cs):
        got = oa[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() if st[i] == 0 else None
        why = compact_cases.mismatch_sv_first(c, st[i], got)
        if why:
            bad.append((c["id"], why))
    assert not bad, f"{len(bad)}/{len(cs)} differ: {bad[:8]}"
