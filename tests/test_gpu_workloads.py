"""GPU parity on the benchmark workloads: the engine's batched mergeUpdates/diffUpdate/
encodeStateVectorFromUpdate (V1 and V2) over yjs-generated C2 / C4 / C3 documents must equal the
oracle's bytes document by document, and the fast path must actually take the C2/C4 V1 documents."""
import numpy as np
import pytest

import oracle_ref as O
from yjs_amd.workloads import load_ymb, random_state_vectors

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from yjs_amd import Engine
    return Engine(0)


def _compare(res, outs, status):
    out_arena, out_off, out_len, st = res
    bad = []
    for d in range(len(st)):
        if int(st[d]) & 0xff != int(status[d]):  # (the engine adds the exception detail above bit 7)
            bad.append((d, "status", int(st[d]), int(status[d])))
            continue
        if st[d] == 0:
            got = out_arena[int(out_off[d]):int(out_off[d]) + int(out_len[d])].tobytes()
            if got != outs[d]:
                bad.append((d, "bytes", len(got), len(outs[d])))
    return bad


@pytest.mark.parametrize("name", ["c2_v1", "c2_v2", "c4_v1", "c4_v2", "c1_v1", "c1_v2", "c2r_v1", "c2r_v2", "c4r_v1", "c4r_v2",
                                  "c2u_v1", "c2u_v2"])
def test_merge_workload_matches_oracle(engine, name):
    arena, upd_off, doc_upd = load_ymb(name)
    fmt = 2 if name.endswith("v2") else 1
    outs, status, _ = O.batch("merge", fmt, arena, upd_off, doc_upd, nthreads=8)
    res = engine.run_host("merge", fmt, arena, upd_off, doc_upd)
    bad = _compare(res, outs, status)
    assert not bad, bad[:10]
    st = engine.stats
    if name in ("c2_v1", "c4_v1", "c2_v2", "c4_v2", "c2u_v1", "c2u_v2"):
        assert st["docs_fast"] == st["docs"], st  # every C2/C4 (and C2U) doc takes the LDS fast path (V1 and V2)


@pytest.mark.parametrize("fmt", [1, 2])
def test_sv_and_diff_workload_matches_oracle(engine, fmt):
    arena, upd_off, doc_upd = load_ymb(f"c2_v{fmt}")
    merged, status, _ = O.batch("merge", fmt, arena, upd_off, doc_upd, nthreads=8)
    assert (status == 0).all()
    from yjs_amd import pack_docs
    a2, o2, d2 = pack_docs([[m] for m in merged])
    outs, st, _ = O.batch("sv", fmt, a2, o2, d2, nthreads=8)
    bad = _compare(engine.run_host("sv", fmt, a2, o2, d2), outs, st)
    assert not bad, bad[:10]
    assert engine.stats["docs_fast"] == engine.stats["docs"], engine.stats  # streamed wave walker
    svs = []
    for i, m in enumerate(merged):
        svs.extend(random_state_vectors(outs[i], 1, seed=i))
    sva, svo, _ = pack_docs([[s] for s in svs])
    outs2, st2, _ = O.batch("diff", fmt, a2, o2, d2, sva, svo, nthreads=8)
    bad = _compare(engine.run_host("diff", fmt, a2, o2, d2, sva, svo), outs2, st2)
    assert not bad, bad[:10]
    assert engine.stats["docs_fast"] == engine.stats["docs"], engine.stats


@pytest.mark.parametrize("op", ["sv", "meta"])
@pytest.mark.parametrize("fmt", [1, 2])
def test_c3_sv_matches_oracle(engine, fmt, op):
    arena, upd_off, doc_upd = load_ymb(f"c3_v{fmt}")
    from yjs_amd import pack_docs
    upd = arena.tobytes()
    a2, o2, d2 = pack_docs([[upd] for _ in range(4)])
    outs, st, _ = O.batch(op, fmt, a2, o2, d2)
    bad = _compare(engine.run_host(op, fmt, a2, o2, d2), outs, st)
    assert not bad, bad[:10]
    assert engine.stats["docs_fast"] == engine.stats["docs"], engine.stats
    # the chunk-parallel walk (V1) / column-parallel path (V2) takes every C3 update
    assert engine.stats["docs_chunked"] == engine.stats["docs"], engine.stats


@pytest.mark.parametrize("fmt", [1, 2])
def test_c3_diff_random_svs(engine, fmt):
    arena, upd_off, doc_upd = load_ymb(f"c3_v{fmt}")
    upd = arena.tobytes()
    _, st0, _ = O.batch("sv", fmt, arena, upd_off, doc_upd)
    svo_full = O.sv_from_update(upd, fmt)[1]
    svs = random_state_vectors(svo_full, 8, seed=3)
    from yjs_amd import pack_docs
    a2, o2, d2 = pack_docs([[upd] for _ in svs])
    sva, svo, _ = pack_docs([[s] for s in svs])
    outs, st, _ = O.batch("diff", fmt, a2, o2, d2, sva, svo, nthreads=8)
    bad = _compare(engine.run_host("diff", fmt, a2, o2, d2, sva, svo), outs, st)
    assert not bad, bad[:10]
    assert engine.stats["docs_fast"] == engine.stats["docs"], engine.stats
    assert engine.stats["docs_chunked"] == engine.stats["docs"], engine.stats


def test_lane_parser_short_cut_agrees(engine):
    """The chunk walk's branch-free short cut (ym_lane.h parse_fast) decides most structs; wherever it
    decides -- at every byte position of real V1 updates (C3, merged C2 / C5 / C4 documents) and of random
    bytes -- it must agree with the full parser exactly (next position, clock length, flags)."""
    import ctypes
    from yjs_amd import pack_docs
    bufs = [load_ymb("c3_v1")[0].tobytes()]
    for name in ("c2_v1", "c5_v1", "c4_v1"):
        a, o, d = load_ymb(name)
        docs = [[a[int(o[u]):int(o[u + 1])].tobytes() for u in range(int(d[i]), int(d[i + 1]))] for i in range(2)]
        ma, mo, ml, mst = engine.run_host("merge", 1, *pack_docs(docs))
        bufs += [ma[int(mo[i]):int(mo[i]) + int(ml[i])].tobytes() for i in range(2)]
    bufs.append(np.random.default_rng(1).integers(0, 256, 1 << 20, dtype=np.uint8).tobytes())
    decided = 0
    for b in bufs:
        out = (ctypes.c_ulonglong * 2)()
        assert engine.lib.ym__lane_selftest(b, ctypes.c_uint32(len(b)), out) == 0
        assert out[1] == 0, (len(b), out[0], out[1])
        decided += out[0]
    assert decided > 100000


@pytest.mark.parametrize("fmt", [1, 2])
def test_c3_damaged_updates_chunked_walk(engine, fmt):
    """Truncated and byte-flipped C3 updates through the chunk-parallel walk (V1) / column-parallel path
    (V2): wherever the damage lands (struct section or columns, a string, the delete set) the result must
    be the oracle's -- the same bytes or the same exception -- whether the path declines the document or not."""
    arena, upd_off, doc_upd = load_ymb(f"c3_v{fmt}")
    upd = arena.tobytes()
    rng = np.random.default_rng(11 + fmt)
    docs, svs = [], []
    svo_full = O.sv_from_update(upd, fmt)[1]
    full_svs = random_state_vectors(svo_full, 24, seed=5)
    for i in range(24):
        b = bytearray(upd)
        if i % 3 == 0:
            b = b[:int(rng.integers(len(b) // 2, len(b)))]
        else:
            for _ in range(1 + i % 4):
                b[int(rng.integers(8, len(b)))] = int(rng.integers(0, 256))
        docs.append(bytes(b))
        svs.append(full_svs[i])
    from yjs_amd import pack_docs
    a2, o2, d2 = pack_docs([[u] for u in docs])
    sva, svo, _ = pack_docs([[s] for s in svs])
    for op in ("diff", "sv", "meta"):
        extra = (sva, svo) if op == "diff" else ()
        outs, st, _ = O.batch(op, fmt, a2, o2, d2, *extra, nthreads=8)
        bad = _compare(engine.run_host(op, fmt, a2, o2, d2, *extra), outs, st)
        assert not bad, (op, bad[:10])


@pytest.mark.parametrize("fmt", [1, 2])
def test_c5_damaged_updates_chunked_walk(engine, fmt):
    """Truncated and byte-flipped merged C5 updates (~1,000 client sections each: V1 through the chunk walk's
    pre-roll and the stitch's LDS state-vector map, V2 through the multi-section column path): the oracle's
    bytes or exception for every document, whether the path takes it or declines it."""
    from yjs_amd import pack_docs
    arena, upd_off, doc_upd = load_ymb(f"c5_v{fmt}")
    merged, status, _ = O.batch("merge", fmt, arena, upd_off, doc_upd, nthreads=8)
    assert (status == 0).all()
    rng = np.random.default_rng(23 + fmt)
    docs, svs = [], []
    for i in range(16):
        b = bytearray(merged[i % len(merged)])
        if i % 4 == 0:
            b = b[:int(rng.integers(len(b) // 2, len(b)))]
        elif i % 4 != 3:  # (every 4th document undamaged)
            for _ in range(1 + i % 3):
                b[int(rng.integers(8, len(b)))] = int(rng.integers(0, 256))
        docs.append(bytes(b))
        svs.append(random_state_vectors(O.sv_from_update(merged[i % len(merged)], fmt)[1], 1, seed=40 + i)[0])
    a2, o2, d2 = pack_docs([[u] for u in docs])
    sva, svo, _ = pack_docs([[s] for s in svs])
    for op in ("diff", "sv", "meta"):
        extra = (sva, svo) if op == "diff" else ()
        outs, st, _ = O.batch(op, fmt, a2, o2, d2, *extra, nthreads=8)
        bad = _compare(engine.run_host(op, fmt, a2, o2, d2, *extra), outs, st)
        assert not bad, (op, bad[:10])


def _subset(arena, upd_off, doc_upd, docs, keep):
    """Documents `docs` of a template file, each restricted to the updates u (local index) with keep(u)."""
    from yjs_amd import pack_docs
    out = []
    for d in docs:
        u0, u1 = int(doc_upd[d]), int(doc_upd[d + 1])
        out.append([arena[int(upd_off[u]):int(upd_off[u + 1])].tobytes() for u in range(u0, u1) if keep(u - u0)])
    return pack_docs(out)


@pytest.mark.parametrize("fmt", [1, 2])
def test_large_merge_c5_matches_oracle(engine, fmt):
    """configs[4] C5 (1,024 clients, ~16 k updates per document): the large-document pipeline."""
    arena, upd_off, doc_upd = load_ymb(f"c5_v{fmt}")
    outs, status, _ = O.batch("merge", fmt, arena, upd_off, doc_upd, nthreads=8)
    bad = _compare(engine.run_host("merge", fmt, arena, upd_off, doc_upd), outs, status)
    assert not bad, bad[:10]
    st = engine.stats
    assert st["docs_large"] == st["docs"], st


@pytest.mark.parametrize("fmt", [1, 2])
def test_large_merge_gaps_matches_oracle(engine, fmt):
    """Dropped updates leave clock gaps: Skips inside client parts, delete sets of absent structs."""
    arena, upd_off, doc_upd = load_ymb(f"c5_v{fmt}")
    a, o, d = _subset(arena, upd_off, doc_upd, range(4), lambda u: u % 5 != 3)
    outs, status, _ = O.batch("merge", fmt, a, o, d, nthreads=8)
    bad = _compare(engine.run_host("merge", fmt, a, o, d), outs, status)
    assert not bad, bad[:10]
    assert engine.stats["docs_large"] == 4, engine.stats


@pytest.mark.parametrize("fmt", [1, 2])
def test_large_merge_mixed_batch(engine, fmt):
    """One batch of small (fast path), large (pipeline) and overlapping (general path) documents:
    C2 docs, C5 docs cut to 3,000 updates, and two C2 docs concatenated (same clients: overlaps)."""
    from yjs_amd import pack_docs
    a2, o2, d2 = load_ymb(f"c2_v{fmt}")
    a5, o5, d5 = load_ymb(f"c5_v{fmt}")
    docs = []
    upd = lambda a, o, u: a[int(o[u]):int(o[u + 1])].tobytes()
    for i in range(6):
        docs.append([upd(a2, o2, u) for u in range(int(d2[i]), int(d2[i + 1]))])
        docs.append([upd(a5, o5, u) for u in range(int(d5[i % 8]), int(d5[i % 8]) + 3000)])
    docs.append(docs[0] + docs[2])
    docs.append([upd(a2, o2, u) for u in range(int(d2[7]), int(d2[9]))])
    a, o, d = pack_docs(docs)
    outs, status, _ = O.batch("merge", fmt, a, o, d, nthreads=8)
    bad = _compare(engine.run_host("merge", fmt, a, o, d), outs, status)
    assert not bad, bad[:10]
    st = engine.stats
    assert st["docs_fast"] == 6 and st["docs_large"] == 6, st


@pytest.mark.parametrize("fmt", [1, 2])
def test_c5_sv_and_diff_many_clients(engine, fmt):
    """configs[4] diffUpdate[V2] / encodeStateVectorFromUpdate[V2] over merged C5 documents (one update
    of ~1,000 client parts each) against random per-client state vectors: the streamed wave walkers
    (section / state-vector / delete-set tables in per-block HBM scratch) must take every document."""
    from yjs_amd import pack_docs
    arena, upd_off, doc_upd = load_ymb(f"c5_v{fmt}")
    merged, status, _ = O.batch("merge", fmt, arena, upd_off, doc_upd, nthreads=8)
    assert (status == 0).all()
    a2, o2, d2 = pack_docs([[m] for m in merged])
    outs, st, _ = O.batch("sv", fmt, a2, o2, d2, nthreads=8)
    bad = _compare(engine.run_host("sv", fmt, a2, o2, d2), outs, st)
    assert not bad, bad[:10]
    assert engine.stats["docs_fast"] == engine.stats["docs"], engine.stats
    svs = []
    for i in range(len(merged)):
        svs.extend(random_state_vectors(outs[i], 2, seed=100 + i))
    a3, o3, d3 = pack_docs([[merged[i // 2]] for i in range(len(svs))])
    sva, svo, _ = pack_docs([[s] for s in svs])
    outs2, st2, _ = O.batch("diff", fmt, a3, o3, d3, sva, svo, nthreads=8)
    bad = _compare(engine.run_host("diff", fmt, a3, o3, d3, sva, svo), outs2, st2)
    assert not bad, bad[:10]
    assert engine.stats["docs_fast"] == engine.stats["docs"], engine.stats
    if fmt == 2:  # the multi-section column path (ym_pv2ms.hip) takes every merged C5 document
        assert engine.stats["docs_chunked"] == engine.stats["docs"], engine.stats


def test_state_does_not_leak_between_calls(engine):
    """A large diff (big bump allocation) followed by a tiny merge on the same engine: the second call's
    allocator starts clean (regression: a stale device counter made the merge report CAPACITY)."""
    from yjs_amd import pack_docs
    arena, upd_off, doc_upd = load_ymb("c3_v1")
    upd = arena.tobytes()
    a2, o2, d2 = pack_docs([[upd] for _ in range(8)])
    sva, svo, _ = pack_docs([[b"\x00"] for _ in range(8)])
    _, _, _, st = engine.run_host("diff", 1, a2, o2, d2, sva, svo)
    assert (st == 0).all()
    a, o, d = load_ymb("c2_v1")
    docs = [[a[int(o[u]):int(o[u + 1])].tobytes() for u in range(int(d[0]), int(d[1]))]]
    a3, o3, d3 = pack_docs(docs)
    outs, status, _ = O.batch("merge", 1, a3, o3, d3)
    bad = _compare(engine.run_host("merge", 1, a3, o3, d3), outs, status)
    assert not bad, bad


@pytest.mark.parametrize("fmt", [1, 2])
def test_convert_workloads_match_oracle(engine, fmt):
    """convertUpdateFormatV1ToV2 / V2ToV1 (13.5.x convertUpdateFormat) over merged C2 and C5 documents
    and over the raw C4 updates, against the oracle (pinned by tests/golden/conv.json)."""
    from yjs_amd import pack_docs
    ups = []
    for wl in (f"c2_v{fmt}", f"c5_v{fmt}"):
        a, o, d = load_ymb(wl)
        if wl.startswith("c2"):
            a, o, d = pack_docs([[a[int(o[u]):int(o[u + 1])].tobytes() for u in range(int(d[i]), int(d[i + 1]))]
                                 for i in range(64)])
        merged, st, _ = O.batch("merge", fmt, a, o, d, nthreads=8)
        ups += [m for m, s in zip(merged, st) if s == 0]
    a, o, d = load_ymb(f"c4_v{fmt}")
    ups += [a[int(o[u]):int(o[u + 1])].tobytes() for u in range(0, 2000)]
    a2, o2, d2 = pack_docs([[u] for u in ups])
    outs, st, _ = O.batch("conv", fmt, a2, o2, d2, nthreads=8)
    assert (st == 0).all()
    bad = _compare(engine.run_host("conv", fmt, a2, o2, d2), outs, st)
    assert not bad, bad[:10]


def _vu(v):
    out = bytearray()
    while v > 127:
        out.append(0x80 | (v & 127))
        v >>= 7
    out.append(v)
    return bytes(out)


def _ds_update(ranges):
    """A V1 update with no structs and the delete set {client: [(clock, len), ...]} (DeleteSet.js:219-232)."""
    b = bytearray(b"\x00")
    b += _vu(len(ranges))
    for client, rs in ranges.items():
        b += _vu(client) + _vu(len(rs))
        for clock, ln in rs:
            b += _vu(clock) + _vu(ln)
    return bytes(b)


@pytest.mark.parametrize("fmt", [1, 2])
def test_delete_set_merges_duplicates_and_large_clocks(engine, fmt):
    """Delete-set-only updates with equal (client, clock) ranges across inputs (the common case the fast
    path's slot-tagged keys handle) and documents with clocks >= 2^25 (declined to the general path):
    bytes equal the oracle's and only the large-clock documents leave the fast path."""
    from yjs_amd import pack_docs
    rng = np.random.default_rng(5)
    docs, big = [], []
    for d in range(96):
        large = d % 4 == 3
        clients = [int(c) for c in rng.choice([7, 300, 123456, 2**31 + 5], size=2, replace=False)]
        # disjoint ranges (V2 delta-codes clocks against the previous range's end); updates pick
        # overlapping subsets of them, so equal (client, clock) keys recur across inputs
        base = [(8 * int(k) + (2**25 if large else 0), int(rng.integers(1, 6)))
                for k in rng.choice(12, size=6, replace=False)]
        # one struct (Y.Text insert of "ab" by client 99, ykey "t"): the fast path takes documents with structs
        ups = [bytes([1, 1, 99, 0, 0x04, 1, 1, ord("t"), 2, ord("a"), ord("b"), 0])]
        for _ in range(int(rng.integers(2, 9))):
            sel = {}
            for c in clients:
                picks = rng.choice(len(base), size=int(rng.integers(1, 4)), replace=False)
                sel[c] = sorted(base[int(i)] for i in picks)
            ups.append(_ds_update(sel))
        if fmt == 2:
            ups = [O.convert(u, 1)[1] for u in ups]
        docs.append(ups)
        big.append(large)
    a, o, d = pack_docs(docs)
    outs, status, _ = O.batch("merge", fmt, a, o, d)
    assert (status == 0).all()
    bad = _compare(engine.run_host("merge", fmt, a, o, d), outs, status)
    assert not bad, bad[:10]
    st = engine.stats
    assert st["docs_fast"] == len(docs) - sum(big), st


@pytest.mark.parametrize("fmt", [1, 2])
def test_meta_workloads_match_oracle(engine, fmt):
    """parseUpdateMeta[V2] over the raw C2 updates (~1 M single updates, each one client section or a
    few) and over merged C2 / C5 documents (4 and ~1,000 client sections): engine == oracle per update."""
    from yjs_amd import pack_docs
    arena, upd_off, doc_upd = load_ymb(f"c2_v{fmt}")
    n_upd = int(doc_upd[1000])  # the first 1,000 documents' updates, one per batch document
    a1, o1 = arena[:int(upd_off[n_upd])], upd_off[:n_upd + 1]
    d1 = np.arange(n_upd + 1, dtype=np.uint32)
    outs, st, _ = O.batch("meta", fmt, a1, o1, d1, nthreads=8)
    bad = _compare(engine.run_host("meta", fmt, a1, o1, d1), outs, st)
    assert not bad, bad[:10]
    for name in (f"c2_v{fmt}", f"c5_v{fmt}"):
        arena, upd_off, doc_upd = load_ymb(name)
        if name.startswith("c5"):  # merged by the engine (C5 merges are checked against the oracle above)
            oa, oo, ol, ost = engine.run_host("merge", fmt, arena, upd_off, doc_upd)
            assert (ost == 0).all()
            merged = [oa[int(oo[d]):int(oo[d]) + int(ol[d])].tobytes() for d in range(len(ost))]
        else:
            merged, status, _ = O.batch("merge", fmt, arena, upd_off, doc_upd, nthreads=8)
            assert (status == 0).all()
        a2, o2, d2 = pack_docs([[m] for m in merged])
        outs, st, _ = O.batch("meta", fmt, a2, o2, d2, nthreads=8)
        assert (st == 0).all()
        bad = _compare(engine.run_host("meta", fmt, a2, o2, d2), outs, st)
        assert not bad, (name, bad[:10])
        # the streamed walkers (ym_big.hip / ym_big2.hip, meta mode) take every merged document
        assert engine.stats["docs_fast"] == engine.stats["docs"], engine.stats


def _encode_ds(clients, v2):
    out = bytearray(_vu(len(clients)))
    for client, items in clients:
        out += _vu(client) + _vu(len(items))
        cur = 0
        for clock, ln in items:
            if v2:
                out += _vu(clock - cur) + _vu(ln - 1)
                cur = clock + ln
            else:
                out += _vu(clock) + _vu(ln)
    return bytes(out)


@pytest.mark.parametrize("fmt", [1, 2])
def test_ds_merge_batch_matches_oracle(engine, fmt):
    """PermanentUserData's delete-set merge over 20,000 documents of 1..48 encoded delete sets each
    (64 clients, overlapping / touching / duplicated intervals, clocks up to 2^32 - 1)."""
    from yjs_amd import pack_docs
    rng = np.random.default_rng(77 + fmt)
    docs = []
    for d in range(20000):
        k = int(rng.integers(1, 49)) if d % 50 else int(rng.integers(0, 3))
        blobs = []
        for _ in range(k):
            cl = []
            for client in rng.choice(64, size=int(rng.integers(0, 5)), replace=False):
                base = 4294967000 if client == 63 else 0
                n = int(rng.integers(0, 6))
                starts = np.sort(rng.integers(0, 200, size=n))
                items, end = [], -1
                for s in starts:
                    s = int(s) + base
                    if fmt == 2 and s < end:
                        continue  # a DSEncoderV2 writes clocks in order (delta coded)
                    ln = int(rng.integers(1, 8))
                    items.append((s, ln))
                    end = s + ln
                cl.append((int(client) * 7919 + 1, items))
            blobs.append(_encode_ds(cl, fmt == 2))
        docs.append(blobs)
    a, o, dd = pack_docs(docs)
    outs, status, _ = O.batch("dsmerge", fmt, a, o, dd, nthreads=8)
    assert (status == 0).all()
    bad = _compare(engine.run_host("dsmerge", fmt, a, o, dd), outs, status)
    assert not bad, bad[:10]
    st = engine.stats
    # the fast kernel (delete-set-only mode) takes the documents that fit its LDS tables
    assert st["docs_fast"] > 0.3 * st["docs"], st  # (the rest: > 128 ranges or clocks >= 2^25)


def _run_device_u32(engine, op, fmt, arena, upd_off, doc_upd):
    """run_device with the batch resident on cuda:0 and the update offsets as u32 (YM_OFF32)."""
    import torch
    dev = torch.device("cuda", 0)
    nd = len(doc_upd) - 1
    ga = torch.from_numpy(np.ascontiguousarray(arena)).to(dev)
    go = torch.from_numpy(upd_off.astype(np.uint32).view(np.int32)).to(dev)
    gd = torch.from_numpy(doc_upd.view(np.int32)).to(dev)
    oa = torch.empty(4 * len(arena) + 128 * nd + 8192, dtype=torch.uint8, device=dev)
    oo = torch.empty(nd, dtype=torch.int64, device=dev)
    ol = torch.empty(nd, dtype=torch.int64, device=dev)
    st = torch.empty(nd, dtype=torch.int32, device=dev)
    rc, _ = engine.run_device(op, fmt, ga, go, gd, oa, oo, ol, st)
    assert rc == 0, rc
    return oa.cpu().numpy(), oo.cpu().numpy(), ol.cpu().numpy(), st.cpu().numpy()


@pytest.mark.parametrize("name", ["c2_v1", "c4_v1", "c2_v2", "c5_v1"])
def test_device_batch_u32_offsets(engine, name):
    """Device-resident batches with u32 update offsets (YM_OFF32): the V1 fast kernel reads them directly,
    every other path (V2 fast kernel, large-document pipeline) after the on-device widening."""
    arena, upd_off, doc_upd = load_ymb(name)
    fmt = 2 if name.endswith("v2") else 1
    outs, status, _ = O.batch("merge", fmt, arena, upd_off, doc_upd, nthreads=8)
    bad = _compare(_run_device_u32(engine, "merge", fmt, arena, upd_off, doc_upd), outs, status)
    assert not bad, bad[:10]


def test_device_u32_offsets_mixed_paths(engine):
    """YM_OFF32 with documents the fast kernel declines (general path after widening): golden merges."""
    import golden_io
    cases = [c for c in golden_io.load_cases() if c["op"] == "merge" and c["fmt"] == 1 and len(c["inputs"]) > 0]
    from yjs_amd import pack_docs
    a, o, d = pack_docs([c["inputs"] for c in cases])
    oa, oo, ol, st = _run_device_u32(engine, "merge", 1, a, o, d)
    bad = []
    for i, c in enumerate(cases):
        if "error" in c:
            if O.js_error_mismatch(st[i], c["error"], c["message"]):
                bad.append(c["id"])
        elif st[i] != 0 or oa[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() != c["expect"]:
            bad.append(c["id"])
    assert not bad, bad[:10]
    assert engine.stats["docs_general"] > 0, engine.stats


def _many_client_update(clients, ds):
    """A V1 update with one two-character Y.Text insert per client (descending client order, clock 0;
    no origin, parent ykey "t") and the delete set `ds` = [(client, [(clock, len), ...]), ...]."""
    b = bytearray(_vu(len(clients)))
    for c in clients:
        b += _vu(1) + _vu(c) + _vu(0) + bytes([0x04, 1, 1, ord("t"), 2, ord("a"), ord("b")])
    return bytes(b + _encode_ds(ds, False))


@pytest.mark.parametrize("pw_min", ["1", None], ids=["chunked", "streamed"])
@pytest.mark.parametrize("fmt", [1, 2])
def test_client_map_many_clients(engine, fmt, pw_min, monkeypatch):
    """Above 64 state-vector entries / delete-set clients the walkers look clients up in a per-block hash
    map (ym_cmap.h) instead of scanning the list: state vectors with 65-300 entries, repeated clients
    (decodeStateVector: the later entry wins) and absent ones; delete sets of 65-200 clients, some with a
    client repeated (readDeleteSet merges it: the walkers must decline to the general path).  Diff, state
    vector and meta through the chunk walk / column path (threshold 1 byte) and the streamed walkers."""
    if pw_min:
        monkeypatch.setenv("YMERGE_PW_MIN", pw_min)
    from yjs_amd import pack_docs
    rng = np.random.default_rng(31 + fmt)
    docs, svs = [], []
    for d in range(48):
        nc = int(rng.integers(65, 200))
        clients = sorted((int(c) for c in rng.choice(10**6, size=nc, replace=False)), reverse=True)
        nd = int(rng.integers(65, 200)) if d % 3 else int(rng.integers(1, 8))
        ds = [(int(c), [(0, 1)] if i % 2 else [(0, 1), (3, 2)]) for i, c in enumerate(rng.choice(10**6, size=nd, replace=False))]
        if d % 4 == 1:  # a repeated delete-set client
            ds.append((ds[int(rng.integers(0, len(ds)))][0], [(9, 1)]))
        u = _many_client_update(clients if fmt == 1 or d % 8 else clients[:1], ds)
        if fmt == 2:
            u = O.convert(u, 1)[1]
        docs.append(u)
        sv = [(c, int(rng.integers(0, 3))) for c in rng.choice(clients, size=min(nc, int(rng.integers(60, 300))))]
        sv += [(int(c), 5) for c in rng.integers(10**6, 2 * 10**6, size=8)]  # absent clients
        rng.shuffle(sv)
        svs.append(_vu(len(sv)) + b"".join(_vu(int(c)) + _vu(k) for c, k in sv))
    a, o, dd = pack_docs([[u] for u in docs])
    sva, svo, _ = pack_docs([[s] for s in svs])
    for op in ("diff", "sv", "meta"):
        extra = (sva, svo) if op == "diff" else ()
        outs, st, _ = O.batch(op, fmt, a, o, dd, *extra, nthreads=8)
        bad = _compare(engine.run_host(op, fmt, a, o, dd, *extra), outs, st)
        assert not bad, (op, bad[:10])


def _cmap_hash(c):
    return ((c * 0x9E3779B1) & 0xFFFFFFFF) >> 20  # ym_cmap.h hash over 4,096 slots


def _colliding_clients(rng, n):
    """n distinct client ids sharing one client-map slot (long probe chains)."""
    target = _cmap_hash(12345)
    out = []
    while len(out) < n:
        c = [int(x) for x in rng.integers(0, 2**32, size=1 << 16, dtype=np.uint64)]
        out += [x for x in c if _cmap_hash(x) == target and x not in out]
    return out[:n]


@pytest.mark.parametrize("pw_min", ["1", None], ids=["chunked", "streamed"])
@pytest.mark.parametrize("fmt", [1, 2])
def test_client_map_boundary_keys(engine, fmt, pw_min, monkeypatch):
    """The client map's boundary keys: clients 0, 0xFFFFFFFE and 0xFFFFFFFF (whose client + 1 key would
    wrap to the empty marker) in the struct section, the state vector and the delete set (also repeated),
    clients whose hashes all land on one slot (probe chains of ~100), and delete sets of ~2,000 clients
    (near BS_NDSC).  Diff, state vector and meta against the oracle."""
    if pw_min:
        monkeypatch.setenv("YMERGE_PW_MIN", pw_min)
    from yjs_amd import pack_docs
    rng = np.random.default_rng(57 + fmt)
    edge = [0, 0xFFFFFFFE, 0xFFFFFFFF]
    coll = _colliding_clients(rng, 160)
    docs, svs = [], []
    for d in range(24):
        pool = coll if d % 2 else [int(c) for c in rng.choice(10**6, size=150, replace=False)]
        clients = sorted(set(pool[:int(rng.integers(70, 150))] + edge[:1 + d % 3]), reverse=True)
        if d % 6 == 5:
            nd = int(rng.integers(1900, 2040))
            dsc = [int(c) for c in rng.choice(2**31, size=nd, replace=False)] + edge
        else:
            dsc = pool[::-1][:int(rng.integers(65, 140))] + edge[d % 3:]
        ds = [(c, [(0, 1)] if i % 2 else [(0, 1), (3, 2)]) for i, c in enumerate(dsc)]
        if d % 4 == 1:  # repeated delete-set client: 0xFFFFFFFF itself, or a colliding one
            ds.append((0xFFFFFFFF if d % 8 == 1 else ds[int(rng.integers(0, len(ds)))][0], [(9, 1)]))
        u = _many_client_update(clients if fmt == 1 or d % 8 else clients[:1], ds)
        if fmt == 2:
            u = O.convert(u, 1)[1]
        docs.append(u)
        sv = [(c, int(rng.integers(0, 3))) for c in rng.choice(clients, size=min(len(clients), int(rng.integers(66, 200))))]
        sv += [(c, int(rng.integers(0, 3))) for c in edge for _ in range(1 + d % 2)]  # later entry wins
        sv += [(int(c), 5) for c in coll[150:]]  # absent clients on the same probe chain
        rng.shuffle(sv)
        svs.append(_vu(len(sv)) + b"".join(_vu(int(c)) + _vu(k) for c, k in sv))
    a, o, dd = pack_docs([[u] for u in docs])
    sva, svo, _ = pack_docs([[s] for s in svs])
    for op in ("diff", "sv", "meta"):
        extra = (sva, svo) if op == "diff" else ()
        outs, st, _ = O.batch(op, fmt, a, o, dd, *extra, nthreads=8)
        bad = _compare(engine.run_host(op, fmt, a, o, dd, *extra), outs, st)
        assert not bad, (op, bad[:10])


@pytest.mark.parametrize("how", ["hash", "bytes"])
def test_multi_device_engine_real_engine(how):
    """MultiDeviceEngine with the real Engine on two worker threads bound to device 0 (the 1-GPU box's
    stand-in for two GPUs): per-(thread, device) library state (ym_api.hip g_states) driven from two
    threads at once, over a mixed batch of C2 (fast path) and C5 (large pipeline) documents, merged and
    then diffed against random state vectors; results in docIndex order against the oracle, repeated
    calls reuse each thread's state (device memory flat after the first call)."""
    import torch
    from yjs_amd import pack_docs
    from yjs_amd.distributed import MultiDeviceEngine
    a2, o2, d2 = load_ymb("c2_v1")
    a5, o5, d5 = load_ymb("c5_v1")
    upd = lambda a, o, u: a[int(o[u]):int(o[u + 1])].tobytes()
    docs = [[upd(a2, o2, u) for u in range(int(d2[i]), int(d2[i + 1]))] for i in range(60)]
    for i in range(4):
        docs.insert(7 + 13 * i, [upd(a5, o5, u) for u in range(int(d5[i]), int(d5[i + 1]))])
    a, o, d = pack_docs(docs)
    ref, st, _ = O.batch("merge", 1, a, o, d, nthreads=8)
    assert (st == 0).all()
    ma, mo, md = pack_docs([[m] for m in ref])
    svs = []
    for i, m in enumerate(ref):
        svs.extend(random_state_vectors(O.sv_from_update(m, 1)[1], 1, seed=i))
    sva, svo, _ = pack_docs([[s] for s in svs])
    dref, dst, _ = O.batch("diff", 1, ma, mo, md, sva, svo, nthreads=8)
    dexp = [x if s == 0 else int(s) for x, s in zip(dref, dst)]
    free = []
    with MultiDeviceEngine([0, 0], how) as eng:
        for it in range(3):
            assert eng.run_host("merge", 1, a, o, d) == list(ref)
            got = eng.run_host("diff", 1, ma, mo, md, sva, svo)
            assert [g if isinstance(g, bytes) else g & 0xff for g in got] == dexp
            torch.cuda.synchronize()
            free.append(torch.cuda.mem_get_info(0)[0])
    assert abs(free[2] - free[1]) < (64 << 20), free  # no per-call leak of streams / scratch


@pytest.mark.parametrize("name", ["c2r_v1", "c2r_v2", "c4r_v1", "c4r_v2"])
def test_rich_content_stays_on_the_specialised_paths(engine, name):
    """Rich content (number / object formats, image embeds, maps of objects and arrays: the C2R / C4R
    templates) through the LDS merges, then the merged documents' state vectors and diffs against random
    state vectors through the streamed walkers: equal to the oracle, and no document on the general path
    (nested `any` values and JSON texts are checked canonical, ym_canon_chk.h, and copied)."""
    from yjs_amd import pack_docs
    fmt = 2 if name.endswith("v2") else 1
    arena, upd_off, doc_upd = load_ymb(name)
    n = 400
    docs = [[arena[int(upd_off[u]):int(upd_off[u + 1])].tobytes() for u in range(int(doc_upd[i]), int(doc_upd[i + 1]))]
            for i in range(n)]
    a, o, d = pack_docs(docs)
    outs, status, _ = O.batch("merge", fmt, a, o, d, nthreads=8)
    bad = _compare(engine.run_host("merge", fmt, a, o, d), outs, status)
    assert not bad, bad[:10]
    assert engine.stats["docs_general"] == 0, engine.stats
    # the LDS merge kernels' retry pass with nested payload checks takes most of them (the rest: inputs
    # over the kernels' staging size, to the large-document pipeline)
    assert engine.stats["docs_fast"] >= 0.6 * n, engine.stats
    a2, o2, d2 = pack_docs([[m] for m in outs])
    svo, sst, _ = O.batch("sv", fmt, a2, o2, d2, nthreads=8)
    bad = _compare(engine.run_host("sv", fmt, a2, o2, d2), svo, sst)
    assert not bad, bad[:10]
    assert engine.stats["docs_general"] == 0, engine.stats
    svs = [random_state_vectors(svo[i], 1, seed=i)[0] for i in range(n)]
    sva, svoff, _ = pack_docs([[s] for s in svs])
    douts, dst, _ = O.batch("diff", fmt, a2, o2, d2, sva, svoff, nthreads=8)
    bad = _compare(engine.run_host("diff", fmt, a2, o2, d2, sva, svoff), douts, dst)
    assert not bad, bad[:10]
    assert engine.stats["docs_general"] == 0, engine.stats


@pytest.mark.parametrize("name", ["c2r_v2", "c4r_v2", "c4_v2"])
def test_v2_small_kernels_rich_and_wide_match_oracle(engine, name, monkeypatch):
    """The V2 lane-per-document kernels (k_diff_small_v2 forced at this batch size with YMERGE_DF2_MIN=0;
    k_small_v2 for state vectors) over merged rich (Quill formats / embeds, maps of objects and arrays) and
    wide (64-client) documents against random state vectors: every document byte-identical to the oracle,
    whichever kernel completes it (the lane kernels or, for what they decline, k_big_v2)."""
    import ctypes
    from yjs_amd import pack_docs
    monkeypatch.setenv("YMERGE_DF2_MIN", "0")
    arena, upd_off, doc_upd = load_ymb(name)
    n = min(len(doc_upd) - 1, 600)
    doc_upd = doc_upd[:n + 1].copy()
    merged, status, _ = O.batch("merge", 2, arena, upd_off, doc_upd, nthreads=8)
    assert (status == 0).all()
    a2, o2, d2 = pack_docs([[m] for m in merged])
    outs, st, _ = O.batch("sv", 2, a2, o2, d2, nthreads=8)
    bad = _compare(engine.run_host("sv", 2, a2, o2, d2), outs, st)
    assert not bad, bad[:10]
    svs = []
    for i in range(n):
        svs.extend(random_state_vectors(outs[i], 1, seed=100 + i))
    sva, svo, _ = pack_docs([[s] for s in svs])
    outs2, st2, _ = O.batch("diff", 2, a2, o2, d2, sva, svo, nthreads=8)
    bad = _compare(engine.run_host("diff", 2, a2, o2, d2, sva, svo), outs2, st2)
    assert not bad, bad[:10]
    done = np.zeros(n, np.uint8)
    assert engine.lib.ym__pv2_done(done.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), ctypes.c_uint32(n)) == 0
    if name == "c2r_v2":  # most rich text documents are within the lane kernel's acceptance
        assert (done == 1).sum() > n // 2, np.unique(done, return_counts=True)


@pytest.mark.parametrize("fmt", [1, 2])
def test_merge_nested_first_adapts(engine, fmt):
    """Merge batches of mostly rich documents make the next calls start with the nested LDS pass (per format,
    re-probed with the hot pass every 16 calls); a plain batch after them, and every call in between, must
    still give the oracle's bytes."""
    rich = load_ymb(f"c2r_v{fmt}")
    plain = load_ymb(f"c2_v{fmt}")
    want = {}
    for name, (arena, upd_off, doc_upd) in (("rich", rich), ("plain", plain)):
        n = min(len(doc_upd) - 1, 300)
        d = doc_upd[:n + 1].copy()
        want[name] = (arena, upd_off, d) + O.batch("merge", fmt, arena, upd_off, d, nthreads=8)[:2]
    seq = ["rich"] * 18 + ["plain", "plain", "rich", "plain"]
    for i, name in enumerate(seq):
        arena, upd_off, d, outs, status = want[name]
        bad = _compare(engine.run_host("merge", fmt, arena, upd_off, d), outs, status)
        assert not bad, (i, name, bad[:5])


@pytest.mark.parametrize("fmt", [1, 2])
def test_c2u_realistic_text_matches_oracle(engine, fmt):
    """C2U (the C2 shape with CJK / emoji / accented words and 20-200 character pastes, bench_data/c2u_*):
    merges, state vectors and diffs against random state vectors (which cut some emoji in half: yjs's
    URIError) equal the oracle's bytes and statuses, with no document on the general path (VERDICT r5
    item 5: non-ASCII string columns on the V2 kernels, split surrogates reported by the V1 / V2 diff kernels)."""
    from yjs_amd import pack_docs
    from yjs_amd.workloads import replicate
    arena, upd_off, doc_upd = load_ymb(f"c2u_v{fmt}")
    outs, status, _ = O.batch("merge", fmt, arena, upd_off, doc_upd, nthreads=8)
    assert not _compare(engine.run_host("merge", fmt, arena, upd_off, doc_upd), outs, status)
    assert engine.stats["docs_general"] == 0 and engine.stats["docs_large"] == 0, engine.stats
    assert (status == 0).all()
    # 5,000 merged documents (the V2 diff's lane kernel takes batches above 4,096)
    n = 5000
    merged = [outs[i % len(outs)] for i in range(n)]
    a2, o2, d2 = pack_docs([[m] for m in merged])
    souts, sst, _ = O.batch("sv", fmt, a2, o2, d2, nthreads=8)
    assert not _compare(engine.run_host("sv", fmt, a2, o2, d2), souts, sst)
    assert engine.stats["docs_general"] == 0, engine.stats
    svs = [random_state_vectors(souts[i], 1, seed=i)[0] for i in range(n)]
    sva, svo, _ = pack_docs([[s] for s in svs])
    douts, dst, _ = O.batch("diff", fmt, a2, o2, d2, sva, svo, nthreads=8)
    assert not _compare(engine.run_host("diff", fmt, a2, o2, d2, sva, svo), douts, dst)
    assert engine.stats["docs_general"] == 0, engine.stats
    assert (dst == 3).sum() > 0  # some cuts split an emoji: URIError, reported by the diff kernels themselves


def _text_update(client, s):
    """A V1 update inserting the raw bytes `s` as one ContentString (client, clock 0, no origin, parent ykey
    "t"); the string's UTF-16 length is not encoded in V1, so any bytes fit."""
    return _vu(1) + _vu(1) + _vu(client) + _vu(0) + bytes([0x04, 1, 1, ord("t")]) + _vu(len(s)) + s + _vu(0)


def _utf8_text(rng, nbytes):
    """Valid UTF-8 of about nbytes: ASCII, 2-byte (accents), 3-byte (CJK, Hangul near the surrogates) and
    4-byte (emoji, U+10FFFF) characters."""
    out = bytearray()
    pool = [0x61, 0xe9, 0x7ff, 0x800, 0x4e2d, 0xd7ff, 0xe000, 0xfffd, 0x1f600, 0x10000, 0x10ffff]
    while len(out) < nbytes:
        k = int(rng.integers(0, 4))
        cp = int(rng.choice(pool)) if rng.random() < 0.3 else [0x20 + int(rng.integers(0, 90)), 0xc0 + int(rng.integers(0, 0x700)),
                                                                  0x4e00 + int(rng.integers(0, 0x5000)), 0x1f300 + int(rng.integers(0, 0x300))][k]
        out += chr(cp).encode("utf-8")
    return bytes(out)


def test_long_non_ascii_strings_deferred_validation(engine):
    """ContentStrings of >= 32 non-ASCII bytes in the LDS merge kernel are counted by their lane and validated
    by the whole wave after the walk (ym_fast_common.h rstr_defer / deferred_ok: 4 bytes per lane, carries
    between lanes and 256-byte steps).  Valid texts of 30-700 bytes, and the same with each kind of invalid
    sequence (stray continuation, overlong C0 / E0 / F0, surrogate ED A0, above U+10FFFF, F5-FF, a sequence cut
    by the string's end) placed at random and at the 4-byte / 256-byte step boundaries, 1-20 long strings per
    document: merged bytes and statuses (yjs's URIError) equal the oracle's."""
    from yjs_amd import pack_docs
    rng = np.random.default_rng(2026)
    bad_seqs = [b"\x80", b"\xc0\x80", b"\xc1\xbf", b"\xe0\x80\x80", b"\xe0\x9f\xbf", b"\xed\xa0\x80", b"\xed\xbf\xbf",
                b"\xf0\x80\x80\x80", b"\xf0\x8f\xbf\xbf", b"\xf4\x90\x80\x80", b"\xf5\x80\x80\x80", b"\xff", b"\xe4\xb8",
                b"\xf0\x9f\x98"]
    docs = []
    for d in range(3000):
        nstr = 1 if d % 5 else int(rng.integers(2, 21))
        ups = []
        for u in range(nstr + 1):
            n = int(rng.choice([30, 31, 32, 33, 63, 64, 255, 256, 257, 300, 511, 512, 513, 700])) if u < nstr else 5
            s = _utf8_text(rng, n)
            kind = d % 4
            if u < nstr and kind == 1:  # an invalid sequence somewhere
                b = bad_seqs[int(rng.integers(0, len(bad_seqs)))]
                at = int(rng.choice([0, 3, 4, 5, 252, 253, 254, 255, 256, 257, len(s) // 2, len(s)]))
                at = min(at, len(s))
                s = s[:at] + b + s[at:]
            elif u < nstr and kind == 2:  # a cut multi-byte sequence at the end, or a step-boundary end
                s = s[:-1] if s[-1] >= 0x80 else s + b"\xe4"
            ups.append(_text_update(1000 + 7 * (nstr - u), s))
        docs.append(ups)
    a, o, dd = pack_docs(docs)
    outs, st, _ = O.batch("merge", 1, a, o, dd, nthreads=8)
    assert (st != 0).sum() > 100 and (st == 0).sum() > 1000
    assert not _compare(engine.run_host("merge", 1, a, o, dd), outs, st)
