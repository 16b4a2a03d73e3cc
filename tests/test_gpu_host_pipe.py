"""GPU parity of the pipelined host merge path (ym_api.hip run_host_pipe: host batches of >= 4,096 documents
with u32 offsets are cut into ~3 MiB chunks, copied in, merged and copied out chunk by chunk).  It must give
the unpipelined path's bytes, lengths and statuses for every document -- also when some documents are
declined by the fast kernels, where the call falls back to the exact flow -- and the oracle's bytes."""
import numpy as np
import pytest

import oracle_ref as O
from yjs_amd.workloads import load_ymb, replicate

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from yjs_amd import Engine
    return Engine(0)


def _same(a, b):
    (aa, ao, al, ast), (ba, bo, bl, bst) = a, b
    assert np.array_equal(ast, bst)
    assert np.array_equal(al, bl)
    bad = [d for d in range(len(ast)) if aa[int(ao[d]):int(ao[d]) + int(al[d])].tobytes() !=
           ba[int(bo[d]):int(bo[d]) + int(bl[d])].tobytes()]
    assert not bad, bad[:10]


@pytest.mark.parametrize("name", ["c2_v1", "c4_v1", "c2_v2"])
def test_pipelined_host_merge_matches_unpipelined(engine, name):
    arena, upd_off, doc_upd = replicate(*load_ymb(name), 10000)
    fmt = 2 if name.endswith("v2") else 1
    ref = engine.run_host("merge", fmt, arena, upd_off, doc_upd)  # u64 offsets: unpipelined
    got = engine.run_host("merge", fmt, arena, upd_off.astype(np.uint32), doc_upd)
    _same(ref, got)
    # packed back to back in document order, as the unpipelined path packs them
    assert np.array_equal(got[1][1:], (got[1] + got[2])[:-1])
    hout = engine.host_out(len(doc_upd) - 1, 2 * int(upd_off[-1]) + 64 * (len(doc_upd) - 1) + 8192)
    for _ in range(2):  # reused page-locked outputs
        _same(ref, engine.run_host("merge", fmt, arena, upd_off.astype(np.uint32), doc_upd, out=hout))
    # the batch itself in page-locked pool memory (as the Node addon packs it): the merge kernels read it in
    # place (zero-copy) and the packing kernels write the outputs straight into the page-locked outputs
    pa = engine.host_array(len(arena))
    pa[:] = arena
    po = engine.host_array(len(upd_off), np.uint32)
    po[:] = upd_off
    pd = engine.host_array(len(doc_upd), np.uint32)
    pd[:] = doc_upd
    for _ in range(2):
        _same(ref, engine.run_host("merge", fmt, pa, po, pd, out=hout))
    _same(ref, engine.run_host("merge", fmt, pa, po, pd))  # pool inputs, pageable outputs (copies out)
    hout.close()
    # a sample against the oracle
    idx = list(range(0, len(doc_upd) - 1, 97))
    docs = [[arena[int(upd_off[u]):int(upd_off[u + 1])].tobytes() for u in range(int(doc_upd[d]), int(doc_upd[d + 1]))]
            for d in idx]
    from yjs_amd import pack_docs
    a2, o2, d2 = pack_docs(docs)
    outs, status, _ = O.batch("merge", fmt, a2, o2, d2, nthreads=8)
    for i, d in enumerate(idx):
        assert int(got[3][d]) == int(status[i])
        assert got[0][int(got[1][d]):int(got[1][d]) + int(got[2][d])].tobytes() == outs[i]


def test_pipelined_host_merge_falls_back_on_declines(engine):
    """Rich documents (nested payloads: the hot kernel declines them) spread through a C2 batch: the pipelined
    call must notice and give the exact flow's results."""
    a, o, d = replicate(*load_ymb("c2_v1"), 6000)
    ra, ro, rd = replicate(*load_ymb("c2r_v1"), 200)
    from yjs_amd import pack_docs
    docs = []
    for k in range(6000):
        docs.append([a[int(o[u]):int(o[u + 1])].tobytes() for u in range(int(d[k]), int(d[k + 1]))])
        if k % 30 == 0:
            r = (k // 30) % 200
            docs.append([ra[int(ro[u]):int(ro[u + 1])].tobytes() for u in range(int(rd[r]), int(rd[r + 1]))])
    docs.append([b"\x01\x01", b"\x00\x00"])  # a truncated update: an exception in the batch
    arena, upd_off, doc_upd = pack_docs(docs)
    ref = engine.run_host("merge", 1, arena, upd_off, doc_upd)
    got = engine.run_host("merge", 1, arena, upd_off.astype(np.uint32), doc_upd)
    _same(ref, got)
    assert int(got[3][-1]) != 0
