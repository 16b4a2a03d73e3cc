"""ym_merge_async (include/ymerge.h): the LDS fast path enqueued without a host round trip.  Every document
it completes has ym_merge's bytes; a document it declines (larger than the fast path's LDS budget, rich
nested content) is left YM_PENDING and counted; a too-small output arena gives per-document
YM_ERR_CAPACITY; several calls queued back to back on one stream all complete."""
import numpy as np
import pytest

from yjs_amd.workloads import load_ymb

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from yjs_amd import Engine
    return Engine(0)


def _dev(torch, arena, upd_off, doc_upd, cap, off32):
    g = dict(arena=torch.from_numpy(np.array(arena, np.uint8)).cuda(),
             off=torch.from_numpy(upd_off.astype(np.uint32).view(np.int32) if off32 else upd_off.view(np.int64)).cuda(),
             doc=torch.from_numpy(doc_upd.view(np.int32)).cuda())
    nd = len(doc_upd) - 1
    g.update(out=torch.zeros(cap, dtype=torch.uint8, device="cuda"), oo=torch.zeros(nd, dtype=torch.int64, device="cuda"),
             ol=torch.zeros(nd, dtype=torch.int64, device="cuda"), st=torch.full((nd,), -1, dtype=torch.int32, device="cuda"))
    return g


def _outputs(g):
    a, oo, ol, st = g["out"].cpu().numpy(), g["oo"].cpu().numpy(), g["ol"].cpu().numpy(), g["st"].cpu().numpy()
    return [a[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() if st[i] == 0 else int(st[i]) for i in range(len(st))]


@pytest.mark.parametrize("name,off32", [("c2_v1", True), ("c2_v1", False), ("c4_v1", True), ("c2_v2", True), ("c4_v2", False)])
def test_async_equals_sync(engine, name, off32):
    import torch
    from yjs_amd.engine import _unpack
    fmt = 2 if name.endswith("v2") else 1
    arena, upd_off, doc_upd = load_ymb(name)
    n = min(len(doc_upd) - 1, 3000)
    doc_upd = doc_upd[:n + 1].copy()
    upd_off = upd_off[:int(doc_upd[-1]) + 1].copy()
    arena = arena[:int(upd_off[-1])].copy()
    want = _unpack(*engine.run_host("merge", fmt, arena, upd_off, doc_upd), False)
    cap = 2 * int(upd_off[-1]) + 64 * n + 64
    g = _dev(torch, arena, upd_off, doc_upd, cap, off32)
    pend = torch.zeros(1, dtype=torch.int32, device="cuda")
    call = engine.prepare_merge_async(fmt, g["arena"], g["off"], g["doc"], g["out"], g["oo"], g["ol"], g["st"], pending=pend,
                                      stream=torch.cuda.current_stream())
    for _ in range(4):  # queued back to back, one sync at the end
        assert call() == 0
    torch.cuda.synchronize()
    assert int(pend.item()) == 0
    got = _outputs(g)
    assert got == want


def test_async_declines_and_capacity(engine):
    import torch
    from yjs_amd import pack_docs
    from yjs_amd.engine import YM_PENDING, _unpack
    arena, upd_off, doc_upd = load_ymb("c2_v1")
    small = [[arena[int(upd_off[u]):int(upd_off[u + 1])].tobytes() for u in range(int(doc_upd[i]), int(doc_upd[i + 1]))]
             for i in range(6)]
    a5, o5, d5 = load_ymb("c5_v1")  # a C5 document: ~16 k updates, beyond the fast path
    big = [a5[int(o5[u]):int(o5[u + 1])].tobytes() for u in range(int(d5[0]), int(d5[1]))]
    docs = small[:3] + [big] + small[3:]
    a, o, d = pack_docs(docs)
    want = _unpack(*engine.run_host("merge", 1, a, o, d), False)
    cap = 2 * int(o[-1]) + 64 * len(docs) + 64
    g = _dev(torch, a, o, d, cap, True)
    pend = torch.zeros(1, dtype=torch.int32, device="cuda")
    call = engine.prepare_merge_async(1, g["arena"], g["off"], g["doc"], g["out"], g["oo"], g["ol"], g["st"], pending=pend)
    assert call() == 0
    torch.cuda.synchronize()
    got = _outputs(g)
    assert int(pend.item()) == 1 and got[3] == YM_PENDING
    assert [x for i, x in enumerate(got) if i != 3] == [x for i, x in enumerate(want) if i != 3]
    # an arena that ends inside the second document's slot: YM_ERR_CAPACITY from there on, the first intact
    ends = 2 * (o[d[1:]].astype(np.int64) - o[0]) + 64 * np.arange(1, len(docs) + 1)
    g2 = _dev(torch, a, o, d, int(ends[0]) + 8, True)
    call = engine.prepare_merge_async(1, g2["arena"], g2["off"], g2["doc"], g2["out"], g2["oo"], g2["ol"], g2["st"])
    assert call() == 0
    torch.cuda.synchronize()
    got = _outputs(g2)
    assert got[0] == want[0]
    assert all(x in (9, YM_PENDING) for x in got[1:]), got


def test_async_v2_off32_overlaps_host_merges(engine):
    """V2 + YM_OFF32 async calls widen their offsets into their own buffer, so synchronous host-batch
    merges issued while they run (on the library's stream, writing its staging offsets) cannot change what
    the async kernels read."""
    import torch
    from yjs_amd.engine import _unpack
    arena, upd_off, doc_upd = load_ymb("c2_v2")
    n = min(len(doc_upd) - 1, 2000)
    doc_upd = doc_upd[:n + 1].copy()
    upd_off = upd_off[:int(doc_upd[-1]) + 1].copy()
    arena = arena[:int(upd_off[-1])].copy()
    want = _unpack(*engine.run_host("merge", 2, arena, upd_off, doc_upd), False)
    a1, o1, d1 = load_ymb("c4_v2")  # the host batches: other documents, other offsets
    m = 500
    d1 = d1[:m + 1].copy()
    o1 = o1[:int(d1[-1]) + 1].copy()
    a1 = a1[:int(o1[-1])].copy()
    want1 = _unpack(*engine.run_host("merge", 2, a1, o1, d1), False)
    cap = 2 * int(upd_off[-1]) + 64 * n + 64
    g = _dev(torch, arena, upd_off, doc_upd, cap, True)
    s1 = torch.cuda.Stream()
    pend = torch.zeros(1, dtype=torch.int32, device="cuda")
    call = engine.prepare_merge_async(2, g["arena"], g["off"], g["doc"], g["out"], g["oo"], g["ol"], g["st"], pending=pend,
                                      stream=s1)
    for _ in range(3):
        for _ in range(4):
            assert call() == 0
        assert _unpack(*engine.run_host("merge", 2, a1, o1, d1), False) == want1
    torch.cuda.synchronize()
    assert int(pend.item()) == 0
    assert _outputs(g) == want
