"""ym_diff_async / ym_sv_async (include/ymerge.h): the single-update walkers enqueued without a host round
trip.  Every document they complete has ym_diff's / ym_sv's bytes; a document they decline (several updates,
invalid input) is left YM_PENDING and counted; large single updates run on the one-wave walker; a too-small
output arena gives per-document YM_ERR_CAPACITY; calls queued back to back on two streams all complete."""
import numpy as np
import pytest

from yjs_amd.workloads import load_ymb, random_state_vectors

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from yjs_amd import Engine
    return Engine(0)


def _merged(engine, name, n):
    """The first n documents of a workload, merged (one update each)."""
    from yjs_amd.engine import _unpack
    fmt = 2 if name.endswith("v2") else 1
    arena, upd_off, doc_upd = load_ymb(name)
    doc_upd = doc_upd[:n + 1].copy()
    upd_off = upd_off[:int(doc_upd[-1]) + 1].copy()
    arena = arena[:int(upd_off[-1])].copy()
    return fmt, _unpack(*engine.run_host("merge", fmt, arena, upd_off, doc_upd), True)


def _dev(torch, a, o, d, sva, svo, cap, off32):
    g = dict(arena=torch.from_numpy(np.array(a, np.uint8)).cuda(),
             off=torch.from_numpy(o.astype(np.uint32).view(np.int32) if off32 else o.view(np.int64)).cuda(),
             doc=torch.from_numpy(d.view(np.int32)).cuda())
    if sva is not None:
        g.update(sva=torch.from_numpy(np.array(sva, np.uint8)).cuda(), svo=torch.from_numpy(svo.view(np.int64)).cuda())
    nd = len(d) - 1
    g.update(out=torch.zeros(cap, dtype=torch.uint8, device="cuda"), oo=torch.zeros(nd, dtype=torch.int64, device="cuda"),
             ol=torch.zeros(nd, dtype=torch.int64, device="cuda"), st=torch.full((nd,), -1, dtype=torch.int32, device="cuda"))
    return g


def _outputs(g):
    a, oo, ol, st = g["out"].cpu().numpy(), g["oo"].cpu().numpy(), g["ol"].cpu().numpy(), g["st"].cpu().numpy()
    return [a[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() if st[i] == 0 else int(st[i]) for i in range(len(st))]


def _call(engine, torch, op, fmt, g, pend=None, stream=None):
    return engine.prepare_async(op, fmt, g["arena"], g["off"], g["doc"], g["out"], g["oo"], g["ol"], g["st"],
                                sv_arena=g.get("sva"), sv_off=g.get("svo"), pending=pend, stream=stream)


def _cap(o, sva, nd, sections=64):
    """include/ymerge.h: 8 x the input bytes + 2 x the state vectors + 1 KB + 384 B per client section per
    document (a V2 diff's walker re-encodes the columns in scratch taken from the output arena)."""
    return 8 * int(o[-1]) + 2 * len(sva) + (1024 + 384 * sections) * nd + 8192


def _inputs(engine, docs, fmt, seed=0):
    """docs (lists of updates) packed, with one random state vector per document (of its first update)."""
    from yjs_amd import pack_docs
    from yjs_amd.engine import _unpack
    a, o, d = pack_docs(docs)
    a1, o1, d1 = pack_docs([[u[0]] for u in docs])
    fulls = _unpack(*engine.run_host("sv", fmt, a1, o1, d1), False)
    svs = [random_state_vectors(f if isinstance(f, bytes) else b"\x00", 1, seed=seed + i)[0] for i, f in enumerate(fulls)]
    sva, svo, _ = pack_docs([[s] for s in svs])
    return a, o, d, sva, svo


@pytest.mark.parametrize("op", ["diff", "sv"])
@pytest.mark.parametrize("name,off32", [("c2_v1", True), ("c2_v1", False), ("c4_v1", True), ("c2r_v1", False),
                                        ("c2_v2", True), ("c4_v2", False), ("c2r_v2", True)])
def test_async_equals_sync(engine, name, off32, op, monkeypatch):
    import torch
    from yjs_amd.engine import _unpack
    monkeypatch.setenv("YMERGE_DF2_MIN", "0")  # (V2 diffs through k_diff_small_v2 at this batch size too)
    fmt, merged = _merged(engine, name, 2000)
    a, o, d, sva, svo = _inputs(engine, [[m] for m in merged], fmt)
    want = _unpack(*engine.run_host(op, fmt, a, o, d, *((sva, svo) if op == "diff" else ())), False)
    cap = _cap(o, sva, len(merged))
    g = _dev(torch, a, o, d, sva if op == "diff" else None, svo, cap, off32)
    pend = torch.zeros(1, dtype=torch.int32, device="cuda")
    call = _call(engine, torch, op, fmt, g, pend, torch.cuda.current_stream())
    for _ in range(3):  # queued back to back, one sync at the end
        assert call() == 0
    torch.cuda.synchronize()
    assert int(pend.item()) == 0
    assert _outputs(g) == want


@pytest.mark.parametrize("fmt", [1, 2])
@pytest.mark.parametrize("op", ["diff", "sv"])
def test_async_declines_large_and_capacity(engine, fmt, op):
    import torch
    from yjs_amd import pack_docs
    from yjs_amd.engine import YM_PENDING, _unpack
    _, merged = _merged(engine, f"c2_v{fmt}", 6)
    a3, _, _ = load_ymb(f"c3_v{fmt}")  # one C3 update (~0.5-0.9 MB): the one-wave walker
    docs = [[m] for m in merged[:2]] + [[merged[2], merged[3]]] + [[a3.tobytes()]] + [[merged[4][:-3]]] + [[merged[5]]]
    a, o, d, sva, svo = _inputs(engine, docs, fmt, seed=7)
    extra = (sva, svo) if op == "diff" else ()
    want = _unpack(*engine.run_host(op, fmt, a, o, d, *extra), False)
    cap = _cap(o, sva, len(docs))
    g = _dev(torch, a, o, d, sva if op == "diff" else None, svo, cap, True)
    pend = torch.zeros(1, dtype=torch.int32, device="cuda")
    assert _call(engine, torch, op, fmt, g, pend)() == 0
    torch.cuda.synchronize()
    got = _outputs(g)
    # the two-update document is pending; the truncated one is pending or reports ym_diff's / ym_sv's error
    assert got[2] == YM_PENDING
    assert got[4] == YM_PENDING or got[4] == want[4]
    assert int(pend.item()) == sum(x == YM_PENDING for x in got)
    assert [x for i, x in enumerate(got) if i not in (2, 4)] == [x for i, x in enumerate(want) if i not in (2, 4)]
    # an arena far too small: every document is YM_ERR_CAPACITY or pending, none is corrupted
    g2 = _dev(torch, a, o, d, sva if op == "diff" else None, svo, 16, True)
    assert _call(engine, torch, op, fmt, g2)() == 0
    torch.cuda.synchronize()
    got2 = _outputs(g2)
    assert all(x in (9, YM_PENDING) or x == want[i] for i, x in enumerate(got2)), got2


def test_async_two_streams_share_scratch(engine):
    """Async calls on two streams: each waits for the previous one's scratch, so all results are exact."""
    import torch
    from yjs_amd.engine import _unpack
    fmt, merged = _merged(engine, "c4_v1", 1500)
    a, o, d, sva, svo = _inputs(engine, [[m] for m in merged], fmt, seed=11)
    wd = _unpack(*engine.run_host("diff", fmt, a, o, d, sva, svo), False)
    ws = _unpack(*engine.run_host("sv", fmt, a, o, d), False)
    cap = _cap(o, sva, len(merged))
    gd = _dev(torch, a, o, d, sva, svo, cap, True)
    gs = _dev(torch, a, o, d, None, svo, cap, False)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()  # (the inputs were copied on the current stream)
    cd = _call(engine, torch, "diff", fmt, gd, stream=s1)
    cs = _call(engine, torch, "sv", fmt, gs, stream=s2)
    for _ in range(4):
        assert cd() == 0 and cs() == 0
    torch.cuda.synchronize()
    assert _outputs(gd) == wd
    assert _outputs(gs) == ws
