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
        if int(st[d]) != int(status[d]):
            bad.append((d, "status", int(st[d]), int(status[d])))
            continue
        if st[d] == 0:
            got = out_arena[int(out_off[d]):int(out_off[d]) + int(out_len[d])].tobytes()
            if got != outs[d]:
                bad.append((d, "bytes", len(got), len(outs[d])))
    return bad


@pytest.mark.parametrize("name", ["c2_v1", "c2_v2", "c4_v1", "c4_v2", "c1_v1", "c1_v2"])
def test_merge_workload_matches_oracle(engine, name):
    arena, upd_off, doc_upd = load_ymb(name)
    fmt = 2 if name.endswith("v2") else 1
    outs, status, _ = O.batch("merge", fmt, arena, upd_off, doc_upd, nthreads=8)
    res = engine.run_host("merge", fmt, arena, upd_off, doc_upd)
    bad = _compare(res, outs, status)
    assert not bad, bad[:10]
    st = engine.stats
    if name in ("c2_v1", "c4_v1", "c2_v2", "c4_v2"):
        assert st["docs_fast"] == st["docs"], st  # every C2/C4 doc takes the LDS fast path (V1 and V2)


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


@pytest.mark.parametrize("fmt", [1, 2])
def test_c3_sv_matches_oracle(engine, fmt):
    arena, upd_off, doc_upd = load_ymb(f"c3_v{fmt}")
    from yjs_amd import pack_docs
    upd = arena.tobytes()
    a2, o2, d2 = pack_docs([[upd] for _ in range(4)])
    outs, st, _ = O.batch("sv", fmt, a2, o2, d2)
    bad = _compare(engine.run_host("sv", fmt, a2, o2, d2), outs, st)
    assert not bad, bad[:10]
    assert engine.stats["docs_fast"] == engine.stats["docs"], engine.stats


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
