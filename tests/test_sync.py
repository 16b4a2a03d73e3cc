"""y-protocols sync framing over stored updates (yjs_amd/sync.py).  CPU tests pin
the framing (y-protocols 0.2.3 sync.js: varUint type + varUint8Array payload); the GPU test runs a
batched sync round (SyncStep1 -> SyncStep2 from diffUpdate, SyncStep2 -> mergeUpdates) and checks it
against the oracle and for convergence of the peers' state vectors."""
import pytest

from yjs_amd import sync as S


def test_framing_bytes():
    assert S.encode_message(S.messageYjsSyncStep1, b"\x01\x02") == b"\x00\x02\x01\x02"
    assert S.encode_message(S.messageYjsUpdate, b"") == b"\x02\x00"
    big = bytes(300)
    m = S.encode_message(S.messageYjsSyncStep2, big)
    assert m[:3] == b"\x01\xac\x02" and len(m) == 303
    assert S.decode_message(m) == (1, big, 303)


def test_framing_errors():
    from yjs_amd.engine import YjsError, YjsRangeError
    with pytest.raises(YjsError, match="Integer out of range"):
        S.decode_message(b"\x80")
    with pytest.raises(YjsRangeError):
        S.decode_message(b"\x01\x05ab")


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [1, 2])
def test_sync_round_batched(fmt):
    import oracle_ref as O
    from yjs_amd import pack_docs
    from yjs_amd.workloads import load_ymb
    a, o, d = load_ymb(f"c2_v{fmt}")
    upd = lambda u: a[int(o[u]):int(o[u + 1])].tobytes()
    full_docs = [[upd(u) for u in range(int(d[i]), int(d[i + 1]))] for i in range(48)]
    half_docs = [x[: len(x) // 2] for x in full_docs]
    fa, fo, fd = pack_docs(full_docs)
    ha, ho, hd = pack_docs(half_docs)
    server, st1, _ = O.batch("merge", fmt, fa, fo, fd, nthreads=8)
    client, st2, _ = O.batch("merge", fmt, ha, ho, hd, nthreads=8)
    assert (st1 == 0).all() and (st2 == 0).all()
    # the client's SyncStep1 carries its state vector; the server answers with SyncStep2
    sv = lambda u: O.sv_from_update(u, fmt)[1]
    msgs = [S.encode_message(S.messageYjsSyncStep1, sv(c)) for c in client]
    types, replies, stored = S.readSyncMessagesBatch(msgs, server, fmt)
    assert types == [S.messageYjsSyncStep1] * len(msgs) and stored == server
    for c, r, s in zip(client, replies, server):
        t, payload, _ = S.decode_message(r)
        assert t == S.messageYjsSyncStep2
        assert payload == O.diff(s, sv(c), fmt)[1]
    # the client applies the SyncStep2 (server side of the same code path: readSyncMessage on the client)
    types2, replies2, client2 = S.readSyncMessagesBatch(replies, client, fmt)
    assert types2 == [S.messageYjsSyncStep2] * len(msgs) and replies2 == [None] * len(msgs)
    for c2, s in zip(client2, server):
        assert sv(c2) == sv(s)  # converged
    bad = S.readSyncMessagesBatch([b"\x07\x00"], server[:1], fmt)[0][0]
    assert str(bad) == "Unknown message type"
