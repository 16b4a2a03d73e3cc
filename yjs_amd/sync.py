"""y-protocols sync over stored updates, batched on the MI355X.

A sync server that keeps each document as one (merged) update answers the y-protocols sync messages
with the three batched update functions: SyncStep1 (the peer's state vector) -> SyncStep2 carrying
diffUpdate(stored, sv); SyncStep2 / Update (an update from the peer) -> stored := mergeUpdates([stored,
update]); the server's own SyncStep1 carries encodeStateVectorFromUpdate(stored).

The message framing is y-protocols 0.2.3 sync.js (an un-vendored dependency of gaberogan/yjs@v0:
package.json "y-protocols": "^0.2.3"; used by tests/testHelper.js:48-86,144-168):
    messageYjsSyncStep1 = 0 | messageYjsSyncStep2 = 1 | messageYjsUpdate = 2
    message = writeVarUint(type) + writeVarUint8Array(payload)
and readSyncMessage throws Error('Unknown message type') for any other type.  The Doc-based reference
functions (writeSyncStep1(encoder, doc), readSyncStep1(decoder, encoder, doc), ...) are restated over a
stored update instead of a Y.Doc; payload bytes are what the lazy 13.5.16 functions produce.
"""
from . import engine as E

messageYjsSyncStep1 = 0
messageYjsSyncStep2 = 1
messageYjsUpdate = 2


def _vu(v):
    out = bytearray()
    while v > 127:
        out.append(0x80 | (v & 127))
        v >>= 7
    out.append(v)
    return bytes(out)


def _read_vu(b, pos):
    """lib0 readVarUint: (value, new position); truncated input raises like lib0 (Integer out of range)."""
    num, mult = 0, 1
    while True:
        if pos >= len(b):
            raise E.YjsError("Integer out of range!")
        r = b[pos]
        pos += 1
        num += (r & 127) * mult
        mult *= 128
        if r < 128:
            return num, pos
        if num > 2 ** 53:
            raise E.YjsError("Integer out of range!")


def encode_message(msg_type, payload):
    """writeVarUint(type) + writeVarUint8Array(payload)."""
    return _vu(msg_type) + _vu(len(payload)) + bytes(payload)


def decode_message(msg):
    """(type, payload, bytes consumed) of one sync message."""
    t, pos = _read_vu(msg, 0)
    n, pos = _read_vu(msg, pos)
    if pos + n > len(msg):
        raise E.YjsRangeError("Unexpected end of array")
    return t, bytes(msg[pos:pos + n]), pos + n


def writeSyncStep1(stored, fmt=1):
    """SyncStep1 of the server: the state vector of its stored update."""
    sv = (E.encodeStateVectorFromUpdateV2 if fmt == 2 else E.encodeStateVectorFromUpdate)(stored)
    return encode_message(messageYjsSyncStep1, sv)


def writeSyncStep2(stored, encoded_state_vector, fmt=1):
    return encode_message(messageYjsSyncStep2, (E.diffUpdateV2 if fmt == 2 else E.diffUpdate)(stored, encoded_state_vector))


def writeUpdate(update):
    return encode_message(messageYjsUpdate, update)


def readSyncMessage(msg, stored, fmt=1):
    """One message against one stored document: returns (message type, reply message or None, new stored)."""
    t, payload, _ = decode_message(msg)
    if t == messageYjsSyncStep1:
        return t, writeSyncStep2(stored, payload, fmt), stored
    if t in (messageYjsSyncStep2, messageYjsUpdate):
        merge = E.mergeUpdatesV2 if fmt == 2 else E.mergeUpdates
        return t, None, merge([stored, payload])
    raise E.YjsError("Unknown message type")


def readSyncMessagesBatch(messages, stored, fmt=1):
    """Batched readSyncMessage: message i is applied to stored document i.  All SyncStep1 messages are
    answered by one batched diffUpdate, all SyncStep2 / Update messages merged by one batched
    mergeUpdates call.  Returns (types, replies (bytes or None), new stored list); a malformed message
    or document yields the matching exception object in its slot."""
    n = len(messages)
    types, replies, new_stored = [None] * n, [None] * n, list(stored)
    step1, apply_ = [], []
    for i, m in enumerate(messages):
        try:
            t, payload, _ = decode_message(m)
        except E.YjsError as e:
            types[i] = e
            continue
        types[i] = t
        if t == messageYjsSyncStep1:
            step1.append((i, payload))
        elif t in (messageYjsSyncStep2, messageYjsUpdate):
            apply_.append((i, payload))
        else:
            types[i] = E.YjsError("Unknown message type")
    if step1:
        diffs = E.diffUpdateBatch([stored[i] for i, _ in step1], [sv for _, sv in step1], fmt)
        for (i, _), d in zip(step1, diffs):
            replies[i] = encode_message(messageYjsSyncStep2, d) if isinstance(d, bytes) else _exc(d)
    if apply_:
        merged = E.mergeUpdatesBatch([[stored[i], u] for i, u in apply_], fmt)
        for (i, _), m in zip(apply_, merged):
            if isinstance(m, bytes):
                new_stored[i] = m
            else:
                replies[i] = _exc(m)
    return types, replies, new_stored


def _exc(status):
    try:
        E.raise_for_status(status)
    except E.YjsError as e:
        return e
    return E.YjsError(f"status {status}")
