"""ctypes binding of the CPU restatement (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY -- the oracle is the parity checker for the MI355X engine; product code never
imports this module (tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only).
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "build", "liboracle.so")

STATUS_NAMES = {
    0: "OK", 1: "Error:Integer out of range!", 2: "Error:Unexpected case", 3: "URIError",
    4: "TypeError", 5: "RangeError", 6: "SyntaxError", 7: "UNSUPPORTED", 8: "Error:Method unimplemented",
    9: "CAPACITY",
}

# JS error (constructor name, message) -> status code
def js_error_status(name, message):
    if name == "URIError":
        return 3
    if name == "TypeError":
        return 4
    if name == "RangeError":
        return 5
    if name == "SyntaxError":
        return 6
    if name == "Error":
        if message == "Integer out of range!":
            return 1
        if message == "Unexpected case":
            return 2
        if message == "Method unimplemented":
            return 8
    raise ValueError(f"unmapped JS error {name}: {message}")


# yjs 13.5.16's bundle is minified: its unknown-content-ref TypeError names the minified callee; the
# engine reports the reference's own source text (src/structs/Item.js readItemContent) instead
_MINIFIED = {"ai[(e & b.kr)] is not a function": "contentRefs[(info & binary.BITS5)] is not a function"}


def js_error_mismatch(status_word, name, message):
    """None if status word `status_word` is the exception (class and message) yjs threw, else a reason."""
    want = js_error_status(name, message)
    if int(status_word) & 0xff != want:
        return f"class {int(status_word) & 0xff} != {want}"
    from yjs_amd import status_message
    got = status_message(int(status_word))
    if got != _MINIFIED.get(message, message):
        return f"message {got!r} != {message!r}"
    return None


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.ymo_merge.argtypes = [ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t, ctypes.c_int,
                                ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t)]
        L.ymo_diff.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(u8p),
                               ctypes.POINTER(ctypes.c_size_t)]
        L.ymo_sv_from_update.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(u8p),
                                         ctypes.POINTER(ctypes.c_size_t)]
        L.ymo_convert.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t)]
        L.ymo_meta.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t)]
        L.ymo_ds_merge.argtypes = L.ymo_merge.argtypes
        L.ymo_compact.argtypes = L.ymo_merge.argtypes
        L.ymo_snapshot.argtypes = L.ymo_convert.argtypes
        L.ymo_free.argtypes = [ctypes.c_void_p]
        vp = ctypes.c_void_p
        L.ymo_batch.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, vp, ctypes.c_uint32, vp, vp, ctypes.c_int,
                                vp, vp, vp, vp]
        L.ymo_batch.restype = ctypes.c_int
        _lib = L
    return _lib


def _buf(b):
    b = bytes(b)
    arr = (ctypes.c_uint8 * max(1, len(b))).from_buffer_copy(b if b else b"\0")
    return arr, len(b)


def _take(out, n):
    data = ctypes.string_at(out, n.value) if n.value else b""
    lib().ymo_free(out)
    return data


def merge(updates, fmt=1):
    """mergeUpdates / mergeUpdatesV2 -> (status, bytes)."""
    L = lib()
    bufs = [_buf(u) for u in updates]
    n = len(bufs)
    ptrs = (ctypes.POINTER(ctypes.c_uint8) * max(1, n))(*[ctypes.cast(b[0], ctypes.POINTER(ctypes.c_uint8)) for b in bufs])
    lens = (ctypes.c_size_t * max(1, n))(*[b[1] for b in bufs])
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = L.ymo_merge(ptrs, lens, n, fmt, ctypes.byref(out), ctypes.byref(olen))
    return st, (_take(out, olen) if st == 0 else None)


def compact(updates, fmt=1):
    """Doc round trip (13.4.9, gc: true): applyUpdate[V2] of each update in order, encodeStateAsUpdate[V2]
    -> (status, bytes)."""
    L = lib()
    bufs = [_buf(u) for u in updates]
    n = len(bufs)
    ptrs = (ctypes.POINTER(ctypes.c_uint8) * max(1, n))(*[ctypes.cast(b[0], ctypes.POINTER(ctypes.c_uint8)) for b in bufs])
    lens = (ctypes.c_size_t * max(1, n))(*[b[1] for b in bufs])
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = L.ymo_compact(ptrs, lens, n, fmt, ctypes.byref(out), ctypes.byref(olen))
    return st, (_take(out, olen) if st == 0 else None)


def diff(update, sv, fmt=1):
    L = lib()
    u, ul = _buf(update)
    s, sl = _buf(sv)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = L.ymo_diff(ctypes.cast(u, ctypes.POINTER(ctypes.c_uint8)), ul, ctypes.cast(s, ctypes.POINTER(ctypes.c_uint8)),
                    sl, fmt, ctypes.byref(out), ctypes.byref(olen))
    return st, (_take(out, olen) if st == 0 else None)


def sv_from_update(update, fmt=1):
    L = lib()
    u, ul = _buf(update)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = L.ymo_sv_from_update(ctypes.cast(u, ctypes.POINTER(ctypes.c_uint8)), ul, fmt, ctypes.byref(out),
                              ctypes.byref(olen))
    return st, (_take(out, olen) if st == 0 else None)


def convert(update, fmt=1):
    """convertUpdateFormatV1ToV2 (fmt=1) / convertUpdateFormatV2ToV1 (fmt=2) -> (status, bytes)."""
    L = lib()
    u, ul = _buf(update)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = L.ymo_convert(ctypes.cast(u, ctypes.POINTER(ctypes.c_uint8)), ul, fmt, ctypes.byref(out), ctypes.byref(olen))
    return st, (_take(out, olen) if st == 0 else None)


def meta(update, fmt=1):
    """parseUpdateMeta / parseUpdateMetaV2 -> (status, bytes: from-map then to-map, each as an encoded
    state vector in Map order)."""
    L = lib()
    u, ul = _buf(update)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = L.ymo_meta(ctypes.cast(u, ctypes.POINTER(ctypes.c_uint8)), ul, fmt, ctypes.byref(out), ctypes.byref(olen))
    return st, (_take(out, olen) if st == 0 else None)


def snapshot(buf, fmt=1, to_fmt=1):
    """encodeSnapshot[V2](decodeSnapshot[V2](buf)) -> (status, bytes) (Snapshot.js:84-124)."""
    L = lib()
    p, n = _buf(buf)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = L.ymo_snapshot(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), n, fmt | (0x2000 if to_fmt == 2 else 0x1000), ctypes.byref(out), ctypes.byref(olen))
    return st, (_take(out, olen) if st == 0 else None)


def ds_merge(blobs, fmt=1):
    """PermanentUserData's mergeDeleteSets over encoded delete sets -> (status, encoded delete set)."""
    L = lib()
    bufs = [_buf(u) for u in blobs]
    n = len(bufs)
    ptrs = (ctypes.POINTER(ctypes.c_uint8) * max(1, n))(*[ctypes.cast(b[0], ctypes.POINTER(ctypes.c_uint8)) for b in bufs])
    lens = (ctypes.c_size_t * max(1, n))(*[b[1] for b in bufs])
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = L.ymo_ds_merge(ptrs, lens, n, fmt, ctypes.byref(out), ctypes.byref(olen))
    return st, (_take(out, olen) if st == 0 else None)


def batch(op, fmt, arena, upd_off, doc_upd, sv_arena=None, sv_off=None, nthreads=1, want_output=True):
    """Batched oracle over the engine's arena layout (numpy arrays). op: 'merge'|'diff'|'sv'|'conv'|'meta'|'dsmerge'.
    'compact': the Doc round trip (ymo_compact).  Returns (out_bytes_list_or_None, status ndarray, out_len ndarray)."""
    L = lib()
    if op == "dsmerge_ref":  # the reference's adjacency-only coalescing (DeleteSet.js:113-135)
        op, fmt = "dsmerge", fmt | 0x100
    if op in ("snap_to_v1", "snap_to_v2"):  # snapshot codec, output encoding YM_OUT_V1 / YM_OUT_V2
        op, fmt = "snap", fmt | (0x2000 if op == "snap_to_v2" else 0x1000)
    opc = {"merge": 0, "diff": 1, "sv": 2, "conv": 3, "meta": 4, "dsmerge": 5, "snap": 6, "compact": 7}[op]
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    upd_off = np.ascontiguousarray(upd_off, dtype=np.uint64)
    doc_upd = np.ascontiguousarray(doc_upd, dtype=np.uint32)
    n_docs = len(doc_upd) - 1
    if sv_arena is None:
        sv_arena = np.zeros(1, np.uint8)
        sv_off = np.zeros(n_docs + 1, np.uint64)
    sv_arena = np.ascontiguousarray(sv_arena, dtype=np.uint8)
    sv_off = np.ascontiguousarray(sv_off, dtype=np.uint64)
    in_len = np.array([upd_off[doc_upd[d + 1]] - upd_off[doc_upd[d]] for d in range(n_docs)], dtype=np.uint64) \
        if n_docs else np.zeros(0, np.uint64)
    cap = in_len * 2 + (sv_off[1:] - sv_off[:-1]) * 2 + 256
    cap_off = np.zeros(n_docs + 1, np.uint64)
    np.cumsum(cap, out=cap_off[1:])
    out_arena = np.zeros(int(cap_off[-1]) if want_output else 1, np.uint8)
    out_len = np.zeros(n_docs, np.uint64)
    status = np.zeros(n_docs, np.int32)
    L.ymo_batch(opc, fmt, arena.ctypes.data, upd_off.ctypes.data, doc_upd.ctypes.data, n_docs, sv_arena.ctypes.data,
                sv_off.ctypes.data, nthreads, out_arena.ctypes.data if want_output else None, cap_off.ctypes.data,
                out_len.ctypes.data, status.ctypes.data)
    outs = None
    if want_output:
        outs = [bytes(out_arena[int(cap_off[d]):int(cap_off[d]) + int(out_len[d])]) if status[d] == 0 else None
                for d in range(n_docs)]
    return outs, status, out_len
