"""ctypes binding of libymerge.so (include/ymerge.h) and the yjs-shaped API on top of it.

Function names, argument meaning and error behaviour mirror yjs 13.5.16's update API
(Y.mergeUpdates / Y.diffUpdate / Y.encodeStateVectorFromUpdate and their V2 forms, which sit beside
gaberogan/yjs@v0's public API in src/index.js:53-67): a malformed update raises the error class the
JS function throws (Error('Integer out of range!'), URIError, TypeError, RangeError, SyntaxError).
The *Batch variants take many documents at once -- the engine's reason to exist.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))


def lib_path():
    # YMERGE_LIB: another build of the library (diagnostics / A-B builds: libymerge_prof.so, ...)
    return os.environ.get("YMERGE_LIB") or os.path.join(_HERE, "libymerge.so")


class YjsError(Exception):
    """Error('...') thrown by lib0/yjs (e.g. 'Integer out of range!', 'Unexpected case')."""


class YjsURIError(YjsError):
    """URIError('URI malformed'): invalid UTF-8 or a split surrogate pair."""


class YjsTypeError(YjsError):
    """TypeError: unknown content ref / type ref / any tag."""


class YjsRangeError(YjsError):
    """RangeError: read past the end of the update."""


class YjsSyntaxError(YjsError):
    """SyntaxError: JSON.parse of a V1 JSON field."""


class UnsupportedInput(YjsError):
    """Valid input that needs a canonicalisation the engine does not implement."""


YM_DS_REF = 0x100  # ym_ds_merge: the reference's adjacency-only coalescing (include/ymerge.h)
YM_OFF32 = 0x200   # upd_off holds uint32_t offsets (include/ymerge.h)
YM_OUT_V1, YM_OUT_V2 = 0x1000, 0x2000  # ym_snapshot: output encoding
YM_NO_GC = 0x4000  # ym_compact: new Y.Doc({ gc: false })
YM_SV_FIRST = 0x10000  # ym_compact: the Doc's encodeStateVector, then the update


def _off_flag(upd_off):
    """YM_OFF32 for a 4-byte offsets tensor (int32 / uint32 view of u32 offsets), else 0."""
    return YM_OFF32 if upd_off.element_size() == 4 else 0

_STATUS_EXC = {
    1: YjsError, 2: YjsError, 3: YjsURIError, 4: YjsTypeError, 5: YjsRangeError, 6: YjsSyntaxError,
    7: UnsupportedInput, 8: YjsError, 9: YjsError,
}


def status_class(st):
    """The YM_* class of a status word (bits 0-7; include/ymerge.h YM_STATUS_CLASS)."""
    return int(st) & 0xff


def status_message(st):
    """The message yjs's exception carries for status word `st` (ym_strerror: V8 wording)."""
    return _load_lib().ym_strerror(int(st)).decode()


def raise_for_status(st):
    if st:
        raise _STATUS_EXC.get(status_class(st), YjsError)(status_message(st))


class _Batch(ctypes.Structure):
    _fields_ = [("arena", ctypes.c_void_p), ("upd_off", ctypes.c_void_p), ("doc_upd", ctypes.c_void_p),
                ("n_docs", ctypes.c_uint32), ("n_upd", ctypes.c_uint32), ("format", ctypes.c_int32),
                ("mem", ctypes.c_int32), ("sv_arena", ctypes.c_void_p), ("sv_off", ctypes.c_void_p)]


class _Out(ctypes.Structure):
    _fields_ = [("arena", ctypes.c_void_p), ("cap", ctypes.c_uint64), ("out_off", ctypes.c_void_p),
                ("out_len", ctypes.c_void_p), ("status", ctypes.c_void_p), ("used", ctypes.c_uint64)]


class _Stats(ctypes.Structure):
    _fields_ = [("docs", ctypes.c_uint64), ("docs_fast", ctypes.c_uint64), ("docs_general", ctypes.c_uint64),
                ("docs_error", ctypes.c_uint64), ("bytes_in", ctypes.c_uint64), ("bytes_out", ctypes.c_uint64),
                ("device_ms", ctypes.c_double), ("fast_ms", ctypes.c_double), ("general_ms", ctypes.c_double),
                ("docs_large", ctypes.c_uint64), ("large_ms", ctypes.c_double), ("docs_chunked", ctypes.c_uint64)]


EXPORTS = ("ym_init", "ym_shutdown", "ym_strerror", "ym_out_bound", "ym_merge", "ym_diff", "ym_sv", "ym_convert",
           "ym_meta", "ym_ds_merge", "ym_snapshot", "ym_compact", "ym_merge_async", "ym_diff_async", "ym_sv_async",
           "ym_host_alloc", "ym_host_free")
YM_PENDING = 101  # ym_*_async: declined by the async kernels (pass the document to ym_merge / ym_diff / ym_sv)


def load_library(path=None):
    path = path or lib_path()
    if not os.path.exists(path):
        raise RuntimeError(f"libymerge.so not built ({path}); run __graft_entry__.build()")
    L = ctypes.CDLL(path)
    L.ym_init.argtypes = [ctypes.c_int]
    L.ym_strerror.restype = ctypes.c_char_p
    L.ym_out_bound.restype = ctypes.c_uint64
    for fn in (L.ym_merge, L.ym_diff, L.ym_sv, L.ym_convert, L.ym_meta, L.ym_ds_merge, L.ym_snapshot, L.ym_compact):
        fn.argtypes = [ctypes.POINTER(_Batch), ctypes.POINTER(_Out), ctypes.c_void_p, ctypes.POINTER(_Stats)]
        fn.restype = ctypes.c_int
    L.ym_host_alloc.argtypes = [ctypes.c_size_t]
    L.ym_host_alloc.restype = ctypes.c_void_p
    L.ym_host_free.argtypes = [ctypes.c_void_p]
    L.ym_host_free.restype = None
    for fn in (L.ym_merge_async, L.ym_diff_async, L.ym_sv_async):
        fn.argtypes = [ctypes.POINTER(_Batch), ctypes.POINTER(_Out), ctypes.c_void_p, ctypes.c_void_p]
        fn.restype = ctypes.c_int
    return L


_LIB = None


def _load_lib():
    global _LIB
    if _LIB is None:
        _LIB = load_library()
    return _LIB


def pack_docs(docs):
    """[[bytes, ...], ...] -> (arena u8, upd_off u64, doc_upd u32)."""
    blobs = []
    doc_upd = [0]
    for d in docs:
        blobs.extend(d)
        doc_upd.append(doc_upd[-1] + len(d))
    lens = np.fromiter((len(b) for b in blobs), dtype=np.uint64, count=len(blobs))
    upd_off = np.zeros(len(blobs) + 1, np.uint64)
    np.cumsum(lens, out=upd_off[1:])
    arena = np.frombuffer(b"".join(blobs), np.uint8) if blobs else np.zeros(0, np.uint8)
    return arena, upd_off, np.array(doc_upd, np.uint32)


def _torch_first():
    """torch's wheel bundles its own HIP runtime.  When libymerge.so's runtime initialises the device first,
    torch's first CUDA call in the same process reports "No HIP GPUs are available"; in the other order both
    work.  So by default the engine lets torch initialise first when torch is importable (it is the plumbing
    for device tensors, the multi-GPU launcher and the benchmark).  A failure there is a warning, not an
    error: the library may still see the device (host batches need no torch)."""
    try:
        import torch
    except ImportError:
        return
    try:
        if torch.cuda.is_available():
            torch.cuda.init()
    except RuntimeError as e:  # torch cannot see a device the HIP runtime may still see: say which
        import warnings
        warnings.warn(f"torch could not initialise the GPU before libymerge.so ({e}); device tensors of this "
                      "process may not work", RuntimeWarning)


class HostOut:
    """Reusable page-locked output arrays for run_host (ym_host_alloc): the device-to-host copies land in them
    directly.  The arrays run_host returns with out=... are views into these buffers, valid until the next call
    that uses them; close() (or garbage collection) gives the memory back to the library's pool."""

    def __init__(self, engine, n_docs, cap):
        L = engine.lib
        self._lib = L
        n = max(int(n_docs), 1)
        self.cap = int(cap)
        self._ptrs = []

        def alloc(count, dtype):
            nbytes = max(count * np.dtype(dtype).itemsize, 1)
            p = L.ym_host_alloc(nbytes)
            if not p:
                raise MemoryError("ym_host_alloc failed")
            self._ptrs.append(p)
            buf = (ctypes.c_uint8 * nbytes).from_address(p)
            return np.frombuffer(buf, dtype=dtype, count=count)

        self.arena = alloc(max(self.cap, 1), np.uint8)
        self.out_off = alloc(n, np.uint64)
        self.out_len = alloc(n, np.uint64)
        self.status = alloc(n, np.int32)
        self.n_docs = n

    def close(self):
        for p in self._ptrs:
            self._lib.ym_host_free(p)
        self._ptrs = []

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass


class Engine:
    """One engine per process/GPU (the library keeps one HIP stream and workspace per thread).
    torch_first=False skips importing and initialising torch (host batches only: run_host and the batch
    functions; torch used later in the same process would then not see the GPU)."""

    def __init__(self, device=0, path=None, torch_first=True):
        if torch_first:
            _torch_first()
        self.lib = load_library(path)
        rc = self.lib.ym_init(device)
        if rc != 0:
            raise RuntimeError(f"ym_init({device}) failed: no usable MI355X/HIP device")
        self.device = device
        self.last_stats = _Stats()

    def _fn(self, op):
        L = self.lib
        return {"merge": L.ym_merge, "diff": L.ym_diff, "sv": L.ym_sv, "conv": L.ym_convert, "meta": L.ym_meta,
                "dsmerge": L.ym_ds_merge, "dsmerge_ref": L.ym_ds_merge,
                "snap_to_v1": L.ym_snapshot, "snap_to_v2": L.ym_snapshot, "compact": L.ym_compact,
                "compact_nogc": L.ym_compact, "compact_sv": L.ym_compact, "compact_nogc_sv": L.ym_compact}[op]

    @staticmethod
    def _format(op, fmt):
        extra = {"dsmerge_ref": YM_DS_REF, "snap_to_v1": YM_OUT_V1, "snap_to_v2": YM_OUT_V2, "compact_nogc": YM_NO_GC,
                 "compact_sv": YM_SV_FIRST, "compact_nogc_sv": YM_NO_GC | YM_SV_FIRST}
        return fmt | extra.get(op, 0)

    # ---- host-memory batches ------------------------------------------------------------------
    def host_array(self, count, dtype=np.uint8):
        """A numpy array in page-locked memory from the library's pool (ym_host_alloc): host batches packed
        into such arrays are copied in by the DMA engines directly (no per-call page pinning).  The memory goes
        back to the pool when the array (and every view of it) is garbage collected."""
        import weakref
        nbytes = max(int(count) * np.dtype(dtype).itemsize, 1)
        p = self.lib.ym_host_alloc(nbytes)
        if not p:
            raise MemoryError("ym_host_alloc failed")
        buf = (ctypes.c_uint8 * nbytes).from_address(p)
        weakref.finalize(buf, self.lib.ym_host_free, p)
        return np.frombuffer(buf, dtype=dtype, count=int(count))

    def host_out(self, n_docs, cap):
        """Page-locked output arrays for run_host(..., out=...) (see HostOut)."""
        return HostOut(self, n_docs, cap)

    def run_host(self, op, fmt, arena, upd_off, doc_upd, sv_arena=None, sv_off=None, out=None):
        """Runs op ('merge'|'diff'|'sv'|'conv'|'meta'|'dsmerge') over a packed host batch.
        upd_off: u64 offsets, or u32 (an arena below 4 GiB: passed as YM_OFF32, half the bytes to copy; host
        merges of >= 4,096 documents then run pipelined, include/ymerge.h).  out: a HostOut to write into
        (its arrays are returned, as views); by default fresh arrays.
        Returns (out_arena u8, out_off u64, out_len u64, status i32)."""
        arena = np.ascontiguousarray(arena, np.uint8)
        off32 = isinstance(upd_off, np.ndarray) and upd_off.dtype == np.uint32
        upd_off = np.ascontiguousarray(upd_off, np.uint32 if off32 else np.uint64)
        doc_upd = np.ascontiguousarray(doc_upd, np.uint32)
        n_docs = len(doc_upd) - 1
        n_upd = len(upd_off) - 1
        keep = [arena, upd_off, doc_upd]
        b = _Batch()
        b.arena = arena.ctypes.data if arena.size else None
        b.upd_off = upd_off.ctypes.data
        b.doc_upd = doc_upd.ctypes.data
        b.n_docs = n_docs
        b.n_upd = n_upd
        b.format = self._format(op, fmt) | (YM_OFF32 if off32 else 0)
        b.mem = 0
        if op == "diff" or sv_arena is not None:  # ym_diff's state vectors / ym_compact's target vectors
            # (a non-null arena even when every vector is empty: for ym_compact NULL means "no target")
            sv_arena = np.concatenate([np.ascontiguousarray(sv_arena, np.uint8), np.zeros(1, np.uint8)])
            sv_off = np.ascontiguousarray(sv_off, np.uint64)
            keep += [sv_arena, sv_off]
            b.sv_arena = sv_arena.ctypes.data
            b.sv_off = sv_off.ctypes.data
        cap = int(self.lib.ym_out_bound(ctypes.byref(b)))
        fn = self._fn(op)
        if out is not None and out.n_docs >= n_docs:
            o = _Out(out.arena.ctypes.data, out.cap, out.out_off.ctypes.data, out.out_len.ctypes.data,
                     out.status.ctypes.data, 0)
            rc = fn(ctypes.byref(b), ctypes.byref(o), None, ctypes.byref(self.last_stats))
            if rc == 0:
                del keep
                return out.arena[:int(o.used)], out.out_off[:n_docs], out.out_len[:n_docs], out.status[:n_docs]
            if rc != 9:
                raise RuntimeError(f"libymerge call failed: {rc} ({self.lib.ym_strerror(rc).decode()})")
            cap = int(o.used) + 4096  # too small: fresh arrays below
        for _ in range(4):
            out_arena = np.zeros(max(cap, 1), np.uint8)
            out_off = np.zeros(max(n_docs, 1), np.uint64)
            out_len = np.zeros(max(n_docs, 1), np.uint64)
            status = np.zeros(max(n_docs, 1), np.int32)
            o = _Out(out_arena.ctypes.data, cap, out_off.ctypes.data, out_len.ctypes.data, status.ctypes.data, 0)
            rc = fn(ctypes.byref(b), ctypes.byref(o), None, ctypes.byref(self.last_stats))
            if rc == 9:  # YM_ERR_CAPACITY
                cap = int(o.used) + 4096
                continue
            if rc != 0:
                raise RuntimeError(f"libymerge call failed: {rc} ({self.lib.ym_strerror(rc).decode()})")
            del keep
            return out_arena, out_off[:n_docs], out_len[:n_docs], status[:n_docs]
        raise RuntimeError("output capacity negotiation failed")

    # ---- device-resident batches (torch tensors on cuda) ---------------------------------------
    def run_device(self, op, fmt, arena, upd_off, doc_upd, out_arena, out_off, out_len, status,
                   sv_arena=None, sv_off=None, stream=None):
        """All arguments are torch CUDA tensors (uint8 / int64 / int32 views of the ABI arrays; upd_off
        may be a 4-byte tensor of u32 offsets: YM_OFF32).  Returns (rc, used_bytes).  stream: a
        torch.cuda.Stream or None (library stream)."""
        b = _Batch()
        b.arena = arena.data_ptr()
        b.upd_off = upd_off.data_ptr()
        b.doc_upd = doc_upd.data_ptr()
        b.n_docs = doc_upd.numel() - 1
        b.n_upd = upd_off.numel() - 1
        b.format = self._format(op, fmt) | _off_flag(upd_off)
        b.mem = 1
        if op == "diff" or sv_arena is not None:
            b.sv_arena = sv_arena.data_ptr()
            b.sv_off = sv_off.data_ptr()
        o = _Out(out_arena.data_ptr(), out_arena.numel(), out_off.data_ptr(), out_len.data_ptr(), status.data_ptr(), 0)
        fn = self._fn(op)
        s = ctypes.c_void_p(stream.cuda_stream) if stream is not None else None
        rc = fn(ctypes.byref(b), ctypes.byref(o), s, ctypes.byref(self.last_stats))
        return rc, int(o.used)

    def prepare_device(self, op, fmt, arena, upd_off, doc_upd, out_arena, out_off, out_len, status,
                       sv_arena=None, sv_off=None, stream=None):
        """run_device with the ABI structs built once: returns a zero-argument callable -> (rc, used)
        for repeated calls over the same (fixed) device buffers -- the serving / benchmark loop."""
        b = _Batch()
        b.arena = arena.data_ptr()
        b.upd_off = upd_off.data_ptr()
        b.doc_upd = doc_upd.data_ptr()
        b.n_docs = doc_upd.numel() - 1
        b.n_upd = upd_off.numel() - 1
        b.format = self._format(op, fmt) | _off_flag(upd_off)
        b.mem = 1
        if op == "diff" or sv_arena is not None:
            b.sv_arena = sv_arena.data_ptr()
            b.sv_off = sv_off.data_ptr()
        o = _Out(out_arena.data_ptr(), out_arena.numel(), out_off.data_ptr(), out_len.data_ptr(), status.data_ptr(), 0)
        fn = self._fn(op)
        s = ctypes.c_void_p(stream.cuda_stream) if stream is not None else None
        pb, po, ps = ctypes.byref(b), ctypes.byref(o), ctypes.byref(self.last_stats)
        keep = (b, o)

        def call():
            rc = fn(pb, po, s, ps)
            return rc, o.used
        call.keep = keep
        return call

    def prepare_merge_async(self, fmt, arena, upd_off, doc_upd, out_arena, out_off, out_len, status, pending=None,
                            stream=None):
        """ym_merge_async over fixed device buffers: a zero-argument callable that enqueues one merge of the
        batch on `stream` (the LDS fast path only) and returns its rc without waiting.  Declined documents
        get status YM_PENDING and are counted into `pending` (a 1-element int32 CUDA tensor, or None)."""
        return self.prepare_async("merge", fmt, arena, upd_off, doc_upd, out_arena, out_off, out_len, status,
                                  pending=pending, stream=stream)

    def prepare_async(self, op, fmt, arena, upd_off, doc_upd, out_arena, out_off, out_len, status, sv_arena=None,
                      sv_off=None, pending=None, stream=None):
        """ym_merge_async / ym_diff_async / ym_sv_async (op "merge" / "diff" / "sv") over fixed device buffers:
        a zero-argument callable that enqueues the call on `stream` and returns its rc without waiting.
        Declined documents get status YM_PENDING and are counted into `pending` (a 1-element int32 CUDA tensor,
        or None); diff takes each document's state vector from sv_arena / sv_off (int64 offsets)."""
        b = _Batch()
        b.arena = arena.data_ptr()
        b.upd_off = upd_off.data_ptr()
        b.doc_upd = doc_upd.data_ptr()
        b.n_docs = doc_upd.numel() - 1
        b.n_upd = upd_off.numel() - 1
        b.format = int(fmt) | _off_flag(upd_off)
        b.mem = 1
        o = _Out(out_arena.data_ptr(), out_arena.numel(), out_off.data_ptr(), out_len.data_ptr(), status.data_ptr(), 0)
        s = ctypes.c_void_p(stream.cuda_stream) if stream is not None else None
        if op == "diff":
            b.sv_arena = sv_arena.data_ptr()
            b.sv_off = sv_off.data_ptr()
        pend = ctypes.c_void_p(pending.data_ptr()) if pending is not None else None
        fn = {"merge": self.lib.ym_merge_async, "diff": self.lib.ym_diff_async, "sv": self.lib.ym_sv_async}[op]
        pb, po = ctypes.byref(b), ctypes.byref(o)

        def call():
            return fn(pb, po, s, pend)
        call.keep = (b, o)
        return call

    @property
    def stats(self):
        s = self.last_stats
        return {k: getattr(s, k) for k, _ in _Stats._fields_}


_ENGINE = None


def _engine():
    global _ENGINE
    if _ENGINE is None:
        _ENGINE = Engine(int(os.environ.get("YMERGE_DEVICE", "0")))
    return _ENGINE


def _unpack(out_arena, out_off, out_len, status, raise_errors):
    res = []
    for d in range(len(status)):
        if status[d]:
            if raise_errors:
                raise_for_status(status[d])
            res.append(int(status[d]))
        else:
            o = int(out_off[d])
            res.append(out_arena[o:o + int(out_len[d])].tobytes())
    return res


def mergeUpdatesBatch(docs, fmt=1, raise_errors=False):
    """docs: list of lists of update bytes. Returns one merged update per doc (or the status code)."""
    arena, upd_off, doc_upd = pack_docs(docs)
    return _unpack(*_engine().run_host("merge", fmt, arena, upd_off, doc_upd), raise_errors)


def diffUpdateBatch(updates, state_vectors, fmt=1, raise_errors=False):
    arena, upd_off, doc_upd = pack_docs([[u] for u in updates])
    sva, svo, _ = pack_docs([[s] for s in state_vectors])
    return _unpack(*_engine().run_host("diff", fmt, arena, upd_off, doc_upd, sva, svo), raise_errors)


def encodeStateVectorFromUpdateBatch(updates, fmt=1, raise_errors=False):
    arena, upd_off, doc_upd = pack_docs([[u] for u in updates])
    return _unpack(*_engine().run_host("sv", fmt, arena, upd_off, doc_upd), raise_errors)


def split_state_vector(buf):
    """(encoded state vector, rest) of a YM_SV_FIRST output: the vector is vu(n) then n varuint pairs."""
    pos = 0
    n, pos = _read_vu(buf, pos)
    for _ in range(2 * n):
        _, pos = _read_vu(buf, pos)
    return bytes(buf[:pos]), bytes(buf[pos:])


def compactUpdatesBatch(docs, fmt=1, raise_errors=False, gc=True, target_state_vectors=None, with_state_vector=False):
    """Doc round-trip compaction (ym_compact) over a batch: per document, encodeStateAsUpdate[V2] of a fresh
    Doc({ gc }) after applyUpdate[V2] of every update in order (the reference's own compaction:
    src/utils/encoding.js readUpdate / encodeStateAsUpdate, Transaction.js cleanupTransactions).
    target_state_vectors: one encoded state vector per document -- encodeStateAsUpdate[V2](doc, sv), only
    what the target is missing (encoding.js:94-116; the sync protocol's step-2 answer).
    with_state_vector: per document (encodeStateVector(doc), update) instead -- the Doc's own state vector,
    clients in StructStore insertion order (encoding.js:572-611, StructStore.js:49-56; YM_SV_FIRST)."""
    arena, upd_off, doc_upd = pack_docs(docs)
    sva = svo = None
    if target_state_vectors is not None:
        assert len(target_state_vectors) == len(docs)
        sva, svo, _ = pack_docs([[s] for s in target_state_vectors])
    op = ("compact" if gc else "compact_nogc") + ("_sv" if with_state_vector else "")
    res = _unpack(*_engine().run_host(op, fmt, arena, upd_off, doc_upd, sva, svo), raise_errors)
    return [split_state_vector(r) if with_state_vector and isinstance(r, bytes) else r for r in res]


def compactUpdates(updates, target_state_vector=None):
    t = None if target_state_vector is None else [target_state_vector]
    return compactUpdatesBatch([list(updates)], 1, True, target_state_vectors=t)[0]


def compactUpdatesV2(updates, target_state_vector=None):
    t = None if target_state_vector is None else [target_state_vector]
    return compactUpdatesBatch([list(updates)], 2, True, target_state_vectors=t)[0]


def mergeUpdates(updates):
    if len(updates) == 1:  # yjs returns the very same object
        return updates[0]
    return mergeUpdatesBatch([list(updates)], 1, True)[0]


def mergeUpdatesV2(updates):
    if len(updates) == 1:
        return updates[0]
    return mergeUpdatesBatch([list(updates)], 2, True)[0]


def diffUpdate(update, sv):
    return diffUpdateBatch([update], [sv], 1, True)[0]


def diffUpdateV2(update, sv):
    return diffUpdateBatch([update], [sv], 2, True)[0]


def encodeStateVectorFromUpdate(update):
    return encodeStateVectorFromUpdateBatch([update], 1, True)[0]


def encodeStateVectorFromUpdateV2(update):
    return encodeStateVectorFromUpdateBatch([update], 2, True)[0]


def convertUpdateFormatBatch(updates, fmt=1, raise_errors=False):
    """yjs 13.5.x convertUpdateFormat over a batch: fmt = the input format (1: V1 -> V2, 2: V2 -> V1)."""
    arena, upd_off, doc_upd = pack_docs([[u] for u in updates])
    return _unpack(*_engine().run_host("conv", fmt, arena, upd_off, doc_upd), raise_errors)


def convertUpdateFormatV1ToV2(update):
    return convertUpdateFormatBatch([update], 1, True)[0]


def convertUpdateFormatV2ToV1(update):
    return convertUpdateFormatBatch([update], 2, True)[0]


def _read_vu(b, pos):
    v, shift = 0, 0
    while True:
        x = b[pos]
        pos += 1
        v |= (x & 0x7F) << shift
        shift += 7
        if x < 0x80:
            return v, pos


def decode_meta(b):
    """The engine's parseUpdateMeta bytes -> {"from": {client: clock}, "to": {client: clock}} (dict order =
    the JS Map order)."""
    out, pos = {}, 0
    for key in ("from", "to"):
        n, pos = _read_vu(b, pos)
        m = {}
        for _ in range(n):
            client, pos = _read_vu(b, pos)
            clock, pos = _read_vu(b, pos)
            m[client] = clock
        out[key] = m
    return out


def parseUpdateMetaBatch(updates, fmt=1, raise_errors=False, decode=True):
    """yjs 13.5.16 parseUpdateMeta[V2] over a batch: per update {"from": {...}, "to": {...}} (or, with
    decode=False, the engine's encoding: two encoded state vectors back to back)."""
    arena, upd_off, doc_upd = pack_docs([[u] for u in updates])
    res = _unpack(*_engine().run_host("meta", fmt, arena, upd_off, doc_upd), raise_errors)
    return [decode_meta(r) if decode and isinstance(r, bytes) else r for r in res]


def parseUpdateMeta(update):
    return parseUpdateMetaBatch([update], 1, True)[0]


def parseUpdateMetaV2(update):
    return parseUpdateMetaBatch([update], 2, True)[0]


def mergeDeleteSetsBatch(docs, fmt=1, raise_errors=False, reference=False):
    """PermanentUserData's delete-set merge (reference src/utils/PermanentUserData.js:49-54) over a batch:
    docs is a list of lists of encoded delete sets (DSEncoderV1 bytes, or DSEncoderV2 with fmt=2); returns
    one encoded merged delete set per document.  reference=True: gaberogan/yjs@v0's own coalescing (only
    exactly adjacent ranges merge, DeleteSet.js:113-135); default: yjs 13.5.16's (overlaps merge too)."""
    arena, upd_off, doc_upd = pack_docs(docs)
    return _unpack(*_engine().run_host("dsmerge_ref" if reference else "dsmerge", fmt, arena, upd_off, doc_upd),
                   raise_errors)


def mergeEncodedDeleteSets(encoded_dss, fmt=1, reference=False):
    return mergeDeleteSetsBatch([list(encoded_dss)], fmt, True, reference)[0]


# ---- snapshots (reference src/utils/Snapshot.js:84-124) -----------------------------------------------
class Snapshot:
    """decodeSnapshot's result: ds = {client: [(clock, len), ...]} and sv = {client: clock}, dict order =
    the JS Map order (DeleteSet.clients / the state map)."""

    def __init__(self, ds, sv):
        self.ds = ds
        self.sv = sv

    def __eq__(self, other):  # equalSnapshots (Snapshot.js:48-78) on plain values
        return isinstance(other, Snapshot) and self.ds == other.ds and self.sv == other.sv

    def __repr__(self):
        return f"Snapshot(ds={self.ds!r}, sv={self.sv!r})"


def _vu(v):
    out = bytearray()
    while v > 127:
        out.append(0x80 | (v & 127))
        v >>= 7
    out.append(v)
    return bytes(out)


def _snapshot_v1_bytes(snap):
    """A Snapshot object as DSEncoderV1 bytes: the host side only lays the values out; the engine
    re-encodes them (and raises what encodeSnapshot[V2] raises)."""
    b = bytearray(_vu(len(snap.ds)))
    for client, items in snap.ds.items():
        b += _vu(client) + _vu(len(items))
        for clock, ln in items:
            b += _vu(clock) + _vu(ln)
    b += _vu(len(snap.sv))
    for client, clock in snap.sv.items():
        b += _vu(client) + _vu(clock)
    return bytes(b)


def _parse_snapshot_v1(b):
    pos = 0
    n, pos = _read_vu(b, pos)
    ds = {}
    for _ in range(n):
        client, pos = _read_vu(b, pos)
        m, pos = _read_vu(b, pos)
        items = ds.setdefault(client, [])
        for _ in range(m):
            clock, pos = _read_vu(b, pos)
            ln, pos = _read_vu(b, pos)
            items.append((clock, ln))
    n, pos = _read_vu(b, pos)
    sv = {}
    for _ in range(n):
        client, pos = _read_vu(b, pos)
        clock, pos = _read_vu(b, pos)
        sv[client] = clock
    return Snapshot(ds, sv)


def convertSnapshotBatch(bufs, from_fmt=1, to_fmt=1, raise_errors=False):
    """encodeSnapshot[V2](decodeSnapshot[V2](buf)) for every buf on the GPU (ym_snapshot): normalisation
    (repeated clients merged in Map order) and V1 <-> V2 conversion."""
    arena, upd_off, doc_upd = pack_docs([[b] for b in bufs])
    op = "snap_to_v2" if to_fmt == 2 else "snap_to_v1"
    return _unpack(*_engine().run_host(op, from_fmt, arena, upd_off, doc_upd), raise_errors)


def decodeSnapshotBatch(bufs, fmt=1, raise_errors=False):
    """decodeSnapshot[V2] over a batch: the engine validates and normalises (V1), the host reads the
    canonical bytes into Snapshot objects."""
    res = convertSnapshotBatch(bufs, fmt, 1, raise_errors)
    return [_parse_snapshot_v1(r) if isinstance(r, bytes) else r for r in res]


def encodeSnapshotBatch(snapshots, fmt=1, raise_errors=False):
    """encodeSnapshot / encodeSnapshotV2 (fmt=2) of Snapshot objects over a batch."""
    return convertSnapshotBatch([_snapshot_v1_bytes(s) for s in snapshots], 1, fmt, raise_errors)


def decodeSnapshot(buf):
    return decodeSnapshotBatch([buf], 1, True)[0]


def decodeSnapshotV2(buf):
    return decodeSnapshotBatch([buf], 2, True)[0]


def encodeSnapshot(snapshot):
    return encodeSnapshotBatch([snapshot], 1, True)[0]


def encodeSnapshotV2(snapshot):
    return encodeSnapshotBatch([snapshot], 2, True)[0]
