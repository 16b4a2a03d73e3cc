"""Multi-GPU plumbing: documents are independent, so each GPU takes a disjoint shard
and never exchanges document data.  Partition:

* ``hash``  -- ``gpu = hash32(docIndex) % G`` (C1/C2/C4: many small documents of similar size);
* ``bytes`` -- greedy byte-balanced (longest-processing-time first: each document, largest first, goes
  to the currently lightest shard; C3/C5: few large documents of skewed sizes).

The only collectives are the max of the timed region and the sum of per-rank counters
(torch.distributed: RCCL over xGMI on GPUs, gloo in the CPU tests).  Outputs return to host-side
order by docIndex (``MultiDeviceEngine``, ``scatter_results``)."""
import numpy as np


def hash32(x):
    """32-bit integer mix (murmur3 fmix32) of docIndex, vectorised; the shard of doc i is hash32(i) % G."""
    h = np.asarray(x, dtype=np.uint64) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    return h.astype(np.uint32)


def hash_partition(doc_ids, world):
    """[doc ids of shard r for r in range(world)]: doc i goes to shard hash32(i) % world (ids ascending)."""
    doc_ids = np.asarray(doc_ids, dtype=np.int64)
    r = hash32(doc_ids) % np.uint32(world)
    return [doc_ids[r == k] for k in range(world)]


def byte_partition(doc_bytes, world):
    """Greedy byte-balanced partition of docs 0..n-1 with sizes doc_bytes: largest first, each to the
    lightest shard so far (ties: lowest shard).  Returns [doc ids of shard r] (ids ascending)."""
    doc_bytes = np.asarray(doc_bytes, dtype=np.int64)
    order = np.argsort(-doc_bytes, kind="stable")
    load = np.zeros(world, np.int64)
    owner = np.empty(len(doc_bytes), np.int64)
    if world == 1:
        owner[:] = 0
    else:
        import heapq
        heap = [(0, r) for r in range(world)]
        for i in order:
            ld, r = heapq.heappop(heap)
            owner[i] = r
            heapq.heappush(heap, (ld + int(doc_bytes[i]), r))
    ids = np.arange(len(doc_bytes), dtype=np.int64)
    return [ids[owner == k] for k in range(world)]


def partition(doc_bytes, world, how="hash"):
    if how == "hash":
        return hash_partition(np.arange(len(doc_bytes)), world)
    if how == "bytes":
        return byte_partition(doc_bytes, world)
    raise ValueError(f"unknown partition {how!r}")


def gather_docs(arena, upd_off, doc_upd, doc_ids):
    """Packed sub-batch (arena, upd_off u64, doc_upd u32) of the given documents of a packed batch, in
    the given order (an id may repeat: replicated templates are distinct copies in the new arena)."""
    doc_ids = np.asarray(doc_ids, dtype=np.int64)
    u0 = doc_upd[doc_ids].astype(np.int64)
    u1 = doc_upd[doc_ids + 1].astype(np.int64)
    k = u1 - u0
    new_doc = np.zeros(len(doc_ids) + 1, np.uint32)
    np.cumsum(k, out=new_doc[1:])
    n_upd = int(new_doc[-1])
    # update indices of the new batch, in order
    upd_idx = np.repeat(u0 - new_doc[:-1].astype(np.int64), k) + np.arange(n_upd, dtype=np.int64)
    lens = (upd_off[upd_idx + 1] - upd_off[upd_idx]).astype(np.int64)
    new_off = np.zeros(n_upd + 1, np.uint64)
    np.cumsum(lens, out=new_off[1:])
    # byte gather: one contiguous span per document
    b0 = upd_off[u0].astype(np.int64)
    b1 = upd_off[u1].astype(np.int64)
    blen = b1 - b0
    total = int(blen.sum())
    starts = np.zeros(len(doc_ids), np.int64)
    if len(doc_ids) > 1:
        np.cumsum(blen[:-1], out=starts[1:])
    src = np.repeat(b0 - starts, blen) + np.arange(total, dtype=np.int64)
    new_arena = arena[src] if total else np.zeros(0, np.uint8)
    return np.ascontiguousarray(new_arena, np.uint8), new_off, new_doc


def shard_batch(arena, upd_off, doc_upd, start, end):
    """Sub-batch of documents [start, end) of a packed batch, re-based to its own arena."""
    return gather_docs(arena, upd_off, doc_upd, np.arange(start, end))


def doc_sizes(upd_off, doc_upd):
    return (upd_off[doc_upd[1:]].astype(np.int64) - upd_off[doc_upd[:-1]].astype(np.int64))


def weak_scaling_shard(t_arena, t_off, t_doc, docs_per_gpu, world, rank, how="hash"):
    """The rank's shard of a weak-scaling job: the job has world * docs_per_gpu documents, global doc g is
    a distinct copy of template g % T, and documents are partitioned by ``how``.  Returns
    (arena, upd_off, doc_upd, global doc ids of the shard)."""
    T = len(t_doc) - 1
    n = docs_per_gpu * world
    tsz = doc_sizes(t_off, t_doc)
    sizes = tsz[np.arange(n) % T]
    ids = partition(sizes, world, how)[rank]
    a, o, d = gather_docs(t_arena, t_off, t_doc, ids % T)
    return a, o, d, ids


def reduce_run(dist, elapsed, counters, device=None):
    """(max elapsed over ranks, elementwise sum of counters) -- the benchmark's only collectives."""
    import torch
    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    c = torch.tensor([float(x) for x in counters], dtype=torch.float64, device=device)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), [float(x) for x in c.tolist()]


def scatter_results(n_docs, shards, shard_results):
    """Reassembles per-shard result lists into docIndex order."""
    out = [None] * n_docs
    for ids, res in zip(shards, shard_results):
        for i, r in zip(ids, res):
            out[int(i)] = r
    return out


class MultiDeviceEngine:
    """One host process driving several GPUs of a node (the library keeps one stream and workspace per
    (thread, device)): a batch is partitioned over the devices, each shard runs on its device's own
    long-lived worker thread, and the outputs come back in docIndex order.  The worker threads live as
    long as the engine, so the library state they create (stream, events, pinned staging, device
    scratch) is made once and reused by every call; ``close()`` releases it on the threads that own it
    (``ym_shutdown``).  ``runner(device)`` returns an object with ``run_host`` (default:
    ``yjs_amd.Engine``, created on the worker thread); tests pass a stub."""

    def __init__(self, devices, partition_by="hash", runner=None):
        from concurrent.futures import ThreadPoolExecutor
        self.devices = list(devices)
        self.partition_by = partition_by
        if runner is None:
            from .engine import Engine
            runner = Engine
        self._runner = runner
        self._engines = [None] * len(self.devices)
        self._pools = [ThreadPoolExecutor(max_workers=1, thread_name_prefix=f"ym-dev{d}") for d in self.devices]

    def _engine(self, i):
        # always called on worker thread i: the engine's ym_init binds that thread to device i
        if self._engines[i] is None:
            self._engines[i] = self._runner(self.devices[i])
        return self._engines[i]

    def run_host(self, op, fmt, arena, upd_off, doc_upd, sv_arena=None, sv_off=None):
        """Like Engine.run_host, but returns per-document results in docIndex order: a list of bytes
        (status 0) or int status codes."""
        if self._pools is None:
            raise RuntimeError("MultiDeviceEngine is closed")
        n = len(doc_upd) - 1
        G = len(self.devices)
        shards = partition(doc_sizes(upd_off, doc_upd), G, self.partition_by)

        def work(i):
            ids = shards[i]
            a, o, d = gather_docs(arena, upd_off, doc_upd, ids)
            extra = ()
            if op == "diff":
                sa, so, _ = gather_docs(sv_arena, sv_off, np.arange(n + 1, dtype=np.uint32), ids)
                extra = (sa, so)
            eng = self._engine(i)
            oa, oo, ol, st = eng.run_host(op, fmt, a, o, d, *extra)
            return [int(st[j]) if st[j] else oa[int(oo[j]):int(oo[j]) + int(ol[j])].tobytes()
                    for j in range(len(ids))]

        futs = {i: self._pools[i].submit(work, i) for i in range(G) if len(shards[i])}
        results = [[] for _ in range(G)]
        err = None
        for i, f in futs.items():  # wait for every shard before raising (re-raised on the caller's thread)
            try:
                results[i] = f.result()
            except Exception as e:
                err = err or e
        if err is not None:
            raise err
        return scatter_results(n, shards, results)

    def close(self):
        """Releases each device's library state on the worker thread that created it, then the threads."""
        if self._pools is None:
            return

        def release(i):
            eng = self._engines[i]
            if eng is not None and hasattr(eng, "lib"):
                eng.lib.ym_shutdown()
            self._engines[i] = None

        for i, p in enumerate(self._pools):
            p.submit(release, i).result()
            p.shutdown(wait=True)
        self._pools = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
