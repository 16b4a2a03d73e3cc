"""Multi-GPU plumbing: documents are independent, so ranks take disjoint shards and never exchange
document data.  The only collectives are the max of the timed region and the sum of counters
(torch.distributed: RCCL on GPUs, gloo in the CPU tests)."""
import numpy as np


def shard_ranges(n_docs_total, world):
    """Contiguous, balanced doc ranges [start, end) per rank (weak-scaling benches use a fixed per-rank
    count instead: global docs rank*D .. (rank+1)*D)."""
    base, extra = divmod(n_docs_total, world)
    out, s = [], 0
    for r in range(world):
        e = s + base + (1 if r < extra else 0)
        out.append((s, e))
        s = e
    return out


def shard_batch(arena, upd_off, doc_upd, start, end):
    """Sub-batch of documents [start, end) of a packed batch, re-based to its own arena."""
    u0, u1 = int(doc_upd[start]), int(doc_upd[end])
    b0, b1 = int(upd_off[u0]), int(upd_off[u1])
    return (np.ascontiguousarray(arena[b0:b1]), (upd_off[u0:u1 + 1] - b0).astype(np.uint64),
            (doc_upd[start:end + 1] - u0).astype(np.uint32))


def template_shard(n_templates, rank, docs_per_rank):
    """Template ids for rank's documents in a weak-scaling run: global doc g = rank*D + i uses
    template g % T, so ranks process distinct document streams."""
    g0 = rank * docs_per_rank
    return [(g0 + i) % n_templates for i in range(docs_per_rank)]


def reduce_run(dist, elapsed, counters, device=None):
    """(max elapsed over ranks, elementwise sum of counters) -- the benchmark's only collectives."""
    import torch
    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    c = torch.tensor([float(x) for x in counters], dtype=torch.float64, device=device)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), [float(x) for x in c.tolist()]
