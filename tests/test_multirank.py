"""World-size-2 rehearsal of the multi-GPU path on CPU (gloo): ranks take disjoint document shards,
process them independently (here with the CPU oracle standing in for the device), and the only
collectives are the max-time / sum-of-counters reductions.  The union of the shards' outputs must equal
a single-process run."""
import os
import threading
import socket

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    import oracle_ref
    from yjs_amd.distributed import gather_docs, hash_partition, reduce_run
    from yjs_amd.workloads import load_ymb
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, o, d = load_ymb("c2_v1")
    n = 96
    ids = hash_partition(np.arange(n), world)[rank]
    sa, so, sd = gather_docs(a, o, d, ids)
    outs, st, ol = oracle_ref.batch("merge", 1, sa, so, sd)
    tmax, (docs, bytes_out, errs) = reduce_run(dist, 0.5 + rank, [len(ids), float(np.sum(ol)), float((st != 0).sum())])
    q.put((rank, [int(i) for i in ids], outs, tmax, docs, bytes_out, errs))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_matches_single_process():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref
    from yjs_amd.distributed import shard_batch
    from yjs_amd.workloads import load_ymb
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    a, o, d = load_ymb("c2_v1")
    ref, st, ol = oracle_ref.batch("merge", 1, *shard_batch(a, o, d, 0, 96))
    merged = [None] * 96
    for r in res:
        for i, x in zip(r[1], r[2]):
            assert merged[i] is None
            merged[i] = x
    assert merged == ref
    for r in res:
        assert r[3] == 1.5                      # max over ranks
        assert r[4] == 96                       # docs summed over ranks
        assert r[5] == float(np.sum(ol))        # bytes summed over ranks
        assert r[6] == 0


class _OracleRunner:
    """Stands in for yjs_amd.Engine(device) in the CPU test of MultiDeviceEngine's partition/reassembly."""

    def __init__(self, device):
        self.device = device

    def run_host(self, op, fmt, arena, upd_off, doc_upd, sv_arena=None, sv_off=None):
        import sys
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ref
        from yjs_amd import pack_docs
        outs, st, _ = oracle_ref.batch(op, fmt, arena, upd_off, doc_upd, sv_arena, sv_off)
        blobs = [x if isinstance(x, bytes) else b"" for x in outs]
        oa, oo, _ = pack_docs([[b] for b in blobs])
        return oa, oo[:-1], np.diff(oo.astype(np.int64)).astype(np.uint64), st


def test_multi_device_engine_reassembles_doc_order():
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref
    from yjs_amd.distributed import MultiDeviceEngine, gather_docs
    from yjs_amd.workloads import load_ymb
    a, o, d = load_ymb("c2_v1")
    a, o, d = gather_docs(a, o, d, np.arange(40))
    ref, st, _ = oracle_ref.batch("merge", 1, a, o, d)
    made = []

    def runner(device):
        made.append((device, threading.get_ident()))
        return _OracleRunner(device)

    for how in ("hash", "bytes"):
        made.clear()
        with MultiDeviceEngine([0, 1, 2], how, runner=runner) as eng:
            for _ in range(3):  # one engine per device, made once on its own long-lived worker thread
                assert eng.run_host("merge", 1, a, o, d) == ref
        assert sorted(m[0] for m in made) == [0, 1, 2], made
        assert len({m[1] for m in made}) == 3 and threading.get_ident() not in {m[1] for m in made}
