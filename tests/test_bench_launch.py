"""bench.py's own multi-GPU path, rehearsed on CPU: `bench.py --gpus 2` (no external launcher) must start
two rank processes, shard the weak-scaling job by hash32(docIndex) % N (or greedy byte balance), and
reduce max-time / summed counters with torch.distributed (gloo here, RCCL on the GPUs).  --cpu-stub
replaces the merge by a copy: what is tested is the launcher / sharding / reduce plumbing."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from yjs_amd.distributed import (byte_partition, doc_sizes, gather_docs, hash32, hash_partition,  # noqa: E402
                                 weak_scaling_shard)
from yjs_amd.workloads import load_ymb  # noqa: E402


def _run_bench(*extra):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-stub", "--steps", "2", "--warmup", "1",
                        "--no-secondary", "--no-cpu-baseline", *extra], capture_output=True, text=True, env=env,
                       timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    return json.loads(lines[0])


@pytest.mark.parametrize("partition", ["hash", "bytes"])
def test_bench_launches_two_ranks(partition):
    D = 64
    line = _run_bench("--gpus", "2", "--docs-per-gpu", str(D), "--partition", partition)
    assert line["n_gpus"] == 2
    a, o, d = load_ymb("c2_v1")
    T = len(d) - 1
    sizes = doc_sizes(o, d)[np.arange(2 * D) % T]
    assert line["config"]["docs_total"] == 2 * D
    assert line["config"]["input_bytes_total"] == int(sizes.sum())
    assert line["config"]["output_bytes_total"] == int(sizes.sum())  # the stub copies its input
    assert line["config"]["updates_total"] == int(np.diff(d.astype(np.int64))[np.arange(2 * D) % T].sum())
    assert line["doc_errors"] == 0
    assert partition in line["config"]["parallelism"]


def test_hash_partition_rule_and_cover():
    ids = np.arange(1000)
    shards = hash_partition(ids, 4)
    allid = np.sort(np.concatenate(shards))
    assert (allid == ids).all()
    for r, s in enumerate(shards):
        assert (hash32(s) % 4 == r).all()
    # balanced within a few sqrt(n)
    assert max(len(s) for s in shards) - min(len(s) for s in shards) < 100


def test_byte_partition_balances_skewed_sizes():
    rng = np.random.default_rng(3)
    sizes = (rng.pareto(1.5, 256) * 1e5).astype(np.int64) + 1
    shards = byte_partition(sizes, 8)
    allid = np.sort(np.concatenate(shards))
    assert (allid == np.arange(256)).all()
    loads = [int(sizes[s].sum()) for s in shards]
    # LPT: the heaviest shard exceeds the mean by at most the largest document
    assert max(loads) <= sizes.sum() / 8 + sizes.max()


def test_weak_scaling_shards_are_disjoint_copies():
    a, o, d = load_ymb("c2_v1")
    T = len(d) - 1
    parts = [weak_scaling_shard(a, o, d, 50, 3, r, "hash") for r in range(3)]
    ids = np.sort(np.concatenate([p[3] for p in parts]))
    assert (ids == np.arange(150)).all()
    for sa, so, sd, gid in parts:
        for i, g in enumerate(gid[:10]):
            t = int(g) % T
            want = a[int(o[d[t]]):int(o[d[t + 1]])].tobytes()
            got = sa[int(so[sd[i]]):int(so[sd[i + 1]])].tobytes()
            assert got == want


def test_gather_docs_roundtrip():
    a, o, d = load_ymb("c2_v1")
    ids = np.array([5, 0, 5, 17])
    ga, go, gd = gather_docs(a, o, d, ids)
    assert len(gd) == 5
    for i, t in enumerate(ids):
        for k in range(int(gd[i + 1] - gd[i])):
            u, v = int(d[t]) + k, int(gd[i]) + k
            assert ga[int(go[v]):int(go[v + 1])].tobytes() == a[int(o[u]):int(o[u + 1])].tobytes()
