"""bench.py's real multi-rank path on the one GPU of a test box: `bench.py --gpus 2` starts two rank
processes, each merges its hash32 shard with the real engine (libymerge.so), and the max-time / summed
counters reduce runs over torch.distributed.  Both ranks are pinned to device 0 (YMERGE_BENCH_DEVICE); the
summed counters must equal a one-rank run over the same documents (disjoint shards, no
collective in the hot path)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(gpus, docs_per_gpu, backend=None, pin=True):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    if pin:
        env["YMERGE_BENCH_DEVICE"] = "0"
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    if backend:
        env["YMERGE_BENCH_BACKEND"] = backend
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--steps", "3",
                        "--warmup", "1", "--rotate", "1", "--docs-per-gpu", str(docs_per_gpu), "--no-secondary",
                        "--no-cpu-baseline"], capture_output=True, text=True, env=env, timeout=240, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def _gpus():
    import torch
    return torch.cuda.device_count()


# RCCL refuses two ranks on one device ("Duplicate GPU detected : rank 1 and rank 0 both on CUDA device",
# ncclInvalidUsage, measured on the one-GPU box): with one GPU the ranks reduce over gloo -- the engine, the
# sharding and the max-time / summed-counter reduction are the same code; RCCL runs when the box has two GPUs.
@pytest.mark.parametrize("backend", ["nccl", "gloo"])
def test_bench_two_ranks_real_engine(backend):
    if backend == "nccl" and _gpus() < 2:
        pytest.skip("RCCL rejects two ranks on one device; this box has one GPU")
    one = _bench(1, 4000)
    two = _bench(2, 2000, backend, pin=backend != "nccl")
    assert two["n_gpus"] == 2 and two["config"]["reduce_backend"] == backend
    for k in ("docs_total", "updates_total", "input_bytes_total", "output_bytes_total"):
        assert two["config"][k] == one["config"][k], k
    assert two["doc_errors"] == 0 and one["doc_errors"] == 0
    assert two["docs_fast_path"] + two["docs_general_path"] == one["docs_fast_path"] + one["docs_general_path"]
    assert two["value"] > 0 and "stub" not in two
