"""The Node.js drop-in (js/index.js -> N-API addon -> libymerge.so -> MI355X) reproduces every golden
vector with yjs's own function names and exception classes."""
import json
import os
import shutil
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed on this box")
def test_js_api_golden():
    r = subprocess.run(["node", os.path.join(ROOT, "js", "test", "golden.js")], capture_output=True, text=True, timeout=600)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert line, r.stderr[-3000:]
    res = json.loads(line[-1])
    assert r.returncode == 0 and res["bad"] == 0, res
    assert res["ok"] >= 990 and res["unsupported"] == 0, res
    assert res["async_ok"] >= 800, res  # mergeUpdatesBatchAsync (napi_async_work) over the golden merges
    assert res["compact_ok"] >= 1000, res  # compactUpdatesBatch with gc: false and target state vectors


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed on this box")
def test_js_sync_round():
    r = subprocess.run(["node", os.path.join(ROOT, "js", "test", "sync.js")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed on this box")
def test_js_big_batch_pipelined():
    """10,000 C2 documents in one mergeUpdatesBatch call (page-locked packing, u32 offsets, the pipelined host
    path) give the bytes of the same documents merged 100 at a time."""
    r = subprocess.run(["node", os.path.join(ROOT, "js", "test", "bigbatch.js")], capture_output=True, text=True, timeout=300)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert line, r.stderr[-3000:]
    res = json.loads(line[-1])
    assert r.returncode == 0 and res["bad"] == 0 and res["docs"] == 10000, res
