"""The large-document merge's segmented radix sort (ym_segsort.hip, one workgroup per segment) against
numpy's stable argsort: segments of every size class (empty, one pair, the LDS-resident bound 4096 and one
past it, ~20 k pairs in HBM passes), duplicate keys (stability), constant digits (skipped passes), full
64-bit keys, and pairs between segments left unwritten."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from yjs_amd import Engine
    return Engine(0)


def _run(engine, keys, vals, segs):
    import torch
    dev = torch.device("cuda", 0)
    n = len(keys)
    ki = torch.from_numpy(keys.view(np.int64)).to(dev)
    vi = torch.from_numpy(vals.view(np.int32)).to(dev)
    ko = torch.full((n,), -1, dtype=torch.int64, device=dev)
    vo = torch.full((n,), -1, dtype=torch.int32, device=dev)
    kt = torch.empty(n, dtype=torch.int64, device=dev)
    vt = torch.empty(n, dtype=torch.int32, device=dev)
    sb = torch.from_numpy(np.array([s[0] for s in segs], dtype=np.int32)).to(dev)
    se = torch.from_numpy(np.array([s[1] for s in segs], dtype=np.int32)).to(dev)
    f = engine.lib.ym__segsort
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p] * 8 + [ctypes.c_uint32]
    rc = f(ki.data_ptr(), vi.data_ptr(), ko.data_ptr(), vo.data_ptr(), kt.data_ptr(), vt.data_ptr(), sb.data_ptr(),
           se.data_ptr(), len(segs))
    assert rc == 0
    return ko.cpu().numpy().view(np.uint64), vo.cpu().numpy().view(np.uint32)


def _check(engine, keys, vals, segs):
    ko, vo = _run(engine, keys, vals, segs)
    covered = np.zeros(len(keys), bool)
    for b, e in segs:
        if e <= b:
            continue
        order = np.argsort(keys[b:e], kind="stable")
        assert np.array_equal(ko[b:e], keys[b:e][order]), (b, e)
        assert np.array_equal(vo[b:e], vals[b:e][order]), (b, e)
        covered[b:e] = True
    assert np.all(ko[~covered] == np.uint64(0xFFFFFFFFFFFFFFFF))
    assert np.all(vo[~covered] == np.uint32(0xFFFFFFFF))


def _layout(sizes, gap=3):
    segs, p = [], 0
    for s in sizes:
        segs.append((p, p + s))
        p += s + gap
    return segs, p


def test_segsort_size_classes(engine):
    rng = np.random.default_rng(7)
    sizes = [0, 1, 2, 3, 63, 64, 65, 1000, 1024, 1025, 4095, 4096, 4097, 8192, 20011]
    segs, n = _layout(sizes)
    # run keys: ~client << 32 | clock over a few clients (duplicates on purpose)
    clients = rng.integers(0, 2**32, size=64, dtype=np.uint64)
    ck = (~clients[rng.integers(0, 64, size=n)]) & np.uint64(0xFFFFFFFF)
    keys = (ck << np.uint64(32)) | rng.integers(0, 5000, size=n, dtype=np.uint64)
    vals = np.arange(n, dtype=np.uint32)
    _check(engine, keys, vals, segs)


def test_segsort_stability_and_constant_digits(engine):
    rng = np.random.default_rng(11)
    segs, n = _layout([5000, 300, 9000, 4096])
    keys = np.zeros(n, dtype=np.uint64)
    b, e = segs[0]
    keys[b:e] = np.uint64(0x1234) << np.uint64(40)  # all equal: every digit constant, copied
    b, e = segs[1]
    keys[b:e] = rng.integers(0, 4, size=e - b, dtype=np.uint64) << np.uint64(56)  # one permuting digit
    b, e = segs[2]
    keys[b:e] = rng.integers(0, 2**64, size=e - b, dtype=np.uint64, endpoint=False)  # all eight digits
    b, e = segs[3]
    keys[b:e] = rng.integers(0, 3, size=e - b, dtype=np.uint64)  # heavy duplicates, LDS path
    vals = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    _check(engine, keys, vals, segs)


def test_segsort_many_segments(engine):
    rng = np.random.default_rng(3)
    sizes = list(rng.integers(0, 3000, size=300))
    segs, n = _layout(sizes, gap=0)
    keys = rng.integers(0, 2**40, size=n, dtype=np.uint64)
    vals = np.arange(n, dtype=np.uint32)
    _check(engine, keys, vals, segs)
