"""Benchmark / test workloads: yjs-13.5.16-generated document templates (bench_data/*.ymb.gz, recipe
oracle/gen/make_bench_data.cjs, shapes per SURVEY.md §8(d)) replicated into large batches."""
import gzip
import os

import numpy as np

DATA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench_data")


def load_ymb(name):
    """Returns (arena u8, upd_off u64, doc_upd u32) of bench_data/<name>.ymb.gz."""
    with gzip.open(os.path.join(DATA_DIR, name + ".ymb.gz"), "rb") as f:
        raw = f.read()
    assert raw[:4] == b"YMB1", name
    n_docs, n_upd = np.frombuffer(raw, np.uint32, 2, 4)
    o = 12
    doc_upd = np.frombuffer(raw, np.uint32, n_docs + 1, o).copy()
    o += 4 * (n_docs + 1)
    upd_off = np.frombuffer(raw, np.uint64, n_upd + 1, o).copy()
    o += 8 * (n_upd + 1)
    arena = np.frombuffer(raw, np.uint8, int(upd_off[-1]), o).copy()
    return arena, upd_off, doc_upd


def replicate(arena, upd_off, doc_upd, n_docs):
    """Batch of n_docs documents, doc i = template i % T (each a distinct copy in the arena)."""
    T = len(doc_upd) - 1
    reps = (n_docs + T - 1) // T
    k = np.diff(doc_upd.astype(np.int64))
    doc_bytes = (upd_off[doc_upd[1:]] - upd_off[doc_upd[:-1]]).astype(np.int64)
    # full copies of the template set, then truncate to n_docs docs
    arena_r = np.tile(arena, reps)
    lens = np.diff(upd_off.astype(np.int64))
    lens_r = np.tile(lens, reps)
    upd_off_r = np.zeros(len(lens_r) + 1, np.uint64)
    np.cumsum(lens_r, out=upd_off_r[1:])
    k_r = np.tile(k, reps)[:n_docs]
    doc_upd_r = np.zeros(n_docs + 1, np.uint32)
    np.cumsum(k_r, out=doc_upd_r[1:])
    n_upd = int(doc_upd_r[-1])
    upd_off_r = upd_off_r[:n_upd + 1]
    nbytes = int(upd_off_r[-1])
    del doc_bytes
    return arena_r[:nbytes].copy(), upd_off_r, doc_upd_r


def encode_sv(pairs):
    out = bytearray()

    def vu(v):
        while v > 127:
            out.append(0x80 | (v & 127))
            v >>= 7
        out.append(v)
    vu(len(pairs))
    for c, k in pairs:
        vu(c)
        vu(k)
    return bytes(out)


def decode_sv(b):
    pos = 0

    def vu():
        nonlocal pos
        s, n = 0, 0
        while True:
            x = b[pos]
            pos += 1
            s |= (x & 127) << n
            n += 7
            if x < 128:
                return s
    cnt = vu()
    return [(vu(), vu()) for _ in range(cnt)]


def random_state_vectors(full_sv, n_docs, seed=1):
    """SV per doc: {client: U[0, state]}, with 10% empty and 10% full."""
    rng = np.random.default_rng(seed)
    pairs = decode_sv(full_sv)
    svs = []
    for _ in range(n_docs):
        r = rng.random()
        if r < 0.1:
            svs.append(encode_sv([]))
        elif r < 0.2:
            svs.append(full_sv)
        else:
            svs.append(encode_sv([(c, int(rng.integers(0, k + 1))) for c, k in pairs]))
    return svs
