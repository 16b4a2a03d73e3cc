"""Runs batches through the TEST-ONLY host build of the device core (tests/native/core_host.cpp: the
general path's general_doc() compiled for the CPU, optionally under ASan + UBSan).  Same batch layout as
the C ABI; returns (outputs list (bytes or None), status ndarray)."""
import os
import struct
import subprocess
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
OPS = {"merge": 0, "diff": 1, "sv": 2, "conv": 3, "meta": 4, "dsmerge": 5, "snap": 6, "compact": 7}


def binary(san=False):
    exe = os.path.join(NATIVE, "_build", "core_host_san" if san else "core_host")
    subprocess.check_call(["make", "-s", "-C", NATIVE, os.path.relpath(exe, NATIVE)])
    return exe


def run(op, fmt, arena, upd_off, doc_upd, sv_arena=None, sv_off=None, san=False):
    arena = np.ascontiguousarray(arena, np.uint8)
    upd_off = np.ascontiguousarray(upd_off, np.uint64)
    doc_upd = np.ascontiguousarray(doc_upd, np.uint32)
    nd = len(doc_upd) - 1
    if op in ("compact_sv", "compact_nogc_sv"):  # YM_SV_FIRST: encodeStateVector(doc), then the update
        op, fmt = op[:-3], fmt | 0x10000
    if op in ("compact", "compact_nogc") and sv_arena is not None:
        fmt |= 0x8000  # core_host.cpp: the batch carries target state vectors (ym_batch.sv_arena != NULL)
    if sv_arena is None:
        sv_arena = np.zeros(0, np.uint8)
        sv_off = np.zeros(nd + 1, np.uint64)
    sv_arena = np.ascontiguousarray(sv_arena, np.uint8)
    sv_off = np.ascontiguousarray(sv_off, np.uint64)
    if op == "dsmerge_ref":  # ym_ds_merge with YM_DS_REF: the reference's adjacency-only coalescing
        op, fmt = "dsmerge", fmt | 0x100
    if op == "compact_nogc":  # ym_compact with YM_NO_GC: new Y.Doc({ gc: false })
        op, fmt = "compact", fmt | 0x4000
    if op in ("snap_to_v1", "snap_to_v2"):  # ym_snapshot with YM_OUT_V1 / YM_OUT_V2
        op, fmt = "snap", fmt | (0x2000 if op == "snap_to_v2" else 0x1000)
    exe = binary(san)
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in"), os.path.join(td, "out")
        with open(fin, "wb") as f:
            f.write(struct.pack("<IIIIQQ", OPS[op], fmt, nd, len(upd_off) - 1, len(arena), len(sv_arena)))
            f.write(doc_upd.tobytes())
            f.write(upd_off.tobytes())
            f.write(arena.tobytes())
            f.write(sv_off.tobytes())
            f.write(sv_arena.tobytes())
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
        r = subprocess.run([exe, fin, fout], capture_output=True, text=True, env=env, timeout=600)
        assert r.returncode == 0, r.stderr[-4000:]
        raw = open(fout, "rb").read()
    outs, st, pos = [], np.zeros(nd, np.int32), 0
    for d in range(nd):
        s, n = struct.unpack_from("<iQ", raw, pos)
        pos += 12
        st[d] = s
        outs.append(raw[pos:pos + n] if s == 0 else None)
        pos += n
    return outs, st
