#!/usr/bin/env python3
"""Benchmark: batched Y.mergeUpdates on MI355X (BASELINE.json configs[1] = C2).

A step is one ym_merge call over the rank's device-resident batch of C2 documents (10k docs x ~100
Y.Text updates each, 4 clients, V1): inputs already in HBM when the timed region starts, outputs left
in HBM.  N GPUs = N ranks (torch.distributed over RCCL), each processing its own shard of distinct
documents (weak scaling: docs per GPU fixed).  The only collectives are the max of the elapsed time
and the sum of the per-rank stats.

Prints ONE JSON line (rank 0) with value = whole-job merged-update input GB/s, plus docs/s, the
roofline of the dominant kernel (the LDS fast-path merge, algorithmic bytes = sum of input + output
bytes of its documents, timed with HIP events on the call's stream) and the CPU baseline (the C
restatement in oracle/ -- a faithful port of yjs 13.5.16's algorithm -- on a bounded sample, timed on
the host cores of the same box).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md: 8.0 TB/s spec)
METRIC = "merged update GB/s (node) + docs/sec, batched Y.mergeUpdates; % HBM peak"

WORKLOADS = {
    # name: (template file, format, description)
    "c2": ("c2_v1", 1, "C2: 10k docs x 100 Y.Text updates (4 clients), batched mergeUpdates V1"),
    "c2v2": ("c2_v2", 2, "C2 shape, batched mergeUpdatesV2"),
    "c4": ("c4_v1", 1, "C4: Y.Map docs, 64 clients, 128 broadcast tx, delete-heavy, mergeUpdates V1"),
    "c5": ("c5_v1", 1, "C5: Y.XmlFragment docs, 1,024 clients x 16 tx (~16 k updates), mergeUpdates V1"),
    "c5v2": ("c5_v2", 2, "C5: Y.XmlFragment docs, 1,024 clients x 16 tx (~16 k updates), mergeUpdatesV2"),
}
PARTITION = {"c2": "hash", "c2v2": "hash", "c4": "hash", "c5": "bytes", "c5v2": "bytes"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    p.add_argument("--docs-per-gpu", type=int, default=10000)
    p.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--partition", default="auto", choices=["auto", "hash", "bytes"],
                   help="document -> rank assignment: hash32(docIndex) % N, or greedy byte balance "
                        "(auto: hash for the small-document workloads, bytes for C3 / C5)")
    p.add_argument("--cpu-stub", action="store_true",
                   help="gloo on CPU with a copy standing in for the merge (tests of the launcher only)")
    p.add_argument("--rotate", type=int, default=12,
                   help="distinct device copies of the batch, one per step in turn (12 x the C2 batch = "
                        "~1 GB of inputs + outputs: above the 256 MiB on-die cache, so the roofline is HBM's)")
    p.add_argument("--submit", default="auto", choices=["auto", "async", "sync"],
                   help="async: each step is one ym_merge_async call (the LDS fast path enqueued on the "
                        "stream, no host round trip; the serving loop's form), verified in the warmup to "
                        "complete every document with the bytes of ym_merge; sync: one ym_merge call per "
                        "step (host waits for each); auto: async when the verification passes")
    p.add_argument("--no-secondary", action="store_true",
                   help="skip the secondary workload lines (C4/C2-V2/C4-V2 merges, C3 diff/sv)")
    return p.parse_args()


def cpu_baseline(arena, upd_off, doc_upd, fmt, seconds, op="merge"):
    """The oracle (CPU port of yjs 13.5.16 mergeUpdates; op="compact": of the reference's Doc round trip)
    over the same documents, all host threads of this process's CPU share, repeated until `seconds` of wall
    time."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref  # test infrastructure: only the cpu_baseline leg may load it
    threads = host_cores()
    n_docs = len(doc_upd) - 1
    reps, t0 = 0, time.perf_counter()
    while True:
        _, st, out_len = oracle_ref.batch(op, fmt, arena, upd_off, doc_upd, nthreads=threads, want_output=False)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    bytes_in = float(upd_off[-1] - upd_off[0]) * reps
    return {
        "value": round(bytes_in / el / 1e9, 5),
        "unit": "GB/s",
        "docs_per_s": round(n_docs * reps / el, 1),
        "cores": threads,
        "host_cpu_count": os.cpu_count(),
        "kind": "port",
        "sample": f"{reps} x {n_docs} docs ({bytes_in / reps / 1e6:.1f} MB input each) in {el:.1f} s, "
                  + ("oracle/ymerge_oracle.c compact_impl (the reference's 13.4.9 Doc round trip restated)"
                     if op == "compact" else "oracle/ymerge_oracle.c (literal yjs 13.5.16 mergeUpdates)")
                  + f", {threads} threads",
        "errors": int((st != 0).sum()),
        # the port is faster than the JS it restates: per-thread ratios measured on identical C2 / C4
        # documents in the build container by tools/calibrate.py (JS cannot run on the GPU box)
        "calibration": _calibration() if op == "merge" else None,
        # the whole machine's cores at the measured per-thread rate (what a host-side deployment could reach)
        "all_host_cores_estimate": {"cores": os.cpu_count(),
                                    "docs_per_s": round(n_docs * reps / el / threads * (os.cpu_count() or 1), 1)},
    }


def _calibration():
    """The per-thread C-port / JS ratios of the last tools/calibrate.py run (profiles/calibration.json)."""
    try:
        c = json.load(open(os.path.join(ROOT, "profiles", "calibration.json")))
    except (OSError, ValueError):
        return None
    w = c.get("workloads", {})
    return {"port_over_yjs_13_5_16_js": {k.split("_")[0]: v["port_over_yjs_13_5_16_js"] for k, v in w.items()},
            "port_over_reference_13_4_9_doc_roundtrip": {k.split("_")[0]: v["port_over_reference_13_4_9_doc_roundtrip"]
                                                         for k, v in w.items()},
            "source": f"profiles/calibration.json (tools/calibrate.py, {c.get('docs')} docs, 1 thread, "
                      f"measured {c.get('measured_utc')})"}


def _ds_v1_to_v2(b):
    """An encoded delete set, DSEncoderV1 -> DSEncoderV2 bytes (delta-coded clocks, len - 1)."""
    pos, out = 0, bytearray()

    def rd():
        nonlocal pos
        v, sh = 0, 0
        while True:
            x = b[pos]
            pos += 1
            v |= (x & 127) << sh
            sh += 7
            if x < 128:
                return v

    def wr(v):
        while v > 127:
            out.append(0x80 | (v & 127))
            v >>= 7
        out.append(v)
    n = rd()
    wr(n)
    for _ in range(n):
        wr(rd())
        m = rd()
        wr(m)
        cur = 0
        for _ in range(m):
            clock, ln = rd(), rd()
            wr(clock - cur)
            wr(ln - 1)
            cur = clock + ln
    return bytes(out)


def secondary(dev, eng):
    """Quick device-resident measurements of the other BASELINE.json workloads (1 GPU): C4 and V2
    merges (10k docs), C3 diffUpdate / encodeStateVectorFromUpdate (configs[2]: 4,096 V1 docs of
    0.9 MB V1 and 0.47 MB V2) against random state vectors, C5 (configs[4]: 256 docs of ~16 k updates
    from 1,024 clients) mergeUpdates[V2] and diffUpdate[V2] of the merged documents against random
    per-client state vectors, parseUpdateMeta over the ~1 M C2 updates, PermanentUserData's
    delete-set merge over the C4 updates' delete sets.  Whole-call GB/s of input."""
    import torch
    from yjs_amd import pack_docs
    from yjs_amd.workloads import load_ymb, replicate, random_state_vectors
    res = {}
    only = os.environ.get("YM_SECONDARY")  # comma-separated subset of the case names
    cases = [("merge_c4_v1", "merge", "c4_v1", 10000), ("merge_c2_v2", "merge", "c2_v2", 10000),
             ("merge_c4_v2", "merge", "c4_v2", 10000), ("diff_c3_v1", "diff", "c3_v1", 4096),
             ("sv_c3_v1", "sv", "c3_v1", 4096), ("diff_c3_v2", "diff", "c3_v2", 4096),
             ("sv_c3_v2", "sv", "c3_v2", 4096),
             ("merge_c5_v1", "merge", "c5_v1", 256), ("merge_c5_v2", "merge", "c5_v2", 256),
             ("diff_c5_v1", "diff", "c5_v1", 256), ("diff_c5_v2", "diff", "c5_v2", 256),
             ("meta_c2_v1", "meta", "c2_v1", 10000), ("meta_c2_v2", "meta", "c2_v2", 10000),
             ("meta_c3_v1", "meta", "c3_v1", 4096), ("meta_c3_v2", "meta", "c3_v2", 4096),
             ("dsmerge_c4_v1", "dsmerge", "c4_v1", 10000), ("dsmerge_c4_v2", "dsmerge", "c4_v1", 10000),
             # configs[3] at its per-GPU shard: 1 M docs over 8 GPUs = 125 k docs, 4,096 distinct templates
             ("merge_c4_v1_125k", "merge", "c4_v1", 125000),
             # Doc round-trip compaction (the reference's applyUpdate x N +
             # encodeStateAsUpdate on a gc=true Doc) of the C2 / C4 documents
             ("compact_c2_v1", "compact", "c2_v1", 10000), ("compact_c2_v2", "compact", "c2_v2", 10000),
             ("compact_c4_v1", "compact", "c4_v1", 10000),
             # rich content: Quill-style formats / embeds, maps of objects and arrays
             ("merge_c2r_v1", "merge", "c2r_v1", 10000), ("merge_c2r_v2", "merge", "c2r_v2", 10000),
             ("merge_c4r_v1", "merge", "c4r_v1", 10000), ("merge_c4r_v2", "merge", "c4r_v2", 10000),
             ("diff_c2r_v1", "diff", "c2r_v1", 4096), ("diff_c2r_v2", "diff", "c2r_v2", 4096),
             ("sv_c4r_v1", "sv", "c4r_v1", 4096), ("diff_c4r_v2", "diff", "c4r_v2", 4096),
             # the sync server's SyncStep1 -> SyncStep2 load: diffUpdate / state vector of
             # the merged C2 documents (~1 KB each) against random state vectors
             ("diff_c2_v1", "diff", "c2_v1", 10000), ("sv_c2_v1", "sv", "c2_v1", 10000),
             ("diff_c2_v2", "diff", "c2_v2", 10000), ("sv_c2_v2", "sv", "c2_v2", 10000),
             # realistic text: C2U, the C2 shape with CJK / emoji / accented words and pastes
             ("merge_c2u_v1", "merge", "c2u_v1", 10000), ("merge_c2u_v2", "merge", "c2u_v2", 10000),
             ("diff_c2u_v1", "diff", "c2u_v1", 10000), ("sv_c2u_v1", "sv", "c2u_v1", 10000),
             ("diff_c2u_v2", "diff", "c2u_v2", 10000), ("sv_c2u_v2", "sv", "c2u_v2", 10000)]
    for name, op, wl, n in cases:
        if only and name not in only.split(","):
            continue
        try:
            res[name] = _secondary_case(dev, eng, name, op, wl, n)
        except Exception as e:  # one failing line must not take the headline line down with it
            res[name] = {"error": f"{type(e).__name__}: {e}"}
        torch.cuda.empty_cache()
    return res


def _secondary_case(dev, eng, name, op, wl, n):
    """One secondary line (see secondary())."""
    import torch
    from yjs_amd import pack_docs
    from yjs_amd.workloads import load_ymb, replicate, random_state_vectors
    if True:
        fmt = 2 if wl.endswith("v2") else 1
        a, o, d = load_ymb(wl)
        sva = svo = None
        if op in ("merge", "compact"):
            a, o, d = replicate(a, o, d, n)
        elif op == "meta":
            # parseUpdateMeta of every update of n C2 documents (~1 M single-update batch entries)
            a, o, d = replicate(a, o, d, n)
            d = np.arange(len(o), dtype=np.uint32)
        elif op == "dsmerge":
            # PermanentUserData-style: per document, the encoded delete sets of its C4 updates (the DS of
            # update u is diffUpdate(u, parseUpdateMeta(u).to) minus its empty struct section, vu(0)),
            # merged into one
            from yjs_amd import decode_meta
            from yjs_amd.workloads import encode_sv
            nt = min(1000, len(d) - 1)  # 1,000 templates (128 k updates), replicated to n documents
            a, o, d = a[:int(o[d[nt]])], o[:int(d[nt]) + 1], d[:nt + 1]
            per = np.arange(len(o), dtype=np.uint32)
            sa, so_, sl, sst = eng.run_host("meta", 1, a, o, per)
            svs = [encode_sv(list(decode_meta(sa[int(so_[i]):int(so_[i]) + int(sl[i])].tobytes())["to"].items()))
                   for i in range(len(sst))]
            sva_, svo_, _ = pack_docs([[x] for x in svs])
            da, do_, dl, dst = eng.run_host("diff", 1, a, o, per, sva_, svo_)
            assert (sst == 0).all() and (dst == 0).all()
            blobs = [da[int(do_[i]) + 1:int(do_[i]) + int(dl[i])].tobytes() for i in range(len(dst))]
            if name.endswith("v2"):  # the same delete sets in the DSEncoderV2 format
                blobs = [_ds_v1_to_v2(x) for x in blobs]
                fmt = 2
            docs = [[blobs[u] for u in range(int(d[t]), int(d[t + 1]))] for t in range(len(d) - 1)]
            a, o, d = replicate(*pack_docs(docs), n)
        elif wl.startswith("c5") or wl[:3] in ("c2r", "c4r") or (op in ("diff", "sv") and wl[:2] in ("c2", "c4")):
            # the merged documents (merged here by the engine), random per-client state vectors
            ma, mo, ml, _ = eng.run_host("merge", fmt, a, o, d)
            ups = [ma[int(mo[i]):int(mo[i]) + int(ml[i])].tobytes() for i in range(len(d) - 1)]
            sa, so_, sl, _ = eng.run_host("sv", fmt, *pack_docs([[u] for u in ups]))
            fulls = [sa[int(so_[i]):int(so_[i]) + int(sl[i])].tobytes() for i in range(len(ups))]
            svs = [random_state_vectors(fulls[i % len(ups)], 1, seed=i)[0] for i in range(n)]
            a, o, d = pack_docs([[ups[i % len(ups)]] for i in range(n)])
            sva, svo, _ = pack_docs([[x] for x in svs])
        else:
            upd = a.tobytes()
            a, o, d = replicate(a, o, d, n)  # n copies of the single C3 update (diff / sv / meta)
            if op == "diff":
                # the update's own state vector (one client: the trace's), random cuts per document
                full = _sv_of_single_client_update(upd, fmt)
                svs = random_state_vectors(full, n, seed=7)
                sva, svo, _ = pack_docs([[x] for x in svs])
        nd = len(d) - 1
        ga = torch.from_numpy(a).to(dev)
        # u32 update offsets (YM_OFF32) for the merges, as the headline line
        off32 = op in ("merge", "dsmerge") and len(a) < 2 ** 32
        go = torch.from_numpy(o.astype(np.uint32).view(np.int32) if off32 else o.view(np.int64)).to(dev)
        gd = torch.from_numpy(d.view(np.int32)).to(dev)
        gsa = torch.from_numpy(sva).to(dev) if sva is not None else None
        gso = torch.from_numpy(svo.view(np.int64)).to(dev) if svo is not None else None
        cap = 4 * len(a) + 128 * nd + 8192 + (2 * len(sva) if sva is not None else 0)
        oa = torch.empty(cap, dtype=torch.uint8, device=dev)
        oo = torch.empty(nd, dtype=torch.int64, device=dev)
        ol = torch.empty(nd, dtype=torch.int64, device=dev)
        st = torch.empty(nd, dtype=torch.int32, device=dev)
        steps = 5 if op in ("merge", "meta", "dsmerge") else 2
        rc0, used0 = eng.run_device(op, fmt, ga, go, gd, oa, oo, ol, st, gsa, gso)
        for _ in range(3):  # YM_ERR_CAPACITY: the call reports what it needed so far (the streamed V2 diff
            # walker uses the output arena as scratch, ~2 KB per client section); a caller grows the arena
            if rc0 != 9:
                break
            cap = 2 * used0 + 65536
            oa = torch.empty(cap, dtype=torch.uint8, device=dev)
            rc0, used0 = eng.run_device(op, fmt, ga, go, gd, oa, oo, ol, st, gsa, gso)
        if rc0 != 0:
            raise RuntimeError(f"rc {rc0} (used {used0} of cap {cap})")
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        kms = []
        for _ in range(steps):
            rc, _ = eng.run_device(op, fmt, ga, go, gd, oa, oo, ol, st, gsa, gso)
            assert rc == 0, rc
            # device time of the call's kernels: the specialised path, the large-document pipeline and the
            # general path (one thread per document: parseUpdateMeta of ~1 M small updates runs there)
            kms.append(eng.last_stats.fast_ms + eng.last_stats.large_ms + eng.last_stats.general_ms)
        torch.cuda.synchronize(dev)
        el = (time.perf_counter() - t0) / steps
        sts = eng.stats
        out_b = int(ol[st == 0].sum().item())
        kms_mean = float(np.mean(kms))
        cpu = None
        if op == "compact" and not os.environ.get("YM_NO_CPU_BASELINE"):
            # the host baseline of the same documents (a bounded sample: 2,000 of them, ~2 s per pass)
            k = min(nd, 2000)
            cpu = cpu_baseline(a[:int(o[d[k]])], o[:int(d[k]) + 1], d[:k + 1], fmt, 2.0, op="compact")
        # roofline of the call's dominant kernel(s): algorithmic bytes (inputs + outputs) / their device time
        kgbs = (len(a) + out_b) / (kms_mean * 1e-3) / 1e9 if kms_mean > 0 else 0.0
        return {"docs": nd, "input_bytes": int(len(a)), "output_bytes": out_b,
                     "value_gbs": round(len(a) / el / 1e9, 3),
                     "docs_per_s": round(nd / el, 1), "ms_per_step": round(el * 1e3, 3),
                     "kernel_ms": round(kms_mean, 3), "kernel_in_plus_out_gbs": round(kgbs, 2),
                     "roofline_frac": round(kgbs / HBM_PEAK_GBS, 5), "docs_fast": int(sts["docs_fast"]),
                     "docs_large": int(sts["docs_large"]), "docs_general": int(sts["docs_general"]),
                     "errors": int(sts["docs_error"]), "update_offsets": "u32" if off32 else "u64",
                     **({"cpu_baseline": cpu} if cpu else {})}


def _sv_of_single_client_update(upd, fmt):
    """encodeStateVectorFromUpdate of a C3 template computed on the GPU engine (one client)."""
    from yjs_amd import encodeStateVectorFromUpdate, encodeStateVectorFromUpdateV2
    return (encodeStateVectorFromUpdateV2 if fmt == 2 else encodeStateVectorFromUpdate)(upd)


def host_cores():
    """Cores this process may use: the CPU affinity set, capped by a cgroup CPU quota when one is set
    (on the GPU box os.cpu_count() reports the whole machine, not this job's share)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(-(-int(q) // int(per)))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def launch(args):
    """--gpus N without an external launcher: start N rank processes (this script, RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* in their environment) before anything here touches a GPU, wait for all of them
    and return the first failing exit code.  Rank 0 prints the JSON line."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:  # one rank failed: the others would wait in a collective forever
                    q.kill()
        time.sleep(0.05)
    return rc


class StubEngine:
    """--cpu-stub: the launcher / sharding / reduce path without a GPU (gloo on CPU tensors).  The "op"
    copies each rank's arena into its output arena; it stands in for ym_merge only in the multi-rank CPU
    test of this script's own plumbing (tests/test_bench_launch.py)."""

    last_stats = type("S", (), {"fast_ms": 0.0, "large_ms": 0.0, "device_ms": 0.0})()
    stats = {"docs_fast": 0, "docs_general": 0, "docs_large": 0}

    def prepare_device(self, op, fmt, g_arena, g_off, g_doc, o_arena, o_off, o_len, o_st, stream=None):
        n = g_arena.numel()
        nd = g_doc.numel() - 1
        lens = g_off[g_doc[1:].long()] - g_off[g_doc[:-1].long()]

        def call():
            o_arena[:n].copy_(g_arena)
            o_len.copy_(lens)
            o_st.zero_()
            return 0, n
        self.stats = {"docs_fast": nd, "docs_general": 0, "docs_large": 0}
        return call


def pcie_inclusive(eng, arena, upd_off, doc_upd, fmt, in_bytes):
    """The host-resident path's rate (not `value`)."""
    # PCIe-inclusive rate of the same batch from host memory (what the Node addon hands over): the
    # arena and u32 offsets in pageable memory, the outputs into reused page-locked buffers
    # (ym_host_alloc, as the addon's output arenas); host merges of this size run pipelined (H2D of
    # chunk c + 1 under the merge and D2H of chunk c, include/ymerge.h).  Not `value`.
    # the batch as the addon packs it: arena, u32 offsets and doc ranges in page-locked pool memory
    # (addon.hostBuffer), so the copies in are DMA transfers the host does not wait on
    pa = eng.host_array(len(arena))
    pa[:] = arena
    po = eng.host_array(len(upd_off), np.uint32)
    po[:] = upd_off
    pd = eng.host_array(len(doc_upd), np.uint32)
    pd[:] = doc_upd
    hout = eng.host_out(len(doc_upd) - 1, int(2 * in_bytes + 64 * (len(doc_upd) - 1) + 8192))
    ref = eng.run_host("merge", fmt, arena, upd_off, doc_upd)  # unpipelined u64 path: same bytes
    got = eng.run_host("merge", fmt, pa, po, pd, out=hout)
    same = (np.array_equal(ref[1], got[1]) and np.array_equal(ref[2], got[2]) and
            np.array_equal(ref[3], got[3]) and np.array_equal(ref[0][:len(got[0])], got[0]))
    reps = 16
    ths = []
    for _ in range(reps):
        t1 = time.perf_counter()
        eng.run_host("merge", fmt, pa, po, pd, out=hout)
        ths.append(time.perf_counter() - t1)
    th = float(np.median(ths))  # (median: a call now and then waits several ms for the host / driver)
    tq = time.perf_counter()
    for _ in range(reps):  # the same from pageable input arrays
        eng.run_host("merge", fmt, arena, upd_off.astype(np.uint32), doc_upd, out=hout)
    tq = (time.perf_counter() - tq) / reps
    tp = time.perf_counter()
    for _ in range(3):
        eng.run_host("merge", fmt, arena, upd_off, doc_upd)
    tp = (time.perf_counter() - tp) / 3
    res = {"value": round(in_bytes / th / 1e9, 3), "unit": "GB/s",
                              "ms_per_call": round(th * 1e3, 3), "bytes_match_unpipelined": bool(same),
                              "ms_per_call_each": [round(x * 1e3, 3) for x in ths],
                              "mean_ms_per_call": round(float(np.mean(ths)) * 1e3, 3),
                              "source": "batch and outputs in page-locked pool memory (ym_host_alloc: the "
                                        "Node addon packs into it, include/ymerge.h), u32 offsets, "
                                        "pipelined chunks",
                              "pageable_input": {"value": round(in_bytes / tq / 1e9, 3),
                                                 "ms_per_call": round(tq * 1e3, 3)},
                              "fresh_arrays_u64_offsets": {"value": round(in_bytes / tp / 1e9, 3),
                                                           "ms_per_call": round(tp * 1e3, 3)}}
    hout.close()
    return res


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # YMERGE_BENCH_DEVICE pins every rank to one device (the multi-rank path rehearsed on a one-GPU box,
    # tests/test_gpu_workloads.py); YMERGE_BENCH_BACKEND picks the reduce's backend (default: RCCL on GPUs)
    if os.environ.get("YMERGE_BENCH_DEVICE"):
        local = int(os.environ["YMERGE_BENCH_DEVICE"])
    backend = os.environ.get("YMERGE_BENCH_BACKEND", "gloo" if args.cpu_stub else "nccl")
    stub = args.cpu_stub
    if stub:
        dev = torch.device("cpu")
    else:
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    red_dev = dev if backend == "nccl" else torch.device("cpu")  # where the reduce's tensors live

    from yjs_amd.distributed import weak_scaling_shard
    from yjs_amd.workloads import load_ymb

    tname, fmt, desc = WORKLOADS[args.workload]
    how = args.partition if args.partition != "auto" else PARTITION[args.workload]
    t_arena, t_off, t_doc = load_ymb(tname)
    # the job: world * docs_per_gpu documents (weak scaling), global doc g = a distinct copy of template
    # g % T, partitioned over the ranks by hash32(g) % world or greedy byte balance
    arena, upd_off, doc_upd, doc_ids = weak_scaling_shard(t_arena, t_off, t_doc, args.docs_per_gpu, world, rank, how)
    n_docs = len(doc_upd) - 1
    in_bytes = int(upd_off[-1])

    if stub:
        eng = StubEngine()
    else:
        from yjs_amd import Engine
        eng = Engine(local)
    # the host-resident path (the Node addon's), measured first -- its staging buffers and page-locked pool are
    # then allocated before the device-resident sets, as in a serving process that only takes host batches --
    # and again after the device-resident steps (pcie_inclusive.after_device_resident_steps).  Measured only
    # after them, i.e. allocated after the rotated sets' ~1 GB, the pipelined call took 1.19 ms instead of 0.80
    # (the cause is not pinned down)
    pcie_early = pcie_inclusive(eng, arena, upd_off, doc_upd, fmt, in_bytes) if world == 1 and not stub else None
    # u32 offsets (YM_OFF32) when the rank's arena is below 4 GiB: half the offset bytes per update
    off32 = in_bytes < 2 ** 32
    cap = 4 * in_bytes + 128 * n_docs + 8192  # fast-path slots (2*in + 64 per doc) + general-path room
    # a stream of its own (torch's default stream handle is NULL, which the library reads as "its own
    # stream"): the library's kernels and the bench's HIP events are then on the same stream
    stream = None if stub else torch.cuda.Stream(device=dev)
    # `rotate` distinct device copies of the batch (inputs and output arrays), used one per step in turn:
    # each step reads and writes HBM lines the previous steps did not touch
    rot = max(1, args.rotate if not stub else 1)
    sets = []
    for _ in range(rot):
        g_arena = torch.from_numpy(arena).to(dev)
        g_off = torch.from_numpy(upd_off.astype(np.uint32).view(np.int32) if off32 else upd_off.view(np.int64)).to(dev)
        g_doc = torch.from_numpy(doc_upd.view(np.int32)).to(dev)
        o_arena = torch.empty(cap, dtype=torch.uint8, device=dev)
        o_off = torch.empty(n_docs, dtype=torch.int64, device=dev)
        o_len = torch.empty(n_docs, dtype=torch.int64, device=dev)
        o_st = torch.empty(n_docs, dtype=torch.int32, device=dev)
        call = eng.prepare_device("merge", fmt, g_arena, g_off, g_doc, o_arena, o_off, o_len, o_st, stream=stream)
        sets.append((call, (g_arena, g_off, g_doc, o_arena, o_off, o_len, o_st)))
    o_len, o_st = sets[0][1][5], sets[0][1][6]
    cur = [0]

    def sync():
        if not stub:
            torch.cuda.synchronize(dev)

    def step():
        call = sets[cur[0] % rot][0]
        cur[0] += 1
        rc, used = call()
        if rc != 0:
            raise RuntimeError(f"ym_merge rc={rc}")
        return used

    for _ in range(args.warmup):
        step()
    sync()
    cur[0] = 0
    errors = int((o_st != 0).sum().item())
    st0 = dict(eng.stats)
    out_bytes = int(o_len[o_st == 0].sum().item())

    # asynchronous submission (ym_merge_async): used for the timed steps when, on every buffer set, it
    # completes every document (no YM_PENDING) with exactly ym_merge's bytes, lengths and statuses
    submit, async_calls, pending = "sync", None, None
    if not stub and args.submit != "sync":
        import torch as _t
        pending = _t.zeros(1, dtype=_t.int32, device=dev)
        async_calls = [eng.prepare_merge_async(fmt, *bufs[:3], *bufs[3:], pending=pending, stream=stream)
                       for _, bufs in sets]
        ok = True
        for (call, bufs), acall in zip(sets, async_calls):
            if not ok:
                break
            _, _, _, o_arena_k, o_off_k, o_len_k, o_st_k = bufs
            if call()[0] != 0:
                ok = False
                break
            sync()
            ref = (o_arena_k.clone(), o_off_k.clone(), o_len_k.clone(), o_st_k.clone())
            o_arena_k.fill_(0xA5)
            o_len_k.fill_(-1)
            o_st_k.fill_(-1)
            sync()  # (torch's fills run on its default stream, the library on `stream`)
            rc = acall()
            sync()
            why = [k for k, bad in (("rc", rc != 0), ("pending", int(pending.item()) != 0),
                                    ("status", not bool((o_st_k == ref[3]).all().item())),
                                    ("len", not bool((o_len_k == ref[2]).all().item())),
                                    ("off", not bool((o_off_k == ref[1]).all().item()))) if bad]
            ok = not why
            if why:
                print(f"bench: ym_merge_async verification failed ({', '.join(why)}); sync submission",
                      file=sys.stderr)
            if ok:  # every output's bytes: the ranges [off, off + len) of the documents that succeeded
                m = ref[3] == 0
                off_t, len_t = ref[1][m], ref[2][m]
                if off_t.numel():
                    end = int((off_t + len_t).max().item())
                    mark = _t.zeros(end + 1, dtype=_t.int32, device=dev)
                    mark.index_add_(0, off_t, _t.ones_like(off_t, dtype=_t.int32))
                    mark.index_add_(0, off_t + len_t, -_t.ones_like(off_t, dtype=_t.int32))
                    inside = mark.cumsum(0)[:end] > 0
                    ok = bool((o_arena_k[:end][inside] == ref[0][:end][inside]).all().item())
        if ok:
            submit = "async"
        elif args.submit == "async":
            raise RuntimeError("ym_merge_async did not reproduce ym_merge on this batch")
        pending.zero_()

    if world > 1:
        dist.barrier()
    sync()
    fast_ms, dev_ms = [], []
    if submit == "async":
        import torch as _t
        # one HIP event pair on the kernels' stream around the K back-to-back launches (an event pair per
        # launch would put two markers between consecutive kernels): their span / K is the average launch
        # duration, inter-kernel gaps included (an upper bound; the rocprofv3 kernel average is the check)
        ev0, ev1 = _t.cuda.Event(enable_timing=True), _t.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for i in range(args.steps):
            rc = async_calls[i % rot]()
            if rc != 0:
                raise RuntimeError(f"ym_merge_async rc={rc}")
        ev1.record(stream)
        sync()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        # every document of every timed step completed on the fast path (else the line is invalid)
        if int(pending.item()) != 0:
            raise RuntimeError("ym_merge_async declined documents in the timed steps")
        fast_ms = [ev0.elapsed_time(ev1) / args.steps]  # the kernel's launches, HIP events on its stream
        dev_ms = fast_ms
    else:
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
            s = eng.last_stats
            fast_ms.append(s.fast_ms + s.large_ms)  # LDS fast path, or the large-document pipeline (C5)
            dev_ms.append(s.device_ms)
        sync()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0

    # the only collectives: max of the timed region, sum of per-rank counters (RCCL over xGMI)
    from yjs_amd.distributed import reduce_run
    elapsed, (in_all, out_all, docs_all, err_all, fast_all, gen_all, upd_all) = reduce_run(
        dist if world > 1 else None, elapsed,
        [in_bytes, out_bytes, n_docs, errors, st0["docs_fast"], st0["docs_general"], int(doc_upd[-1])], device=red_dev)

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        gbs = in_all * args.steps / elapsed / 1e9
        docs_s = docs_all * args.steps / elapsed
        # roofline of the dominant kernel (fast-path merge): algorithmic bytes per launch / avg launch time
        avg_fast = float(np.mean(fast_ms)) if fast_ms else 0.0
        alg_bytes = float(in_bytes + out_bytes)  # per launch on this rank (all docs take the fast path)
        kernel_name = {1: "k_fast_merge_v1", 2: "k_fast_merge_v2"}[fmt]
        if st0["docs_large"]:
            kernel_name = "large-document pipeline (ym_large.hip: walk, segmented sorts, k_lm_doc)"
        achieved = alg_bytes / (avg_fast * 1e-3) / 1e9 if avg_fast > 0 else 0.0
        traffic, traffic_src = None, None
        pmc = os.path.join(ROOT, "profiles", f"pmc_{args.workload}.json")
        if os.path.exists(pmc) and args.docs_per_gpu == 10000 and world == 1:
            try:
                j = json.load(open(pmc))
                traffic, traffic_src = j.get("hbm_bytes_per_launch"), j.get("source")
            except Exception:
                traffic = None
        line = {
            "metric": METRIC,
            "value": round(gbs, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic: yjs 13.5.16-generated {tname} document templates (bench_data/, recipe "
                    "oracle/gen/make_bench_data.cjs) replicated to docs_per_gpu distinct copies per rank",
            "config": {"workload": desc, "docs_total": int(docs_all), "docs_per_gpu": args.docs_per_gpu,
                       "docs_rank0": n_docs, "updates_total": int(upd_all), "input_bytes_total": int(in_all),
                       "output_bytes_total": int(out_all), "format": f"v{fmt}",
                       "update_offsets": "u32 (YM_OFF32)" if off32 else "u64",
                       "parallelism": f"docs {how}-partitioned over {world} GPU(s) (one process each), "
                                      "no collective in the hot path; max-time / sum-counters all-reduce",
                       "reduce_backend": backend if world > 1 else None},
            "docs_per_s": round(docs_s, 1),
            "hbm_frac_in_plus_out": round((in_all + out_all) * args.steps / elapsed / 1e9 / (HBM_PEAK_GBS * world), 5),
            "docs_fast_path": int(fast_all), "docs_general_path": int(gen_all), "doc_errors": int(err_all),
            "device_ms_per_step": round(float(np.mean(dev_ms)), 4),
            "working_set_bytes": int((in_bytes + cap) * rot), "rotated_buffer_sets": rot,
            "submission": ("async: one ym_merge_async per step, enqueued back to back on the stream (no host "
                           "round trip per step), verified in the warmup to give ym_merge's bytes for every "
                           "document of every buffer set; 0 documents declined in the timed steps"
                           if submit == "async" else "sync: one ym_merge call per step (the host waits for each)"),
            "roofline": {"kernel": kernel_name, "bound": "issue", "roof": "hbm", "achieved": round(achieved, 2),
                         "limiter": "instruction issue (PMC: SQ_ACTIVE_INST_ANY per SIMD ~ the launch's duration, "
                                    "HBM traffic ~1.2x the algorithmic bytes; DESIGN.md section 4.1); frac is "
                                    "against the HBM roof",
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic, "traffic_source": traffic_src, "avg_launch_ms": round(avg_fast, 5),
                         "algorithmic_bytes_per_launch": int(alg_bytes)},
        }
        if stub:
            line["stub"] = "cpu-stub: launcher/sharding/reduce plumbing only, no merge computed"
        if world == 1 and not stub:
            late = pcie_inclusive(eng, arena, upd_off, doc_upd, fmt, in_bytes)
            line["pcie_inclusive"] = dict(pcie_early, after_device_resident_steps={
                k: late[k] for k in ("value", "ms_per_call", "mean_ms_per_call", "bytes_match_unpipelined")})
        if not args.no_cpu_baseline and world == 1 and not stub:  # the host baseline: N = 1 only
            line["cpu_baseline"] = cpu_baseline(arena, upd_off, doc_upd, fmt, args.cpu_baseline_seconds)
        if not args.no_secondary and world == 1 and not stub:
            line["secondary"] = secondary(dev, eng)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
