"""Summarises a rocprofv3 run (kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE PMC passes) into
profiles/<tag>_summary.json and profiles/pmc_<workload>.json (read by bench.py as roofline.traffic).

HBM bytes per launch of the fast-path kernel follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads
half the bytes of wide coalesced streams on gfx950, so read bytes = 2 * FETCH_SIZE * 1024;
WRITE_SIZE (KB) * 1024 is exact for 16-B-per-lane streaming stores.
Usage: python tools/summarize_prof.py <gpurun_out dir> <tag> <workload> <kt dir> <fetch dir> <write dir> [pmc dir]"""
import csv
import glob
import json
import os
import sys

src, tag, wl, kt, fetch, write = sys.argv[1:7]
pmc_sq = sys.argv[7] if len(sys.argv) > 7 else None
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_fast_merge_v1"


def rows(d, suffix):
    f = glob.glob(os.path.join(src, d, "*" + suffix))
    return list(csv.DictReader(open(f[0]))) if f else []


stats = rows(kt, "_kernel_stats.csv")
out = {"kernels": [{"name": r["Name"][:160], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                    "pct": float(r["Percentage"])} for r in stats]}


def counter(d, name):
    vals = [float(r["Counter_Value"]) for r in rows(d, "_counter_collection.csv")
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == name]
    return sum(vals) / len(vals) if vals else None


fk = counter(fetch, "FETCH_SIZE")
wk = counter(write, "WRITE_SIZE")
out["fast_kernel"] = {"FETCH_SIZE_KB": fk, "WRITE_SIZE_KB": wk}
if pmc_sq:
    for c in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
              "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        out["fast_kernel"][c] = counter(pmc_sq, c)
hbm = None
if fk is not None and wk is not None:
    hbm = int(2 * fk * 1024 + wk * 1024)
    out["fast_kernel"]["hbm_bytes_per_launch"] = hbm
os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "profiles", f"{tag}_summary.json"), "w"), indent=1)
if hbm is not None:
    json.dump({"hbm_bytes_per_launch": hbm, "source": f"profiles/{tag}_summary.json"},
              open(os.path.join(ROOT, "profiles", f"pmc_{wl}.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
