"""Summarises one round's rocprofv3 runs into profiles/ (committed): the kernel-trace stats of the
bench command and the per-launch PMC counters of the fast-path merge kernel (tools/pmc_passes.sh),
plus profiles/pmc_<workload>.json with the HBM bytes per launch that bench.py reports as
roofline.traffic.  HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) counts half the bytes
of wide coalesced streaming reads on gfx950, so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE (KB)
* 1024 is the written bytes.
Usage: python tools/summarize_prof.py <kernel_stats.csv> <pmc dir> <tag> <workload>"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_fast_merge_v1"
stats_csv, pmc_dir, tag, wl = sys.argv[1:5]
rows = list(csv.DictReader(open(stats_csv)))
out = {"kernel_stats": [{"name": r["Name"][:160], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                         "pct": float(r["Percentage"])} for r in rows]}
acc = {}
for f in sorted(glob.glob(os.path.join(pmc_dir, "p*", "**", "*counter_collection.csv"), recursive=True)):
    per = {}
    for r in csv.DictReader(open(f)):
        if KERNEL not in r["Kernel_Name"]:
            continue
        key = (r["Counter_Name"], r.get("Dispatch_Id", ""))
        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    for (name, _), v in per.items():
        acc.setdefault(name, []).append(v)
pmc = {k: sum(v) / len(v) for k, v in sorted(acc.items())}
out["fast_kernel_pmc_per_launch"] = pmc
hbm = None
if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
    hbm = int(2 * pmc["FETCH_SIZE"] * 1024 + pmc["WRITE_SIZE"] * 1024)
    out["fast_kernel_hbm_bytes_per_launch"] = hbm
waves = pmc.get("SQ_WAVES")
if waves:
    out["per_document_wave"] = {k: round(pmc[k] / waves, 1) for k in
                                ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_WAVE_CYCLES",
                                 "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if k in pmc}
os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "profiles", f"{tag}_summary.json"), "w"), indent=1)
if hbm is not None:
    json.dump({"hbm_bytes_per_launch": hbm, "source": f"profiles/{tag}_summary.json"},
              open(os.path.join(ROOT, "profiles", f"pmc_{wl}.json"), "w"), indent=1)
print(json.dumps(out, indent=1)[:3000])
