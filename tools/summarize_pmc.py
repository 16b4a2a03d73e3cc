"""Per-launch averages of every PMC counter collected for the fast-path merge kernel under a
directory of rocprofv3 --pmc passes (tools/pmc_passes.sh).  Usage: python tools/summarize_pmc.py <dir>"""
import csv
import glob
import os
import sys

KERNEL = os.environ.get("KERNEL", "k_fast_merge_v1")
acc = {}
for f in sorted(glob.glob(os.path.join(sys.argv[1], "p*", "**", "*counter_collection.csv"), recursive=True)):
    per = {}
    for r in csv.DictReader(open(f)):
        if KERNEL not in r["Kernel_Name"]:
            continue
        key = (r["Counter_Name"], r.get("Dispatch_Id", ""))
        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    for (name, _), v in per.items():
        acc.setdefault(name, []).append(v)
for name in sorted(acc):
    vals = acc[name]
    print(f"{name:28s} {sum(vals) / len(vals):16.1f}   (n={len(vals)})")
