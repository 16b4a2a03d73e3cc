"""Prints the rocprofv3 kernel averages collected by tools/ab.sh: <dir>/<lib>/<workload>/**/*kernel_stats.csv,
the ten largest kernels by total time per (library, workload).  Usage: python tools/ab_summary.py <dir>"""
import csv
import glob
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*", "*", "**", "*kernel_stats.csv"), recursive=True)):
    rel = os.path.relpath(f, d).split(os.sep)
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:10]:
        name = r["Name"].split("(")[0][-70:]
        print(f"{rel[0]:>18} {rel[1]:>8} {float(r['AverageNs']) / 1e3:10.2f} us x{int(r['Calls']):4d}  {name}")
