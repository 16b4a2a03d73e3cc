"""Timeline of the last call(s) in a rocprofv3 --kernel-trace --memory-copy-trace directory: every kernel and
copy with start / end relative to the first event of the window, its stream and duration (us).
Usage: python tools/call_timeline2.py <dir> [window_us]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
win = float(sys.argv[2]) if len(sys.argv) > 2 else 1500.0
ev = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K s%s" % r["Stream_Id"], r["Kernel_Name"][:70]))
for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C s%s" % r["Stream_Id"], r["Direction"].replace("MEMORY_COPY_", "")))
ev.sort()
end = ev[-1][1]
sel = [e for e in ev if e[0] >= end - win * 1000]
t0 = sel[0][0]
for s, e, k, n in sel:
    print("%9.1f %9.1f %8.1f  %-6s %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, k, n))
