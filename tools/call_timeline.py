"""The kernels of the last `ncalls` engine calls in a rocprofv3 kernel trace (run_kernel_trace.csv), in
order, with start offsets and gaps: where one call's time goes.  Usage: python tools/call_timeline.py <trace.csv>
[kernels per call] [calls]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = rows[-k:]
t0 = int(rows[0]["Start_Timestamp"])
prev = t0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.1f} us  gap {(s - prev) / 1e3:7.1f}  dur {(e - s) / 1e3:8.1f}  {r['Kernel_Name'][:100]}")
    prev = e
print(f"span {(prev - t0) / 1e3:.1f} us")
