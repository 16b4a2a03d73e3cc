"""Timeline of the last pipelined host call in a rocprofv3 kernel trace of tools/host_pipe_prof.py: each
kernel's start / end relative to the call's first copy kernel, its queue and name.
Usage: python tools/pipe_timeline.py <run_kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_h2d_copy" in r["Kernel_Name"]]
first = idx[-3]  # the last call's first copy kernel (three chunks per C2 call)
t0 = int(rows[first]["Start_Timestamp"])
for r in rows[first - 1:first + 14]:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{s:8.1f} {e:8.1f} {e - s:7.1f} q{r['Queue_Id']} grid {r['Grid_Size_X']:>7} {r['Kernel_Name'][:70]}")
