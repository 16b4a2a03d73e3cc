"""Average duration of the headline kernel's timed launches in a rocprofv3 kernel trace of
`bench.py --no-secondary --no-cpu-baseline` (default 50 steps): the STEPS full-grid launches right before the
last run of launches of another grid (the host-path measurement after the timed region; bench.py also measures
that path first, before the device-resident steps).
Usage: python tools/timed_stats.py <run_kernel_trace.csv> [steps]"""
import csv
import statistics
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
rows = sorted((r for r in csv.DictReader(open(path)) if "k_fast_merge_v1<0, 8" in r["Kernel_Name"]),
              key=lambda r: int(r["Start_Timestamp"]))
full = max(int(r["Grid_Size_X"]) for r in rows)  # the whole batch in one launch
# the longest run of whole-batch launches is the device-resident phase (verification, warmup, timed steps);
# its last STEPS launches are the timed ones
best, run0 = (0, 0), None
for i, r in enumerate(rows + [None]):
    if r is not None and int(r["Grid_Size_X"]) == full:
        run0 = i if run0 is None else run0
    elif run0 is not None:
        best = max(best, (i - run0, i))
        run0 = None
k = best[1]
ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows[max(0, k - steps):k]]
print(f"k_fast_merge_v1 timed launches: n={len(ds)} avg={statistics.mean(ds):.2f} us median={statistics.median(ds):.2f} "
      f"min={min(ds):.2f} max={max(ds):.2f} (launches {max(0, k - steps)}..{k - 1} of {len(rows)}; grid {full})")
