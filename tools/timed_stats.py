"""Average duration of the headline kernel's timed launches in a rocprofv3 kernel trace of
`bench.py --no-secondary --no-cpu-baseline` (default 50 steps): the STEPS full-grid launches right before the
first launch of another grid (the host-path measurement that follows the timed region).
Usage: python tools/timed_stats.py <run_kernel_trace.csv> [steps]"""
import csv
import statistics
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
rows = [r for r in csv.DictReader(open(path)) if "k_fast_merge_v1<0, 8" in r["Kernel_Name"]]
full = int(rows[0]["Grid_Size_X"])
k = next((i for i, r in enumerate(rows) if int(r["Grid_Size_X"]) != full), len(rows))
ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows[max(0, k - steps):k]]
print(f"k_fast_merge_v1 timed launches: n={len(ds)} avg={statistics.mean(ds):.2f} us median={statistics.median(ds):.2f} "
      f"min={min(ds):.2f} max={max(ds):.2f} (launches {max(0, k - steps)}..{k - 1} of {len(rows)}; grid {full})")
