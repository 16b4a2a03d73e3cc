"""Times the C restatement (oracle/ymerge_oracle.c, the bench's cpu_baseline "port") on the same documents
as oracle/gen/time_js_baselines.cjs (the first N documents of a workload's templates, cycled), with 1 and
with all threads of this host, for the 13.4.9 / 13.5.16 / C-port calibration in BASELINE.md §2.
Usage: python tools/time_cpu_port.py c2_v1 2000"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import oracle_ref  # noqa: E402
from yjs_amd.workloads import load_ymb, replicate  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c2_v1"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
a, o, d = replicate(*load_ymb(wl), n)
res = {"workload": wl, "docs": n, "input_bytes": int(o[-1])}
for th in (1, os.cpu_count()):
    oracle_ref.batch("merge", 1, a, o, d, nthreads=th, want_output=False)
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 3.0:
        oracle_ref.batch("merge", 1, a, o, d, nthreads=th, want_output=False)
        reps += 1
    el = (time.perf_counter() - t0) / reps
    res[f"c_port_{th}_threads"] = {"s": el, "input_gbs": int(o[-1]) / el / 1e9, "docs_per_s": n / el}
print(json.dumps(res))
