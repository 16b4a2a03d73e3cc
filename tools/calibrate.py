"""Measures the CPU-baseline calibration the bench reports: per-thread throughput of the
JavaScript implementations (yjs 13.5.16 mergeUpdates, the byte target; gaberogan/yjs@v0's own Doc round
trip) and of the C port (oracle/ymerge_oracle.c, the bench's cpu_baseline) on the same documents, and their
ratios.  Container-only (the JS needs /root/reference and the offline bundle); writes
profiles/calibration.json, which bench.py reads -- so the ratios come from a run of this script, not from
constants.  Usage: python tools/calibrate.py [docs]"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
res = {"docs": n, "measured_utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()), "threads": 1, "workloads": {}}
for wl in ("c2_v1", "c4_v1"):
    js = json.loads(subprocess.check_output(["node", os.path.join(ROOT, "oracle/gen/time_js_baselines.cjs"), wl, str(n)],
                                            cwd=os.path.join(ROOT, "oracle/gen")).decode().strip().splitlines()[-1])
    port = json.loads(subprocess.check_output([sys.executable, os.path.join(ROOT, "tools/time_cpu_port.py"), wl, str(n)],
                                              cwd=ROOT).decode().strip().splitlines()[-1])
    c1 = port["c_port_1_threads"]["input_gbs"]
    res["workloads"][wl] = {
        "c_port_gbs_1_thread": c1,
        "yjs_13_5_16_js_gbs_1_thread": js["yjs_13_5_16_mergeUpdates"]["input_gbs"],
        "reference_13_4_9_doc_roundtrip_gbs_1_thread": js["reference_13_4_9_doc_roundtrip_gc_false"]["input_gbs"],
        "port_over_yjs_13_5_16_js": round(c1 / js["yjs_13_5_16_mergeUpdates"]["input_gbs"], 3),
        "port_over_reference_13_4_9_doc_roundtrip": round(c1 / js["reference_13_4_9_doc_roundtrip_gc_false"]["input_gbs"], 3),
        "node": js["node"],
    }
    print(wl, res["workloads"][wl], flush=True)
with open(os.path.join(ROOT, "profiles", "calibration.json"), "w") as f:
    json.dump(res, f, indent=1)
