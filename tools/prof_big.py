"""Runs a secondary workload of bench.py on cuda:0 a few times (device-resident): the workload profiled by
rocprofv3 for the diff / state-vector kernels (k_big_v1 / k_big_v2).  CASE = a bench.py secondary case
name (diff_c3_v1, diff_c3_v2, sv_c3_v1, diff_c5_v1, diff_c5_v2, ...).
Usage: CASE=diff_c3_v2 rocprofv3 ... -- python tools/prof_big.py [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["YM_SECONDARY"] = os.environ.get("CASE", "diff_c3_v2")
import torch  # noqa: E402

import bench  # noqa: E402
from yjs_amd import Engine  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
res = bench.secondary(dev, Engine(0))
print(res)
