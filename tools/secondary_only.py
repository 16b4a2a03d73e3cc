"""A subset of bench.py's secondary lines (YM_SECONDARY=name,name,...), one JSON object per line.
Usage: YM_SECONDARY=merge_c2u_v1,merge_c2_v2 python tools/secondary_only.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from yjs_amd import Engine  # noqa: E402

dev = torch.device("cuda", 0)
eng = Engine(0)
for k, v in bench.secondary(dev, eng).items():
    print(json.dumps({k: v}), flush=True)
