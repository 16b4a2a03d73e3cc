"""Per-phase instruction deltas (per document wave) from tools/pmc_stops.sh output (ablation stops in
execution order).  Usage: python tools/stops_table.py gpurun_out/<tag>/stops.txt"""
import re
import sys

s = open(sys.argv[1]).read()
blocks = re.split(r"== stop (\d+)", s)
order, data = [], {}
for i in range(1, len(blocks), 2):
    d = {}
    for line in blocks[i + 1].splitlines():
        m = re.match(r"(\S+)\s+([\d.]+)", line)
        if m:
            d[m.group(1)] = float(m.group(2))
    waves = d.get("SQ_WAVES", 1.0) or 1.0
    data[blocks[i]] = {k: v / waves for k, v in d.items()}
    order.append(blocks[i])
keys = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY"]
names = {"1": "stage", "8": "W1 struct walk", "2": "W2 delete-set walk", "3": "section sort", "4": "layout",
         "7": "struct emit", "5": "delete set", "0": "delete-set emit"}
print(f"{'phase':20s} " + " ".join(f"{k[3:]:>12s}" for k in keys) + "   sum(insts)")
prev = {k: 0.0 for k in keys}
for st in order:
    d = data[st]
    row = [d.get(k, 0.0) - prev[k] for k in keys]
    print(f"{names.get(st, st):20s} " + " ".join(f"{v:12.0f}" for v in row) + f"   {sum(row[:5]):8.0f}")
    prev = {k: d.get(k, 0.0) for k in keys}
