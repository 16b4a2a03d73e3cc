"""Loader for the committed golden vectors (tests/golden/*.json, made by oracle/gen/make_fixtures.cjs)."""
import base64
import glob
import json
import os

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# fixture files with their own case layout and loader (compact*.json: tests/compact_cases.py)
OTHER_FORMATS = {"compact", "compact_nogc", "compact_sv"}


def load_cases(groups=None):
    out = []
    for f in sorted(glob.glob(os.path.join(GOLDEN_DIR, "*.json"))):
        g = os.path.splitext(os.path.basename(f))[0]
        if g in OTHER_FORMATS or (groups and g not in groups):
            continue
        with open(f) as fh:
            d = json.load(fh)
        for c in d["cases"]:
            c = dict(c)
            c["group"] = g
            c["inputs"] = [base64.b64decode(x) for x in c["inputs"]]
            if "sv" in c:
                c["sv"] = base64.b64decode(c["sv"])
            if "expect" in c:
                c["expect"] = base64.b64decode(c["expect"])
            c["id"] = f"{g}/{c['name']}/v{c['fmt']}/{c['op']}"
            out.append(c)
    return out
