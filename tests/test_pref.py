"""P-ref: the bytes the engine must produce (yjs 13.5.16's, tests/golden) agree with
gaberogan/yjs@v0 itself.  tests/pref/pref.json was computed in the survey container by running the
reference's own src/ (oracle/gen/make_pref_fixtures.cjs via ref_yjs.cjs): for every golden merge, the
reference's Doc round trip of the merged bytes has the same structs as the inputs applied one by one
(P-ref-1), the same delete-set coverage as mergeDeleteSets of the inputs (P-ref-2) and no pending structs
(P-ref-3); every golden state vector equals the reference's encodeStateVector of the Doc the update builds;
every golden diff carries, unit for unit, the structs of the reference's encodeStateAsUpdate(Doc(u), sv)
and keeps the input's delete set, which the reference's own delete set contains (P-ref-diff).
Here: the verdicts hold, they were computed on exactly the golden bytes, and the oracle produces them;
tests/test_gpu_golden.py::test_pref_bytes_on_gpu checks the engine produces them on the MI355X."""
import base64
import hashlib
import json
import os

import pytest

import golden_io
import oracle_ref as O

PREF = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "pref", "pref.json")))
GOLD = {c["id"]: c for c in golden_io.load_cases()}


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_pref_verdicts_hold():
    app = [c for c in PREF["cases"] if c.get("applicable")]
    merges = [c for c in app if c["op"] == "merge"]
    svs = [c for c in app if c["op"] == "sv"]
    diffs = [c for c in app if c["op"] == "diff"]
    assert len(merges) >= 800 and len(svs) >= 140 and len(diffs) >= 600
    bad = [c["id"] for c in merges if not (c["pref1"] and c["pref2"] and c["pref3"])]
    bad += [c["id"] for c in svs if not c["pref_sv"]]
    bad += [c["id"] for c in diffs if not (c["pref_diff"] and c["pref_diff_ds"] and c["pref_diff_ds_in_ref"])]
    assert not bad, bad[:10]
    # every case the reference cannot evaluate carries its reason
    assert all(c.get("reason") for c in PREF["cases"] if not c.get("applicable"))


def test_pref_checked_the_golden_bytes():
    for c in PREF["cases"]:
        g = GOLD[c["id"]]
        assert sha(g["expect"]) == c["checked_sha256"], c["id"]


@pytest.mark.parametrize("op", ["merge", "sv", "diff"])
def test_oracle_produces_the_pref_bytes(op):
    for c in PREF["cases"]:
        if c["op"] != op or not c.get("applicable"):
            continue
        g = GOLD[c["id"]]
        if op == "merge":
            st, out = O.merge(g["inputs"], g["fmt"])
        elif op == "diff":
            st, out = O.diff(g["inputs"][0], g["sv"], g["fmt"])
        else:
            st, out = O.sv_from_update(g["inputs"][0], g["fmt"])
        assert st == 0 and sha(out) == c["checked_sha256"], c["id"]
