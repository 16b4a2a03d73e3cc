"""Pins the CPU restatement (oracle/) against the golden vectors produced by yjs 13.5.16 itself
(tests/golden/*.json; recipe oracle/gen/make_fixtures.cjs), including the reference's own three V1
compatibility vectors (gaberogan/yjs tests/compatibility.tests.js:16-46) and the error cases."""
import pytest

import golden_io
import oracle_ref as O

CASES = golden_io.load_cases()


def run_case(c):
    if c["op"] == "merge":
        return O.merge(c["inputs"], c["fmt"])
    if c["op"] == "diff":
        return O.diff(c["inputs"][0], c["sv"], c["fmt"])
    if c["op"] == "conv":
        return O.convert(c["inputs"][0], c["fmt"])
    if c["op"] == "meta":
        return O.meta(c["inputs"][0], c["fmt"])
    if c["op"] == "dsmerge":
        return O.ds_merge(c["inputs"], c["fmt"])
    if c["op"] == "dsmerge_ref":
        return O.ds_merge(c["inputs"], c["fmt"] | 0x100)
    if c["op"] in ("snap_to_v1", "snap_to_v2"):
        return O.snapshot(c["inputs"][0], c["fmt"], 2 if c["op"] == "snap_to_v2" else 1)
    return O.sv_from_update(c["inputs"][0], c["fmt"])


@pytest.mark.parametrize("case", CASES, ids=[c["id"] for c in CASES])
def test_oracle_matches_golden(case):
    st, out = run_case(case)
    if "error" in case:
        assert st == O.js_error_status(case["error"], case["message"]), (st, case["error"], case["message"])
    else:
        assert st == 0, O.STATUS_NAMES.get(st)
        assert out == case["expect"]


def test_golden_coverage():
    groups = {c["group"] for c in CASES}
    assert {"c1_text", "c2_text", "c4_map", "c5_xml", "content", "edge", "refgolden", "conv", "meta", "dsmerge"} <= groups
    for op in ("merge", "diff", "sv", "conv", "meta", "dsmerge", "snap_to_v1", "snap_to_v2"):
        for fmt in (1, 2):
            assert any(c["op"] == op and c["fmt"] == fmt and "expect" in c for c in CASES), (op, fmt)
    assert sum("error" in c for c in CASES) >= 20


def test_oracle_batch_matches_single():
    import numpy as np
    cs = [c for c in CASES if c["group"] == "c2_text" and c["op"] == "merge" and c["fmt"] == 1][:16]
    blobs, upd_off, doc_upd = [], [0], [0]
    for c in cs:
        for u in c["inputs"]:
            blobs.append(u)
            upd_off.append(upd_off[-1] + len(u))
        doc_upd.append(doc_upd[-1] + len(c["inputs"]))
    arena = np.frombuffer(b"".join(blobs), np.uint8)
    outs, status, _ = O.batch("merge", 1, arena, np.array(upd_off, np.uint64), np.array(doc_upd, np.uint32), nthreads=4)
    assert (status == 0).all()
    assert outs == [c["expect"] for c in cs]
