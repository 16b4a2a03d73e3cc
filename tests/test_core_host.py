"""The device core's general path (ym_core.h general_doc, the code k_general runs one thread per document)
compiled for the host and checked on the CPU against every golden vector of yjs 13.5.16, once optimised
and once under AddressSanitizer + UndefinedBehaviorSanitizer.  GPU-free, so the exact
semantics of the device code are tested in this container; tests/test_gpu_golden.py runs the same
vectors through libymerge.so on the MI355X."""
import collections

import numpy as np
import pytest

import core_host
import golden_io
import oracle_ref as O
from yjs_amd.engine import pack_docs

CASES = [c for c in golden_io.load_cases() if not (c["op"] == "merge" and len(c["inputs"]) == 0)]


def _groups():
    g = collections.defaultdict(list)
    for c in CASES:
        g[(c["op"], c["fmt"])].append(c)
    return g


def run_cases(cases, op, fmt, san):
    if op in ("merge", "dsmerge", "dsmerge_ref"):
        a, o, d = pack_docs([c["inputs"] for c in cases])
        return core_host.run(op, fmt, a, o, d, san=san)
    a, o, d = pack_docs([[c["inputs"][0]] for c in cases])
    if op == "diff":
        sa, so, _ = pack_docs([[c["sv"]] for c in cases])
        return core_host.run(op, fmt, a, o, d, sa, so, san=san)
    return core_host.run(op, fmt, a, o, d, san=san)


def check(cases, outs, st):
    bad = []
    for i, c in enumerate(cases):
        if "error" in c:
            why = O.js_error_mismatch(st[i], c["error"], c["message"])
            if why:
                bad.append((c["id"], "error", why))
        elif st[i] != 0 or outs[i] != c["expect"]:
            bad.append((c["id"], "bytes", int(st[i])))
    return bad


@pytest.mark.parametrize("san", [False, True], ids=["opt", "asan_ubsan"])
@pytest.mark.parametrize("key", sorted(_groups().keys()), ids=lambda k: f"{k[0]}-v{k[1]}")
def test_core_general_path_golden(key, san):
    cases = _groups()[key]
    outs, st = run_cases(cases, key[0], key[1], san)
    bad = check(cases, outs, st)
    assert not bad, bad[:20]
