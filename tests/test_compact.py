"""Doc round-trip compaction: the oracle's C restatement of yjs 13.4.9's Doc engine
(oracle/ymerge_oracle.c ymo_compact) pinned against the reference's own outputs for every fixture
(tests/golden/compact.json: golden merge inputs, workload documents C1-C5, randomized formatted-text
histories)."""
import collections

import pytest

import compact_cases
import oracle_ref as O


@pytest.mark.parametrize("group", sorted({c["group"] for c in compact_cases.load()}))
def test_oracle_compact_matches_reference(group):
    cases = [c for c in compact_cases.load() if c["group"] == group]
    bad = []
    for c in cases:
        st, out = O.compact(c["inputs"], c["fmt"])
        why = compact_cases.mismatch(c, st, out, message=False)
        if why:
            bad.append((c["id"], why))
    assert not bad, f"{len(bad)}/{len(cases)} differ: {bad[:8]}"


def test_compact_fixture_coverage():
    cs = compact_cases.load()
    n = collections.Counter(c["group"] for c in cs)
    assert n["fuzz_fmt"] >= 150 and n["wl_c5"] >= 8 and n["canon"] >= 300
    # the carve-outs are pinned: histories the reference leaves pending (gapped workload documents, lost /
    # late messages) and inputs on which it throws
    assert n["gap_c2"] >= 48 and n["gap_c5"] >= 4 and n["fuzz_gap"] >= 150
    assert sum(1 for c in cs if c["pending"]) >= 200
    assert sum(1 for c in cs if c["error"]) >= 75


def test_compact_keeps_the_state_vector():
    """The compacted document covers exactly the inputs' clocks: its state vector equals the one of
    mergeUpdates(inputs) (compaction garbage-collects content, never structs)."""
    for c in compact_cases.load():
        if c["group"] not in ("fuzz_fmt", "c5_xml", "c2_text", "canon"):
            continue
        st, out = O.compact(c["inputs"], c["fmt"])
        st2, merged = O.merge(c["inputs"], c["fmt"])
        assert st == 0 and st2 == 0, c["id"]
        assert O.sv_from_update(out, c["fmt"]) == O.sv_from_update(merged, c["fmt"]), c["id"]


def test_compact_nogc_fixture_coverage():
    """gc: false fixtures (the same inputs on new Y.Doc({ gc: false })): most documents with deletions keep
    their deleted content, so their bytes differ from the gc: true ones."""
    cs = compact_cases.load(nogc=True)
    assert len(cs) >= 1000
    assert sum(1 for c in cs if c["differs"]) >= 500
    assert sum(1 for c in cs if c["pending"]) >= 100 and sum(1 for c in cs if c["error"]) >= 5


@pytest.mark.parametrize("san", [False, True], ids=["opt", "asan_ubsan"])
def test_device_core_compact_nogc_host_build(san):
    """YM_NO_GC (new Y.Doc({ gc: false })): the device code built for the host against every gc: false
    fixture of the reference (the oracle's C restatement models gc: true only; these are pinned by the
    reference's bytes)."""
    import core_host
    from yjs_amd import pack_docs
    for fmt in (1, 2):
        cs = [c for c in compact_cases.load(nogc=True) if c["fmt"] == fmt]
        if san:
            seen = collections.Counter()
            cs = [c for c in cs if seen.update([c["group"]]) is None and seen[c["group"]] <= 12]
        a, o, d = pack_docs([c["inputs"] for c in cs])
        outs, st = core_host.run("compact_nogc", fmt, a, o, d, san=san)
        bad = [(c["id"], why) for c, out, s in zip(cs, outs, st) if (why := compact_cases.mismatch(c, s, out))]
        assert not bad, f"{len(bad)}/{len(cs)} differ: {bad[:8]}"


@pytest.mark.parametrize("san", [False, True], ids=["opt", "asan_ubsan"])
def test_device_core_compact_host_build(san):
    """The device code itself (yjs_amd/csrc/ym_compact.h compact_doc, what k_compact runs one document per
    lane) built for the host (tests/native/core_host.cpp op 7), optimised and under ASan + UBSan, against
    every fixture of the reference."""
    import core_host
    from yjs_amd import pack_docs
    for fmt in (1, 2):
        cs = [c for c in compact_cases.load() if c["fmt"] == fmt]
        if san:  # the sanitizer build on a subset: every group's first cases
            seen = collections.Counter()
            cs = [c for c in cs if seen.update([c["group"]]) is None and seen[c["group"]] <= 12]
        a, o, d = pack_docs([c["inputs"] for c in cs])
        outs, st = core_host.run("compact", fmt, a, o, d, san=san)
        bad = [(c["id"], why) for c, out, s in zip(cs, outs, st) if (why := compact_cases.mismatch(c, s, out))]
        assert not bad, f"{len(bad)}/{len(cs)} differ: {bad[:8]}"


def test_compact_sv_fixture_coverage():
    """encodeStateAsUpdate(doc, sv) fixtures: every target kind, gc: false documents, the slice group's every
    clock (a surrogate pair cut by str.slice: V1 throws URIError), malformed vectors."""
    cs = compact_cases.load_sv()
    n = collections.Counter(c["kind"] for c in cs)
    assert all(n[k] >= 900 for k in ("empty", "full", "prefix", "repeat", "past")) and n["random"] >= 1800
    assert n["clock"] >= 300 and n["zero_length"] >= 10 and n["truncated"] >= 10
    assert sum(1 for c in cs if not c["gc"]) >= 1000
    err = collections.Counter(c["error"]["name"] for c in cs if c["error"])
    assert err["URIError"] >= 20 and sum(err.values()) >= 60
    # a target with the document's own state vector receives no structs, only the delete set
    assert all(c["error"] is None for c in cs if c["kind"] == "full")


@pytest.mark.parametrize("san", [False, True], ids=["opt", "asan_ubsan"])
def test_device_core_compact_target_sv_host_build(san):
    """ym_compact with target state vectors (encodeStateAsUpdate[V2](doc, sv)): the device code built for the
    host against every target fixture of the reference (gc: true and false documents)."""
    import core_host
    from yjs_amd import pack_docs
    for fmt in (1, 2):
        for gc in (True, False):
            cs = [c for c in compact_cases.load_sv() if c["fmt"] == fmt and c["gc"] == gc]
            if san:
                seen = collections.Counter()
                cs = [c for c in cs if seen.update([c["group"] + c["kind"]]) is None and seen[c["group"] + c["kind"]] <= 6]
            a, o, d = pack_docs([c["inputs"] for c in cs])
            sa, so, _ = pack_docs([[c["sv"]] for c in cs])
            outs, st = core_host.run("compact" if gc else "compact_nogc", fmt, a, o, d, sa, so, san=san)
            bad = [(c["id"], why) for c, out, s in zip(cs, outs, st) if (why := compact_cases.mismatch(c, s, out))]
            assert not bad, f"fmt {fmt} gc {gc}: {len(bad)}/{len(cs)} differ: {bad[:8]}"


@pytest.mark.parametrize("san", [False, True], ids=["opt", "asan_ubsan"])
def test_device_core_compact_doc_state_vector_host_build(san):
    """YM_SV_FIRST: encodeStateVector(doc) of the compacted Doc (clients in StructStore insertion order, not the
    descending order of the update) then the update, against the reference's own bytes (the `sv` of
    compact.json / compact_nogc.json), through the host build of the device core."""
    import core_host
    from yjs_amd import pack_docs
    for nogc in (False, True):
        for fmt in (1, 2):
            cs = [c for c in compact_cases.load(nogc=nogc) if c["fmt"] == fmt and c["expect"] is not None or
                  (c["fmt"] == fmt and c["error"])]
            if san:
                cs = cs[::4]
            a, o, d = pack_docs([c["inputs"] for c in cs])
            outs, st = core_host.run("compact_nogc_sv" if nogc else "compact_sv", fmt, a, o, d, san=san)
            bad = [(c["id"], w) for c, s_, g in zip(cs, st, outs) if (w := compact_cases.mismatch_sv_first(c, s_, g))]
            assert not bad, f"{len(bad)}/{len(cs)}: {bad[:5]}"
