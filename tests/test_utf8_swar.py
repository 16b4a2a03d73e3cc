"""The SWAR strict UTF-8 validator / UTF-16 length of the device parsers (yjs_amd/csrc/ym_utf8.h) built for the
host and checked against a byte-wise decoder with lib0's rules (tests/native/utf8_test.cpp: every 1-3 byte input
at several alignments, random 4-byte inputs, random texts with corruptions and arbitrary slices)."""
import os
import subprocess

NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


def test_utf8_swar_matches_bytewise_decoder():
    subprocess.check_call(["make", "-s", "-C", NATIVE, "_build/utf8_test"])
    out = subprocess.run([os.path.join(NATIVE, "_build", "utf8_test")], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok ")
