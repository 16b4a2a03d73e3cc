"""The library's own device-wide prefix sums and flagged selection (yjs_amd/csrc/ym_scan.hip, in place of the
hipcub primitives): u32 and u64 exclusive scans, a device-side element count, and stable selection, against a
host computation at sizes inside one tile, at tile boundaries and over many tiles (ym__scan_check)."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 2, 2047, 2048, 2049, 4096, 100003, 5000000])
def test_scan_and_select(n):
    from yjs_amd import Engine
    e = Engine(0)
    e.lib.ym__scan_check.restype = __import__("ctypes").c_int
    assert e.lib.ym__scan_check(n, 7) == 0
