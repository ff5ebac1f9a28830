"""C-ABI boundary checks that need no GPU: the library loads, exports every entry point that
include/eikonal.h declares, and fails loudly (no CPU fallback) when no device is visible."""
import ctypes
import os
import re

import pytest

import eikonal
from eikonal import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(eik_\w+)\s*\(", src)))


def test_header_symbols_exported():
    lib = ctypes.CDLL(L.LIB_PATH)
    names = declared("eikonal.h")
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(L.EXPORTED) == names  # the ctypes binding covers the whole ABI


def test_version_string():
    assert b"gfx950" in eikonal.lib().eik_version()


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="GPU visible")
def test_no_device_fails_loudly():
    with pytest.raises(eikonal.EikError) as e:
        eikonal.Context(0)
    assert e.value.code == L.EIK_ERR_NODEVICE


def test_solver_options_parse():
    """Context(options=...) input handling (no GPU needed): names of the OPT_* constants, unknown
    names rejected with the list of known ones; nothing is taken from the environment."""
    from eikonal import _lib as L

    assert L.parse_options(None) == {} and L.parse_options("") == {}
    assert L.parse_options("PASSES=16, SCHED=1") == {"PASSES": 16.0, "SCHED": 1.0}
    assert L.parse_options({"PASSES": 8}) == {"PASSES": 8.0}
    for bad in ("PASES=16", "PASSES", {"NOPE": 1}):
        with pytest.raises(ValueError):
            L.parse_options(bad)
