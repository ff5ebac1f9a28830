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
