"""CPU: the C-ABI library loads and exports exactly what include/tmhip.h declares."""
import ctypes as C
import os
import re

import pytest

from util import REPO
from tmlibrary_amd import hip

HEADER = os.path.join(REPO, "include", "tmhip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(tmh_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_functions():
    names = declared_functions()
    assert "tmh_stats_update" in names and "tmh_correct_u16" in names
    assert len(names) >= 30


def test_bindings_cover_header():
    assert sorted(hip.SIGNATURES) == declared_functions()


def test_library_exports_every_symbol():
    lib = hip.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.tmh_abi_version() == hip.ABI_VERSION


def test_errors_without_gpu_are_loud():
    """No CPU fallback: without a device, lib() raises instead of degrading."""
    lib = hip.load_library()
    n = C.c_int(-1)
    rc = lib.tmh_device_count(C.byref(n))
    if rc == 0 and n.value > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(hip.HipUnavailableError):
        hip.lib()


def test_null_arguments_are_rejected():
    lib = hip.load_library()
    assert lib.tmh_device_count(None) == hip.TMH_EINVAL
    assert b"NULL" in lib.tmh_last_error()
