"""CPU: libmaxcover loads and exports every entry point include/maxcover.h declares; error
paths that need no GPU behave as documented. No compute calls here."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "maxcover.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mac_\w+)\s*\(", src)))


def test_every_declared_symbol_is_exported(pkg):
    L = pkg.load_library()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), f"{s} declared in maxcover.h but not exported"
    assert set(syms) == set(pkg._lib.EXPORTS)


def test_library_is_gfx950_code_object(pkg):
    data = open(pkg._lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_version(pkg):
    assert pkg.version().startswith("maxcover ") and "gfx950" in pkg.version()


def test_null_and_option_errors_without_gpu(pkg):
    L = pkg.load_library()
    assert L.mac_set_option(None, 1, 0) == pkg._lib.MAC_E_INVAL
    assert "null" in L.mac_last_error().decode()
    n = ctypes.c_int64()
    assert L.mac_num_points(None, ctypes.byref(n)) == pkg._lib.MAC_E_INVAL
    L.mac_ctx_destroy(None)  # no-op


def test_ctx_create_without_device_fails_loudly(pkg):
    if pkg.device_count() > 0:
        pytest.skip("a GPU is visible here")
    with pytest.raises(pkg.MaxCoverError) as ei:
        pkg.Context(0)
    assert ei.value.code == pkg._lib.MAC_E_NODEVICE


def test_no_cpu_fallback_in_product(pkg):
    """The product package never imports the oracle."""
    pdir = os.path.dirname(pkg.__file__)
    for f in os.listdir(pdir):
        if f.endswith(".py"):
            txt = open(os.path.join(pdir, f)).read()
            assert "oracle" not in txt.replace("oracle/", ""), f
