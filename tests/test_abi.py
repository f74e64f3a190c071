"""The C-ABI library loads and exports every symbol include/sbz.h declares (CPU-only: no compute)."""
import ctypes
import os
import re

from conftest import ROOT
from contact_zones_amd import _lib

HEADER = os.path.join(ROOT, "include", "sbz.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sbz_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_abi():
    names = declared_functions()
    for required in ("sbz_open", "sbz_close", "sbz_last_error", "sbz_loglik_batch",
                     "sbz_loglik_batch_device"):
        assert required in names


def test_library_exports_every_declared_symbol():
    L = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, f"libsbz.so lacks {missing}"


def test_python_binding_covers_the_header():
    assert set(declared_functions()) == set(_lib.SIGNATURES)


def test_version_and_device_count_without_gpu():
    L = _lib.lib()
    assert L.sbz_version().decode().startswith("sbz ")
    assert L.sbz_device_count() >= 0


def test_open_rejects_bad_dims():
    L = _lib.lib()
    ctx = ctypes.c_void_p()
    d = _lib.sbz_dims(0, 5, 3, 1, 0, 0)
    assert L.sbz_open(0, ctypes.byref(d), None, None, ctypes.byref(ctx)) == -1
    d = _lib.sbz_dims(4, 5, 200, 1, 0, 0)
    assert L.sbz_open(0, ctypes.byref(d), None, None, ctypes.byref(ctx)) == -1


def test_lds_budget_query():
    L = _lib.lib()
    # cfg5 (Z=8, Fam=4, S=10): table fits; an absurd class count does not
    d = _lib.sbz_dims(2000, 500, 10, 8, 4, _lib.SBZ_INHERITANCE)
    assert 0 < L.sbz_lik_lds_bytes(ctypes.byref(d), 0) <= 160 * 1024
    d = _lib.sbz_dims(2000, 500, 100, 50, 40, _lib.SBZ_INHERITANCE)
    assert L.sbz_lik_lds_bytes(ctypes.byref(d), 0) == 0
