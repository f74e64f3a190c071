"""ctypes wrapper for oracle/liboracle.so — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py)."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        p = ctypes.c_void_p
        i = ctypes.c_int
        L.oracle_loglik.restype = ctypes.c_double
        L.oracle_loglik.argtypes = [i, i, i, i, i, i] + [p] * 8
        L.oracle_loglik_batch.restype = None
        L.oracle_loglik_batch.argtypes = [i, i, i, i, i, i, i] + [p] * 9
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


def loglik_batch(obs, fam_of_site, zone_of_site, w, p_global, p_zones, p_fam=None,
                 source=None, inheritance=None):
    """Same contract as oracle.lik_numpy.loglik_batch, computed by the C restatement."""
    obs = np.ascontiguousarray(obs, dtype=np.int8)
    fam_of_site = np.ascontiguousarray(fam_of_site, dtype=np.uint8)
    zone_of_site = np.ascontiguousarray(zone_of_site, dtype=np.uint8)
    w = np.ascontiguousarray(w, dtype=np.float64)
    p_global = np.ascontiguousarray(p_global, dtype=np.float64)
    p_zones = np.ascontiguousarray(p_zones, dtype=np.float64)
    if inheritance is None:
        inheritance = w.shape[-1] == 3
    if p_fam is not None:
        p_fam = np.ascontiguousarray(p_fam, dtype=np.float64)
    if source is not None:
        source = np.ascontiguousarray(source, dtype=np.uint8)
    B, N = zone_of_site.shape
    F, S = p_global.shape[1:]
    Z = p_zones.shape[1]
    Fam = 0 if p_fam is None else p_fam.shape[1]
    out = np.empty(B)
    lib().oracle_loglik_batch(B, N, F, S, Z, Fam, int(bool(inheritance)), _ptr(obs),
                              _ptr(fam_of_site), _ptr(zone_of_site), _ptr(w), _ptr(p_global),
                              _ptr(p_zones), _ptr(p_fam), _ptr(source), _ptr(out))
    return out
