"""ctypes binding of the in-tree HIP library contact_zones_amd/libsbz.so (include/sbz.h).

There is no CPU fallback: if the library is missing or fails to load, importing the
product path raises.  Build it with ``python -c "import __graft_entry__ as g; g.build()"``
(or ``make -C contact_zones_amd/csrc``).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SBZ_LIB_PATH") or os.path.join(_HERE, "libsbz.so")

SBZ_OK = 0
SBZ_INHERITANCE = 1
SBZ_SOURCE_BY_SITE = 0
SBZ_SOURCE_BY_POSITION = 1
# sbz_option (include/sbz.h): name -> id
OPTIONS = {"lik_tasks_per_cu": 1, "lik_banked": 2, "src_table": 3, "src_waves": 4, "src_hbm": 5,
           "src_stage": 6, "mh_lookahead": 7, "src_pass_tables": 8, "mh_group": 9, "src_pack": 10}
ERRORS = {-1: "SBZ_EINVAL", -2: "SBZ_EHIP", -3: "SBZ_ENOMEM", -4: "SBZ_ESTATE"}


class SbzError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class sbz_dims(ctypes.Structure):
    _fields_ = [("n_sites", ctypes.c_int32), ("n_features", ctypes.c_int32),
                ("n_states", ctypes.c_int32), ("n_zones", ctypes.c_int32),
                ("n_families", ctypes.c_int32), ("flags", ctypes.c_int32)]


_D = ctypes.c_double


class sbz_mh_config(ctypes.Structure):
    _fields_ = [("op_prob", ctypes.c_double * 16), ("precision", ctypes.c_double * 4),
                ("min_size", ctypes.c_int32), ("warmup", ctypes.c_int32),
                ("sample_source", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class sbz_chains(ctypes.Structure):
    """Device pointers of a sampler run (include/sbz.h)."""
    _fields_ = [("zone_of_site", ctypes.c_void_p), ("w", ctypes.c_void_p),
                ("p_global", ctypes.c_void_p), ("p_zones", ctypes.c_void_p),
                ("p_fam", ctypes.c_void_p), ("ll", ctypes.c_void_p),
                ("max_size", ctypes.c_void_p), ("p_grow_connected", ctypes.c_void_p),
                ("tape", ctypes.c_void_p), ("tape_stride", ctypes.c_int64),
                ("tape_len", ctypes.c_void_p), ("tape_pos", ctypes.c_void_p),
                ("seed", ctypes.c_uint64), ("chain_id0", ctypes.c_uint64),
                ("counter", ctypes.c_void_p), ("accepted", ctypes.c_void_p),
                ("proposed", ctypes.c_void_p), ("status", ctypes.c_void_p),
                ("trace_op", ctypes.c_void_p), ("trace_accept", ctypes.c_void_p),
                ("trace_ll", ctypes.c_void_p), ("trace_zos", ctypes.c_void_p),
                ("prior", ctypes.c_void_p), ("source", ctypes.c_void_p),
                ("alias_pending", ctypes.c_void_p), ("alias_p_global", ctypes.c_void_p),
                ("alias_p_zones", ctypes.c_void_p), ("alias_p_fam", ctypes.c_void_p),
                ("source_layout", ctypes.c_int32)]


class sbz_state(ctypes.Structure):
    """Host arrays of a host-form sampler run (sbz_mh_run, include/sbz.h)."""
    _fields_ = [("zone_of_site", ctypes.c_void_p), ("w", ctypes.c_void_p),
                ("p_global", ctypes.c_void_p), ("p_zones", ctypes.c_void_p),
                ("p_fam", ctypes.c_void_p), ("source", ctypes.c_void_p), ("ll", ctypes.c_void_p),
                ("prior", ctypes.c_void_p), ("max_size", ctypes.c_void_p),
                ("p_grow_connected", ctypes.c_void_p), ("chain_id0", ctypes.c_uint64),
                ("counter", ctypes.c_void_p), ("accepted", ctypes.c_void_p),
                ("proposed", ctypes.c_void_p), ("status", ctypes.c_void_p)]


class sbz_tape(ctypes.Structure):
    _fields_ = [("values", ctypes.c_void_p), ("stride", ctypes.c_int64), ("len", ctypes.c_void_p),
                ("pos", ctypes.c_void_p)]


class sbz_trace(ctypes.Structure):
    _fields_ = [("op", ctypes.c_void_p), ("accept", ctypes.c_void_p), ("ll", ctypes.c_void_p)]


# name -> (restype, argtypes); every symbol declared in include/sbz.h
_P = ctypes.c_void_p
_I = ctypes.c_int
SIGNATURES = {
    "sbz_version": (ctypes.c_char_p, []),
    "sbz_device_count": (_I, []),
    "sbz_open": (_I, [_I, ctypes.POINTER(sbz_dims), _P, _P, ctypes.POINTER(_P)]),
    "sbz_close": (None, [_P]),
    "sbz_last_error": (ctypes.c_char_p, [_P]),
    "sbz_set_stream": (_I, [_P, _P]),
    "sbz_synchronize": (_I, [_P]),
    "sbz_set_option": (_I, [_P, ctypes.c_int32, ctypes.c_int64]),
    "sbz_get_option": (_I, [_P, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]),
    "sbz_site_positions": (_I, [_P, _P]),
    "sbz_loglik_batch_device_pm": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P]),
    "sbz_source_layout_device": (_I, [_P, _I, _P, _P, ctypes.c_int32]),
    "sbz_check_indices_device_pm": (_I, [_P, _I, _P, _P]),
    "sbz_loglik_batch": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P]),
    "sbz_loglik_batch_pm": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P]),
    "sbz_loglik_batch_device": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P]),
    "sbz_check_indices_device": (_I, [_P, _I, _P, _P]),
    "sbz_device_alloc": (_I, [_P, ctypes.c_uint64, ctypes.POINTER(_P)]),
    "sbz_device_free": (_I, [_P, _P]),
    "sbz_memcpy_h2d": (_I, [_P, _P, _P, ctypes.c_uint64]),
    "sbz_memcpy_d2h": (_I, [_P, _P, _P, ctypes.c_uint64]),
    "sbz_lik_lds_bytes": (ctypes.c_uint64, [ctypes.POINTER(sbz_dims), _I]),
    "sbz_set_network": (_I, [_P, _P, ctypes.c_int32, _P, _P]),
    "sbz_set_priors": (_I, [_P, _P, _P, ctypes.c_int32]),
    "sbz_set_geo_prior": (_I, [_P, _P, ctypes.c_double]),
    "sbz_set_gibbs_counts": (_I, [_P, _P, _P]),
    "sbz_mh_run_device": (_I, [_P, _I, _I, ctypes.POINTER(sbz_mh_config), ctypes.POINTER(sbz_chains)]),
    "sbz_mh_run": (_I, [_P, _I, _I, ctypes.POINTER(sbz_mh_config), ctypes.c_uint64,
                        ctypes.POINTER(sbz_tape), ctypes.POINTER(sbz_state), ctypes.POINTER(sbz_trace)]),
    "sbz_mh_lds_bytes": (ctypes.c_uint64, [ctypes.POINTER(sbz_dims)]),
    "sbz_last_kernels": (ctypes.c_char_p, [_P]),
    "sbz_draw_gamma": (_I, [_P, ctypes.c_int32, _P, ctypes.c_uint64, _P]),
}

_lib = None


def lib():
    """Load libsbz.so once (raises if it is missing: there is no fallback path)."""
    global _lib
    if _lib is None:
        # The library links the HIP runtime PyTorch ships (torch/lib/libamdhip64.so, DT_RPATH);
        # importing torch first guarantees a single HIP/HSA runtime in the process.
        import torch  # noqa: F401
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C contact_zones_amd/csrc` "
                              "(or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, ctx=None):
    if rc != SBZ_OK:
        msg = lib().sbz_last_error(ctx).decode() if ctx else ""
        raise SbzError(rc, msg)
