"""GPU likelihood: batched engine + drop-in for ``sbayes.model.Likelihood``.

``LikelihoodEngine`` owns one sbz context (one GPU) holding the shared data
(observations, family membership) and evaluates the full log-likelihood of B
chains per call (``sbz_loglik_batch`` / ``sbz_loglik_batch_device``).

``GpuLikelihood(data, inheritance)`` mirrors the reference interface
``Likelihood(data, inheritance)`` / ``__call__(sample, caching=True) -> float``
(sbayes/model.py:69-171): same constructor arguments, same attributes the
operators read (``na_features``, ``has_family``, ``n_sites`` ...), same call
semantics.  The reference caches component likelihoods behind the sample's
``what_changed`` flags; every GPU evaluation is a full, stateless evaluation
(equal to the cached one by construction), after which the ``lh`` flags are
cleared exactly as ``Likelihood.everything_updated`` does (model.py:186-192).
"""
import ctypes

import numpy as np

from . import packing
from ._lib import OPTIONS, SBZ_INHERITANCE, check, lib, sbz_dims


def _ptr(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


class LikelihoodEngine:
    """Batched full log-likelihood on one MI355X (sbz C-ABI context)."""

    def __init__(self, obs, fam_of_site, n_states, n_zones, n_families, inheritance, device=0,
                 options=None):
        obs = np.ascontiguousarray(obs, dtype=np.int8)
        n_sites, n_features = obs.shape
        if fam_of_site is None:
            fam_of_site = np.full(n_sites, packing.NONE, np.uint8)
        self.fam_of_site = np.ascontiguousarray(fam_of_site, dtype=np.uint8)
        self.inheritance = bool(inheritance)
        self.dims = sbz_dims(n_sites, n_features, int(n_states), int(n_zones),
                             int(n_families) if inheritance else 0,
                             SBZ_INHERITANCE if inheritance else 0)
        self.n_sites, self.n_features, self.n_states = n_sites, n_features, int(n_states)
        self.n_zones = int(n_zones)
        self.n_families = int(n_families) if inheritance else 0
        self.n_components = 3 if inheritance else 2
        self._lib = lib()
        ctx = ctypes.c_void_p()
        check(self._lib.sbz_open(int(device), ctypes.byref(self.dims), _ptr(obs),
                                 _ptr(self.fam_of_site), ctypes.byref(ctx)))
        self.ctx = ctx
        self.device = device
        for name, value in (options or {}).items():
            self.set_option(name, value)
        # the context's site order (sbz_site_positions): positions[p] = site at position p, -1 for
        # padding; the position-major source layout [B][F][Np] follows it
        self.n_positions = int(self._lib.sbz_site_positions(self.ctx, None))
        self.positions = np.empty(self.n_positions, np.int32)
        self._lib.sbz_site_positions(self.ctx, self.positions.ctypes.data_as(ctypes.c_void_p))
        self.position_of_site = np.empty(n_sites, np.int64)
        self.position_of_site[self.positions[:n_sites]] = np.arange(n_sites)

    def set_option(self, name, value):
        """sbz_set_option by name (include/sbz.h sbz_option: lik_tasks_per_cu, lik_banked, src_table,
        src_waves, src_hbm, src_stage, mh_lookahead)."""
        if name not in OPTIONS:
            raise ValueError(f"unknown option {name!r} (one of {sorted(OPTIONS)})")
        check(self._lib.sbz_set_option(self.ctx, OPTIONS[name], int(value)), self.ctx)

    def get_option(self, name):
        v = ctypes.c_int64()
        check(self._lib.sbz_get_option(self.ctx, OPTIONS[name], ctypes.byref(v)), self.ctx)
        return int(v.value)

    def sources_to_positions(self, source):
        """Host sources [B][N][F] (by site) -> [B][F][Np] (by position, padding 0)."""
        src = np.asarray(source, np.uint8)
        out = np.zeros((src.shape[0], self.n_features, self.n_positions), np.uint8)
        out[:, :, :self.n_sites] = src[:, self.positions[:self.n_sites], :].transpose(0, 2, 1)
        return out

    def sources_from_positions(self, source_pm):
        """Host sources [B][F][Np] (by position) -> [B][N][F] (by site)."""
        pm = np.asarray(source_pm, np.uint8)
        return np.ascontiguousarray(pm[:, :, self.position_of_site].transpose(0, 2, 1))

    def source_layout_device(self, B, src, dst, to_positions):
        """sbz_source_layout_device on device pointers (async on the engine's stream)."""
        v = ctypes.c_void_p
        check(self._lib.sbz_source_layout_device(self.ctx, int(B), v(src), v(dst), int(bool(to_positions))),
              self.ctx)

    def close(self):
        if getattr(self, "ctx", None):
            self._lib.sbz_close(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, hip_stream):
        check(self._lib.sbz_set_stream(self.ctx, ctypes.c_void_p(hip_stream or 0)), self.ctx)

    def synchronize(self):
        check(self._lib.sbz_synchronize(self.ctx), self.ctx)

    def last_kernels(self):
        """Names of the kernels the context's last launch ran (sbz_last_kernels): a likelihood
        launch's, or the source-mode sampler's variant."""
        return self._lib.sbz_last_kernels(self.ctx).decode()

    def lds_bytes(self, source_mode=False):
        return int(self._lib.sbz_lik_lds_bytes(ctypes.byref(self.dims), int(bool(source_mode))))

    def _check_shapes(self, B, zone_of_site, w, p_global, p_zones, p_fam, source):
        N, F, S, Z, C = self.n_sites, self.n_features, self.n_states, self.n_zones, self.n_components
        exp = {"zone_of_site": (zone_of_site, (B, N)), "w": (w, (B, F, C)),
               "p_global": (p_global, (B, F, S)), "p_zones": (p_zones, (B, Z, F, S))}
        if self.inheritance:
            exp["p_fam"] = (p_fam, (B, self.n_families, F, S))
        if source is not None:
            exp["source"] = (source, (B, N, F))
        for name, (arr, shape) in exp.items():
            if arr is None or tuple(arr.shape) != shape:
                raise ValueError(f"{name}: expected shape {shape}, got "
                                 f"{None if arr is None else tuple(arr.shape)}")

    def loglik(self, zone_of_site, w, p_global, p_zones, p_fam=None, source=None, source_pm=False):
        """Full log-likelihood of B chains from host arrays; returns float64 (B,).  source_pm: the
        sources are [B][F][Np] by position (sbz_loglik_batch_pm: no device transpose), else
        [B][N][F] by site."""
        zone_of_site = np.ascontiguousarray(zone_of_site, dtype=np.uint8)
        B = zone_of_site.shape[0]
        w = np.ascontiguousarray(w, dtype=np.float64)
        p_global = np.ascontiguousarray(p_global, dtype=np.float64)
        p_zones = np.ascontiguousarray(p_zones, dtype=np.float64)
        if self.inheritance:
            p_fam = np.ascontiguousarray(p_fam, dtype=np.float64)
        else:
            p_fam = None
        if source is not None:
            source = np.ascontiguousarray(source, dtype=np.uint8)
        if source is not None and source_pm:
            if source.shape != (B, self.n_features, self.n_positions):
                raise ValueError(f"source (by position): expected {(B, self.n_features, self.n_positions)}, "
                                 f"got {source.shape}")
            self._check_shapes(B, zone_of_site, w, p_global, p_zones, p_fam, None)
        else:
            self._check_shapes(B, zone_of_site, w, p_global, p_zones, p_fam, source)
        out = np.empty(B, dtype=np.float64)
        fn = self._lib.sbz_loglik_batch_pm if (source is not None and source_pm) else self._lib.sbz_loglik_batch
        check(fn(self.ctx, B, _ptr(zone_of_site), _ptr(w), _ptr(p_global),
                                         _ptr(p_zones), _ptr(p_fam), _ptr(source), _ptr(out)),
              self.ctx)
        return out

    def check_indices_device(self, B, zone_of_site, source=0, source_pm=False):
        """Range-check device index arrays (zone bytes < n_zones or 255, source bytes < C; sources
        by site [B][N][F], or by position [B][F][Np] with source_pm); raises SbzError (SBZ_EINVAL)
        otherwise.  Synchronises the engine's stream."""
        v = ctypes.c_void_p
        fn = self._lib.sbz_check_indices_device_pm if source_pm else self._lib.sbz_check_indices_device
        check(fn(self.ctx, int(B), v(zone_of_site), v(source or 0)), self.ctx)

    def loglik_device(self, B, zone_of_site, w, p_global, p_zones, p_fam, source, out_ll,
                      validate=True, source_pm=False):
        """Device-pointer variant (ints = device addresses, 0 for None); async on the stream.
        source_pm: the sources are [B][F][Np] by position (sbz_loglik_batch_device_pm, read in
        place), else [B][N][F] by site.  The kernels trust the index bytes (include/sbz.h), so by
        default they are range-checked first (one extra pass and a stream sync); callers whose
        arrays the sampler itself maintains pass validate=False."""
        if validate:
            self.check_indices_device(B, zone_of_site, source, source_pm)
        v = ctypes.c_void_p
        if source_pm and source:
            check(self._lib.sbz_loglik_batch_device_pm(self.ctx, int(B), v(zone_of_site), v(w),
                                                       v(p_global), v(p_zones), v(p_fam or 0), v(source),
                                                       v(out_ll)), self.ctx)
            return
        check(self._lib.sbz_loglik_batch_device(self.ctx, int(B), v(zone_of_site), v(w), v(p_global),
                                                v(p_zones), v(p_fam or 0), v(source or 0),
                                                v(out_ll)), self.ctx)


def pack_sample(sample, n_sites):
    """Reference ``Sample`` (zone_sampling.py:49-115) -> packed per-chain arrays."""
    zones = sample.zones
    zone_of_site = packing.zones_to_zone_of_site(zones, n_sites)
    p_global = np.asarray(sample.p_global)
    if p_global.ndim == 3:
        p_global = p_global[0]
    src = None if sample.source is None else packing.source_to_index(sample.source)
    pf = None if sample.p_families is None else np.asarray(sample.p_families, np.float64)
    return (zone_of_site, np.asarray(sample.weights, np.float64), np.asarray(p_global, np.float64),
            np.asarray(sample.p_zones, np.float64), pf, src)


class GpuLikelihood:
    """Drop-in for ``sbayes.model.Likelihood`` (sbayes/model.py:69-171) evaluated on the GPU."""

    def __init__(self, data, inheritance, device=0, n_zones=None):
        self.features = data.features
        self.families = np.asarray(data.families, dtype=bool)
        self.inheritance = inheritance
        self.n_sites, self.n_features, self.n_categories = data.features.shape
        self.na_features = (np.sum(self.features, axis=-1) == 0)
        self.has_global = np.ones(self.n_sites, dtype=bool)
        self.has_family = np.any(self.families, axis=0) if self.families.size else \
            np.zeros(self.n_sites, bool)
        self._obs = packing.features_to_obs(self.features)
        n_fam = self.families.shape[0] if self.families.ndim == 2 else 0
        self._fam = packing.families_to_fam_of_site(self.families if n_fam else None, self.n_sites)
        self._n_families = n_fam
        self._device = device
        self._engine = None
        self._engine_zones = n_zones

    def _engine_for(self, n_zones):
        if self._engine is None or self._engine.n_zones != n_zones:
            if self._engine is not None:
                self._engine.close()
            self._engine = LikelihoodEngine(self._obs, self._fam, self.n_categories, n_zones,
                                            self._n_families, self.inheritance, self._device)
        return self._engine

    def reset_cache(self):
        """No device-side cache to reset: every evaluation is a full evaluation."""

    def __call__(self, sample, caching=True):
        zone_of_site, w, pg, pz, pf, src = pack_sample(sample, self.n_sites)
        eng = self._engine_for(pz.shape[0])
        ll = eng.loglik(zone_of_site[None], w[None], pg[None], pz[None],
                        None if pf is None else pf[None], None if src is None else src[None])[0]
        self.everything_updated(sample)
        return float(ll)

    # ---- the arrays the reference's own CPU operators read from the likelihood object
    # (zone_sampling.py:193-199, 239-240, 283, 305-306, 716-719, 801-804, 878-881), so that this
    # object can also replace Likelihood under the reference's sampler in SAMPLE_SOURCE mode.
    # They are host arrays by contract; the GPU sampler (BatchedZoneMCMC) never calls them.
    # Sites that left a zone get a zone likelihood of 0 here where the reference's cache keeps
    # a stale value; both are masked by a zone weight of 0.
    def _packed(self, sample):
        zone_of_site, w, pg, pz, pf, _ = pack_sample(sample, self.n_sites)
        return zone_of_site, w, pg, pz, pf

    def get_zone_assignment(self, sample):
        """model.py:248-252: has_zone per site."""
        return np.any(np.asarray(sample.zones, bool), axis=0)

    def update_weights(self, sample):
        """model.py:251-294: normalised weights (n_sites, n_features, C)."""
        from .sources import normalized_weights
        zone_of_site, w, _, _, _ = self._packed(sample)
        return normalized_weights(self._fam, zone_of_site, w, self.inheritance)

    def update_component_likelihoods(self, sample, caching=True):
        """model.py:230-249: component likelihoods (n_sites, n_features, C), NA cells 1."""
        from .sources import component_likelihoods
        zone_of_site, _, pg, pz, pf = self._packed(sample)
        return component_likelihoods(self._obs, self._fam, zone_of_site, pg, pz, pf, self.inheritance)

    def get_global_lh(self, sample):
        """model.py:190-202: p_global gathered at every observation (0 at NA cells)."""
        lh = self.update_component_likelihoods(sample)[..., 0].copy()
        lh[self.na_features] = 0.0
        return lh

    def get_family_lh(self, sample):
        """model.py:204-217 (None without inheritance)."""
        if not self.inheritance:
            return None
        lh = self.update_component_likelihoods(sample)[..., 2].copy()
        lh[self.na_features] = 0.0
        return lh

    def get_zone_lh(self, sample):
        """model.py:219-228."""
        lh = self.update_component_likelihoods(sample)[..., 1].copy()
        lh[self.na_features] = 0.0
        return lh

    def everything_updated(self, sample):
        """Clear the 'lh' dirty flags exactly as the reference does (model.py:186-192)."""
        wc = getattr(sample, "what_changed", None)
        if not wc:
            return
        lh = wc["lh"]
        lh["zones"].clear()
        lh["p_global"].clear()
        lh["p_zones"].clear()
        lh["weights"] = False
        if self.inheritance:
            lh["p_families"].clear()
