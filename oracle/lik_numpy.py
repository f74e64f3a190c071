"""CPU restatement (numpy) of the sBayes mixture likelihood — TEST INFRASTRUCTURE ONLY.

This module is the *oracle* for the HIP likelihood path.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it,
and only as the checker / timed CPU baseline.  The product path
(``contact_zones_amd``) never imports anything under ``oracle/``.

It restates, on the packed representation used at the C-ABI boundary, the
array program of the reference ``Likelihood.__call__(sample, caching=False)``:

* component likelihoods as exact one-hot gathers
  (``compute_global_likelihood`` sbayes/model.py:297-330,
  ``compute_zone_likelihood`` :333-392, ``compute_family_likelihood`` :395-433);
* NA cells set to 1 for every component (``update_component_likelihoods`` :242-247);
* per-site normalised weights (``update_weights`` :257-294, ``normalize_weights`` :436-452);
* mixture combine ``sum(log(sum_c w*lh))`` (``combine_lh`` :174-176) and the source
  branch ``sum(log(w*lh)[source])`` with ``-inf`` on a zero selected weight (:177-184).

The temporaries keep the reference's shapes and C-order (N, F, C), so numpy's
reductions run in the same order as in the reference; the golden fixtures under
``tests/golden`` (captured from the reference itself) pin it.

Packed representation (see include/sbz.h):
  obs          int8  (N, F)      state index, -1 = NA
  fam_of_site  uint8 (N,)        family index, 255 = no family
  zone_of_site uint8 (N,)        zone index,   255 = no zone (zones are disjoint)
  w            f64   (F, C)      unnormalised mixture weights (C = 3 with inheritance)
  p_global     f64   (F, S)
  p_zones      f64   (Z, F, S)
  p_fam        f64   (Fam, F, S) or None
  source       uint8 (N, F)      component index per cell, or None (mixture mode)
"""
import numpy as np

NONE = 255


def component_lh(obs, fam_of_site, zone_of_site, p_global, p_zones, p_fam, inheritance):
    """Return all_lh (N, F, C) exactly as update_component_likelihoods builds it."""
    n_sites, n_features = obs.shape
    na = obs < 0
    x = np.where(na, 0, obs).astype(np.intp)
    f_idx = np.broadcast_to(np.arange(n_features)[None, :], x.shape)

    # global: features[:, f, :] . p_global[0, f, :] == p_global[f, x]   (model.py:324-328)
    lh_global = p_global[f_idx, x]

    # zone: zeros for sites outside every zone (model.py:358), gather inside (model.py:387-390)
    lh_zone = np.zeros((n_sites, n_features))
    in_zone = zone_of_site != NONE
    if np.any(in_zone):
        zs = zone_of_site[in_zone].astype(np.intp)
        lh_zone[in_zone] = p_zones[zs[:, None], f_idx[in_zone], x[in_zone]]

    comps = [lh_global, lh_zone]
    if inheritance:
        lh_fam = np.zeros((n_sites, n_features))
        in_fam = fam_of_site != NONE
        if np.any(in_fam):
            fs = fam_of_site[in_fam].astype(np.intp)
            lh_fam[in_fam] = p_fam[fs[:, None], f_idx[in_fam], x[in_fam]]
        comps.append(lh_fam)

    # np.array([...]).transpose((1, 2, 0)) then copy to C order (model.py:242-245)
    all_lh = np.ascontiguousarray(np.array(comps).transpose((1, 2, 0)))
    all_lh[na] = 1.0                                            # model.py:247
    return all_lh


def has_components(fam_of_site, zone_of_site, inheritance):
    """(N, C) bool: [global, zone, family] membership (model.py:272-281)."""
    n = zone_of_site.shape[0]
    cols = [np.ones(n, dtype=bool), zone_of_site != NONE]
    if inheritance:
        cols.append(fam_of_site != NONE)
    return np.array(cols).T


def normalized_weights(w, fam_of_site, zone_of_site, inheritance):
    """(N, F, C) normalised weights (model.py:284-292 -> normalize_weights :436-452)."""
    has = has_components(fam_of_site, zone_of_site, inheritance)
    weights_per_site = w[np.newaxis, :, :] * has[:, np.newaxis, :]
    return weights_per_site / weights_per_site.sum(axis=2, keepdims=True)


def loglik(obs, fam_of_site, zone_of_site, w, p_global, p_zones, p_fam=None,
           source=None, inheritance=None):
    """Log-likelihood of ONE chain (Likelihood.__call__ with caching=False, model.py:145-171)."""
    if inheritance is None:
        inheritance = w.shape[-1] == 3
    all_lh = component_lh(obs, fam_of_site, zone_of_site, p_global, p_zones, p_fam, inheritance)
    weights = normalized_weights(w, fam_of_site, zone_of_site, inheritance)
    if source is None:
        feature_lh = np.sum(weights * all_lh, axis=2)           # model.py:175
        return float(np.sum(np.log(feature_lh)))                # model.py:176
    sel = source.astype(np.intp)[..., None]
    obs_w = np.take_along_axis(weights, sel, axis=2)[..., 0].ravel()
    obs_lh = np.take_along_axis(all_lh, sel, axis=2)[..., 0].ravel()
    if np.any(obs_w == 0):                                      # model.py:181-182
        return -np.inf
    return float(np.sum(np.log(obs_w * obs_lh)))                # model.py:184


def loglik_batch(obs, fam_of_site, zone_of_site, w, p_global, p_zones, p_fam=None,
                 source=None, inheritance=None):
    """Chains stacked on a leading axis B; returns (B,) float64."""
    out = np.empty(zone_of_site.shape[0])
    for b in range(out.shape[0]):
        out[b] = loglik(obs, fam_of_site, zone_of_site[b], w[b], p_global[b], p_zones[b],
                        None if p_fam is None else p_fam[b],
                        None if source is None else source[b], inheritance)
    return out


def source_posterior(obs, fam_of_site, zone_of_site, w, p_global, p_zones, p_fam=None,
                     inheritance=None):
    """normalize(lh * w) over components (zone_sampling.py:202 / util.normalize :1087-1105)."""
    if inheritance is None:
        inheritance = w.shape[-1] == 3
    all_lh = component_lh(obs, fam_of_site, zone_of_site, p_global, p_zones, p_fam, inheritance)
    weights = normalized_weights(w, fam_of_site, zone_of_site, inheritance)
    x = all_lh * weights
    return x / np.sum(x, axis=-1, keepdims=True)
