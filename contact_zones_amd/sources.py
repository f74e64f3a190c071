"""Initial source assignments of SAMPLE_SOURCE = true chains (host side, once per chain).

generate_initial_sample ends with one Gibbs draw of every observation's source
(zone_sampling.py:1227-1231 -> gibbs_sample_sources :180-215): the posterior
normalize(lh_per_component * normalised weights) of each (site, feature) and a categorical draw
with ``np.random.random`` (preprocessing.sample_categorical :321-348).  It runs here, with the
reference's own numpy global RNG and operation order, so a seeded run starts from the
reference's sources; every later source draw happens in the sampler kernel (sbz_mh_src.hip).
"""
import numpy as np

from .packing import NONE


def component_likelihoods(obs, fam_of_site, zone_of_site, p_global, p_zones, p_fam, inheritance):
    """(N, F, C) lh per component as update_component_likelihoods (model.py:224-247): the one-hot
    gathers of p_global / p_zones / p_families (0 for a site outside every zone / family), every
    component 1 at NA cells."""
    N, F = obs.shape
    na = obs < 0
    x = np.where(na, 0, obs).astype(np.intp)
    fi = np.broadcast_to(np.arange(F)[None, :], x.shape)
    comps = [p_global[fi, x]]
    lz = np.zeros((N, F))
    iz = zone_of_site != NONE
    if iz.any():
        lz[iz] = p_zones[zone_of_site[iz].astype(np.intp)[:, None], fi[iz], x[iz]]
    comps.append(lz)
    if inheritance:
        lf = np.zeros((N, F))
        ifm = fam_of_site != NONE
        if ifm.any():
            lf[ifm] = p_fam[fam_of_site[ifm].astype(np.intp)[:, None], fi[ifm], x[ifm]]
        comps.append(lf)
    lh = np.ascontiguousarray(np.array(comps).transpose((1, 2, 0)))
    lh[na] = 1.0
    return lh


def normalized_weights(fam_of_site, zone_of_site, w, inheritance):
    """(N, F, C) update_weights -> normalize_weights (model.py:251-294, 436-452): w * has / sum."""
    N = zone_of_site.shape[0]
    has = [np.ones(N, bool), zone_of_site != NONE]
    if inheritance:
        has.append(fam_of_site != NONE)
    wps = w[None, :, :] * np.stack(has, axis=1)[:, None, :]
    return wps / wps.sum(axis=2, keepdims=True)


def source_posterior(obs, fam_of_site, zone_of_site, w, p_global, p_zones, p_fam, inheritance):
    """(N, F, C) normalize(lh * weights) for one chain in packed form (obs int8 [N][F], -1 = NA):
    lh per component as update_component_likelihoods (model.py:224-247; NA -> 1, a site outside
    every zone / family -> 0), weights as update_weights -> normalize_weights (:284-292, 436-452)."""
    lh = component_likelihoods(obs, fam_of_site, zone_of_site, p_global, p_zones, p_fam, inheritance)
    wn = normalized_weights(fam_of_site, zone_of_site, w, inheritance)
    p = lh * wn
    return p / np.sum(p, axis=-1, keepdims=True)


def draw_sources(post, random=np.random.random):
    """sample_categorical(post) as indices: argmax(u < cumsum(p)) with one uniform per
    (site, feature), drawn in C order by ``random(shape)``."""
    cdf = np.cumsum(post, axis=-1)
    u = random(list(post.shape[:-1]) + [1])
    return np.argmax(u < cdf, axis=-1).astype(np.uint8)
