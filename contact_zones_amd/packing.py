"""Host-side packing between the reference's array layouts and the sbz C-ABI layouts.

Reference layouts (sbayes):
  features   (N, F, S) one-hot bool/int, all-zero row = NA   (sbayes/util.py:289-336)
  families   (Fam, N) bool, disjoint                          (sbayes/util.py:398-403)
  zones      (Z, N) bool, disjoint by construction            (zone_sampling.py:799, 829)
  source     (N, F, C) one-hot bool                           (zone_sampling.py:205, 1229)

sbz layouts (include/sbz.h):
  obs          int8  (N, F)   state index, -1 = NA
  fam_of_site  uint8 (N,)     family index, 255 = none
  zone_of_site uint8 (N,)     zone index, 255 = none
  source       uint8 (N, F)   component index
"""
import numpy as np

NONE = 255
MAX_STATES = 127
MAX_GROUPS = 254


def features_to_obs(features):
    f = np.asarray(features)
    if f.ndim != 3:
        raise ValueError(f"features must be (n_sites, n_features, n_states), got {f.shape}")
    if f.shape[2] > MAX_STATES:
        raise ValueError(f"at most {MAX_STATES} states supported, got {f.shape[2]}")
    fb = f.astype(bool)
    counts = fb.sum(axis=-1)
    if np.any(counts > 1):
        raise ValueError("features must be one-hot per (site, feature)")
    obs = np.argmax(fb, axis=-1).astype(np.int8)
    obs[counts == 0] = -1
    return obs


def obs_to_features(obs, n_states):
    obs = np.asarray(obs)
    eye = np.eye(n_states, dtype=bool)
    feats = eye[np.where(obs < 0, 0, obs)]
    feats[obs < 0] = False
    return feats


def groups_to_index(groups, n_sites, what):
    """(G, N) bool membership -> uint8 (N,) index (255 = none); groups must be disjoint."""
    if groups is None:
        return np.full(n_sites, NONE, dtype=np.uint8)
    g = np.asarray(groups).astype(bool)
    if g.ndim != 2 or g.shape[1] != n_sites:
        raise ValueError(f"{what} must be ({what[:-1]}_count, {n_sites}), got {g.shape}")
    if g.shape[0] > MAX_GROUPS:
        raise ValueError(f"at most {MAX_GROUPS} {what} supported")
    if np.any(g.sum(axis=0) > 1):
        raise ValueError(f"{what} must be disjoint")
    idx = np.full(n_sites, NONE, dtype=np.uint8)
    gi, si = np.nonzero(g)
    idx[si] = gi.astype(np.uint8)
    return idx


def index_to_groups(idx, n_groups):
    idx = np.asarray(idx)
    return (idx[None, :] == np.arange(n_groups)[:, None])


def families_to_fam_of_site(families, n_sites):
    return groups_to_index(families, n_sites, "families")


def zones_to_zone_of_site(zones, n_sites):
    return groups_to_index(zones, n_sites, "zones")


def source_to_index(source):
    s = np.asarray(source).astype(bool)
    if np.any(s.sum(axis=-1) != 1):
        raise ValueError("source must be one-hot over components")
    return np.argmax(s, axis=-1).astype(np.uint8)


def index_to_source(idx, n_components):
    return np.eye(n_components, dtype=bool)[np.asarray(idx)]
