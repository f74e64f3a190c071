"""Batched evaluation of logged samples on the GPU (callers of the likelihood kernel).

``contribution_per_area`` restates sbayes/postprocessing.py:271-313: for every logged sample and
every zone, the log-likelihood and log prior of the sample with only that zone.  The reference
calls ``likelihood`` and ``prior`` once per (sample, zone); here all n_samples x n_zones
single-zone samples go to the likelihood kernel as one batch (a context with n_zones = 1, in
chunks of ``batch`` samples) and the priors are evaluated vectorised on the host
(contact_zones_amd/priors.py).
"""
import numpy as np

from . import packing


def single_zone_batch(stats, s0, s1):
    """The single-zone samples of logged samples s0 .. s1 (sample-major, zone-minor) as packed
    arrays: zone_of_site [B][N] (0 = in the zone, 255 = not), w, p_global, p_zones [B][1][F][S],
    p_fam (or None)."""
    zones = np.asarray(stats["sample_zones"][s0:s1], bool)          # [n][Z][N]
    n, Z, N = zones.shape
    zos = np.where(zones.reshape(n * Z, N), 0, packing.NONE).astype(np.uint8)
    rep = lambda a: np.repeat(np.asarray(a, np.float64), Z, axis=0)  # noqa: E731
    w = rep(stats["sample_weights"][s0:s1])
    pg = rep(np.asarray(stats["sample_p_global"][s0:s1], np.float64)[:, 0])
    pz = np.asarray(stats["sample_p_zones"][s0:s1], np.float64)
    pz = pz.reshape(n * Z, 1, pz.shape[-2], pz.shape[-1])
    pf = None
    fams = stats["sample_p_families"][s0:s1]
    if len(fams) and fams[0] is not None:
        pf = rep(fams)
    return zos, w, pg, pz, pf


def contribution_per_area(mcmc_sampler, batch=4096):
    """Fill statistics['sample_lh_single_zones'], ['sample_prior_single_zones'] and
    ['sample_posterior_single_zones'] (lists of per-zone lists, as the reference) for a
    BatchedZoneMCMC run."""
    from .likelihood import LikelihoodEngine
    smp = mcmc_sampler
    stats = smp.statistics
    n = len(stats["sample_zones"])
    lh, pr = [], []
    if n:
        Z = np.asarray(stats["sample_zones"][0]).shape[0]
        eng = getattr(smp, "_engine_single_zone", None)
        if eng is None:
            fam = packing.families_to_fam_of_site(
                smp.families if smp.inheritance and smp.families.shape[0] else None, smp.n_sites)
            smp._get_engine()  # fixes the device
            eng = LikelihoodEngine(packing.features_to_obs(smp.features), fam, smp.n_states, 1,
                                   smp.families.shape[0] if smp.inheritance else 0,
                                   smp.inheritance, device=smp._device)
            smp._engine_single_zone = eng
        per = max(1, batch // max(Z, 1))
        for s0 in range(0, n, per):
            s1 = min(n, s0 + per)
            zos, w, pg, pz, pf = single_zone_batch(stats, s0, s1)
            lh.append(eng.loglik(zos, w, pg, pz, pf))
            pr.append(smp.priors.log_prior(zos, pg, pf, smp.applicable_states, 1, smp.inheritance))
        lh = np.concatenate(lh).reshape(n, Z)
        pr = np.concatenate(pr).reshape(n, Z)
    else:
        lh = pr = np.zeros((0, 0))
    stats["sample_lh_single_zones"] = [list(r) for r in lh]
    stats["sample_prior_single_zones"] = [list(r) for r in pr]
    stats["sample_posterior_single_zones"] = [list(a + b) for a, b in zip(lh, pr)]
    smp.statistics = stats
