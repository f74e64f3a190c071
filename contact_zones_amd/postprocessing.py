"""Batched evaluation of logged samples on the GPU (callers of the likelihood kernel).

``contribution_per_area`` restates sbayes/postprocessing.py:271-313: for every logged sample and
every zone, the log-likelihood and log prior of the sample with only that zone.  The reference
calls ``likelihood`` and ``prior`` once per (sample, zone); here all n_samples x n_zones
single-zone samples go to the likelihood kernel as one batch (a context with n_zones = 1, in
chunks of ``batch`` samples) and the priors are evaluated vectorised on the host
(contact_zones_amd/priors.py).

``eval_ground_truth`` restates MCMC.eval_ground_truth (sbayes/mcmc_setup.py:122-172) for
simulated data: the true sample and each of its zones alone, in two likelihood launches.
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


def _single_zone_engine(smp):
    """The sampler's likelihood context for single-zone samples (n_zones = 1), made once."""
    from .likelihood import LikelihoodEngine
    eng = getattr(smp, "_engine_single_zone", None)
    if eng is None:
        fam = packing.families_to_fam_of_site(
            smp.families if smp.inheritance and smp.families.shape[0] else None, smp.n_sites)
        smp._get_engine()  # fixes the device
        eng = LikelihoodEngine(packing.features_to_obs(smp.features), fam, smp.n_states, 1,
                               smp.families.shape[0] if smp.inheritance else 0,
                               smp.inheritance, device=smp._device)
        smp._engine_single_zone = eng
    return eng


def contribution_per_area(mcmc_sampler, batch=4096):
    """Fill statistics['sample_lh_single_zones'], ['sample_prior_single_zones'] and
    ['sample_posterior_single_zones'] (lists of per-zone lists, as the reference) for a
    BatchedZoneMCMC run."""
    smp = mcmc_sampler
    stats = smp.statistics
    n = len(stats["sample_zones"])
    lh, pr = [], []
    if n:
        Z = np.asarray(stats["sample_zones"][0]).shape[0]
        eng = _single_zone_engine(smp)
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


def eval_ground_truth(mcmc_sampler, data, inheritance, samples, lh_per_area=True):
    """MCMC.eval_ground_truth (sbayes/mcmc_setup.py:122-172): the likelihood and prior of the
    simulated ground truth (data.areas, data.weights, data.p_universal, data.p_contact,
    data.p_inheritance), and with ``lh_per_area`` of each true zone alone, written into
    ``samples`` under the reference's keys.  Without inheritance the weights are
    normalize(data.weights[:, :2]) (mcmc_setup.py:125-128).  One likelihood launch for the
    true sample (a context with as many zones as the truth) and one for its single zones."""
    from .likelihood import LikelihoodEngine
    smp = mcmc_sampler
    w = np.asarray(data.weights, np.float64)
    weights = w.copy() if inheritance else w[:, :2] / np.sum(w[:, :2], axis=-1, keepdims=True)
    areas = np.asarray(data.areas, bool)
    Z, N = areas.shape
    pg = np.asarray(data.p_universal, np.float64)[np.newaxis, ...]          # [1][F][S]
    pz = np.asarray(data.p_contact, np.float64)                            # [Z][F][S]
    p_inh = getattr(data, "p_inheritance", None)
    pf = np.asarray(p_inh, np.float64) if inheritance else None            # [Fam][F][S]

    samples["true_zones"] = data.areas
    samples["true_weights"] = weights
    samples["true_p_global"] = pg
    samples["true_p_zones"] = data.p_contact
    samples["true_p_families"] = p_inh
    zos = packing.zones_to_zone_of_site(areas, N)[np.newaxis]
    if Z == smp.n_zones:
        eng = smp._get_engine()
    else:  # a truth with another number of zones than the sampler's model
        eng = getattr(smp, "_engine_truth", None)
        if eng is None or eng.dims.n_zones != Z:
            smp._get_engine()
            fam = packing.families_to_fam_of_site(
                smp.families if smp.inheritance and smp.families.shape[0] else None, smp.n_sites)
            eng = LikelihoodEngine(packing.features_to_obs(smp.features), fam, smp.n_states, Z,
                                   smp.families.shape[0] if smp.inheritance else 0,
                                   smp.inheritance, device=smp._device)
            smp._engine_truth = eng
    samples["true_ll"] = float(eng.loglik(zos, weights[np.newaxis], pg, pz[np.newaxis],
                                          None if pf is None else pf[np.newaxis])[0])
    samples["true_prior"] = float(smp.priors.log_prior(zos, pg, None if pf is None else pf[np.newaxis],
                                                       smp.applicable_states, Z, inheritance)[0])
    samples["true_families"] = getattr(data, "families", None)
    if lh_per_area:
        zs = np.where(areas, 0, packing.NONE).astype(np.uint8)              # [Z][N]
        rep = lambda a: np.repeat(a, Z, axis=0)  # noqa: E731
        lh = _single_zone_engine(smp).loglik(zs, rep(weights[np.newaxis]), rep(pg),
                                             pz[:, np.newaxis], None if pf is None else rep(pf[np.newaxis]))
        pr = smp.priors.log_prior(zs, rep(pg), None if pf is None else rep(pf[np.newaxis]),
                                  smp.applicable_states, 1, inheritance)
        samples["true_lh_single_zones"] = [float(v) for v in lh]
        samples["true_prior_single_zones"] = [float(v) for v in pr]
        samples["true_posterior_single_zones"] = [float(a + b) for a, b in zip(lh, pr)]
    return samples


def match_areas(samples):
    """sbayes/postprocessing.py:205-268: relabel every logged sample's zones so that they agree
    best with the running sum of the relabelled earlier samples.  The reference scores every
    permutation p of the zone labels as sum(s_sum * s[:, p]) and keeps the first maximum in
    itertools.permutations order; that score is sum_z M[z, p[z]] with the Z x Z overlap matrix
    M = s_sum^T s, so all Z! scores come from one gather of M per sample.  The counts are
    integers, so the scores (and their ties) are exact as in the reference."""
    from itertools import permutations
    zones = np.asarray([np.asarray(s) for s in samples["sample_zones"]])   # [n][Z][N]
    n, Z, N = zones.shape
    perms = np.array(list(permutations(range(Z))), dtype=np.int64)          # [Z!][Z]
    s_sum = np.zeros((Z, N))                                                 # zone-major
    matching = []
    rows = np.arange(Z)
    for s in zones.astype(np.float64):
        M = s_sum @ s.T                                                      # M[a][b] = sum_site s_sum[a] s[b]
        score = M[rows[None, :], perms].sum(axis=1)
        best = perms[int(np.argmax(score))]
        matching.append(best)
        s_sum += s[best]
    for key in ("sample_zones", "sample_p_zones"):
        if key in samples:  # (a chain logged without parameters has no p_zones: mcmc.ChainLog)
            samples[key] = [samples[key][i][:][m] if key == "sample_zones" else samples[key][i][m]
                            for i, m in enumerate(matching[:len(samples[key])])]
    for key in ("sample_lh_single_zones", "sample_prior_single_zones", "sample_posterior_single_zones"):
        if key in samples:
            samples[key] = [[samples[key][i][j] for j in m] for i, m in enumerate(matching[:len(samples[key])])]
    return samples


def rank_areas(samples):
    """sbayes/postprocessing.py:316-363: order the zones of every sample by their mean posterior
    contribution (sample_posterior_single_zones), largest first (np.argsort(-mean))."""
    to_rank = np.mean(np.asarray(samples["sample_posterior_single_zones"]), axis=0)
    ranked = np.argsort(-to_rank)
    samples["sample_zones"] = [np.asarray(z)[ranked] for z in samples["sample_zones"]]
    for key in ("sample_lh_single_zones", "sample_prior_single_zones", "sample_posterior_single_zones"):
        samples[key] = [[v[r] for r in ranked] for v in samples[key]]
    samples["sample_p_zones"] = [np.asarray(p)[ranked] for p in samples["sample_p_zones"]]
    return samples
