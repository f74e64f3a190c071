"""CPU restatement (numpy) of the sBayes Metropolis-Hastings step — TEST INFRASTRUCTURE ONLY.

The oracle for the HIP sampler.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
CPU-baseline leg may import it, and only as the checker.  The product path never imports
``oracle/``.

It replays a *decision tape* (tests/golden/make_golden_mh.py) through a restatement of
``MCMCGenerative.step`` (sbayes/sampling/mcmc_generative.py:282-351) and the operators of
``ZoneMCMC`` / ``ZoneMCMCWarmup`` with SAMPLE_SOURCE = false; priors zero (uniform), 'counts'
on p_global / p_families and 'uniform' / 'quadratic' on zone sizes (``Model.log_prior``):

  shrink_zone   zone_sampling.py:866-933      (warm-up :1498-1574: q_back = 1/(size+1))
  grow_zone     zone_sampling.py:788-864      (warm-up :1418-1496)
  swap_zone     zone_sampling.py:704-786      (warm-up :1328-1416)
  alter_weights zone_sampling.py:408-452
  alter_p_global / alter_p_zones / alter_p_families   :454-535, :571-612
  dirichlet_proposal  :537-569  (q = exp(scipy dirichlet._logpdf), then log)
  gibbsish_sample_zones :619-702 (warm-up :1323-1326: max_size[c]; SAMPLE_SOURCE: sources of the
                                  available sites redrawn)
  get_neighbours      sbayes/util.py:139-155  (adj . zone > 0, minus occupied sites)

Each random decision the reference draws is read from the tape instead (see the capture
script for the item list); the log-likelihood of a candidate is the full evaluation of
oracle/lik_numpy.py, bit-exact with the reference's Likelihood.__call__.
"""
import math

import numpy as np
from scipy.special import betaln, gammaln, xlogy

from . import lik_numpy

OPS = ["shrink_zone", "grow_zone", "swap_zone", "alter_weights", "alter_p_global",
       "alter_p_zones", "alter_p_families", "gibbsish_sample_zones",
       "gibbs_sample_sources", "gibbs_sample_weights", "gibbs_sample_p_global",
       "gibbs_sample_p_zones", "gibbs_sample_p_families"]
SHRINK, GROW, SWAP, WEIGHTS, P_GLOBAL, P_ZONES, P_FAMILIES, GIBBSISH = range(8)
G_SOURCES, G_WEIGHTS, G_P_GLOBAL, G_P_ZONES, G_P_FAMILIES = range(8, 13)
NONE = 255


class TapeReader:
    """The reference's decisions, in order.  Every draw method names the range it draws from (n,
    the population, alpha) so that DrawTape can make the draws itself; a tape ignores them."""

    def __init__(self, items):
        self.items = items
        self.pos = 0

    def real(self):
        v = self.items[self.pos]
        self.pos += 1
        return float(v)

    def int(self, n=None):
        return int(self.real())

    def op(self):
        return self.int()

    def pair(self, population):
        return [self.int(), self.int()]

    def dirichlet(self, alpha):
        return np.array([self.real(), self.real()])

    def reals(self, n):
        v = self.items[self.pos:self.pos + n]
        assert v.size == n, "tape exhausted"
        self.pos += n
        return np.asarray(v, np.float64)

    def beta(self, a, b):
        """stats.beta(a, b).rvs() per entry (the Gibbs weights draw)."""
        return self.reals(np.size(a))

    def dirichlet_vec(self, alpha):
        """np.random.dirichlet(alpha) over a feature's applicable states (the Gibbs p_* draws)."""
        return self.reals(np.size(alpha))


class DrawTape(TapeReader):
    """The decisions drawn from a numpy Generator instead of a tape (the reference's distributions:
    np.random.choice of the operator by its probability, uniform ints, random.sample pairs,
    np.random.dirichlet proposals, uniform reals) — the CPU baseline's sampler (bench.py), no
    replay.  In SAMPLE_SOURCE = true mode the Gibbs operators draw from the reference's
    distributions too (beta / Dirichlet of the source counts)."""

    def __init__(self, rng, op_probs):
        self.rng = rng
        self.p = np.asarray(op_probs, np.float64) / np.sum(op_probs)
        self.pos = 0

    def real(self):
        return float(self.rng.random())

    def int(self, n=None):
        return int(self.rng.integers(n))

    def op(self):
        return int(self.rng.choice(len(self.p), p=self.p))

    def pair(self, population):
        return [int(v) for v in self.rng.choice(np.asarray(population), 2, replace=False)]

    def dirichlet(self, alpha):
        return self.rng.dirichlet(alpha)

    def reals(self, n):
        return self.rng.random(n)

    def beta(self, a, b):
        return self.rng.beta(a, b)

    def dirichlet_vec(self, alpha):
        return self.rng.dirichlet(alpha)


def geo_prior_distance(zone, cost, scale):
    """geo_prior_distance (model.py:1096-1139) for one zone mask: scipy MST of the zone's cost
    submatrix (csgraph_from_dense, null_value inf), mean exponential log density of its edges."""
    from scipy import stats
    from scipy.sparse.csgraph import csgraph_from_dense, minimum_spanning_tree
    cz = np.asarray(cost)[zone][:, zone]
    if cz.shape[0] <= 1:
        raise ValueError("Too few locations to compute distance.")
    mst = minimum_spanning_tree(csgraph_from_dense(cz, null_value=np.inf))
    distances = mst.tocsr()[mst.nonzero()] if mst.nnz > 0 else 0
    return float(np.mean(stats.expon.logpdf(distances, loc=0, scale=scale)))


def dirichlet_logpdf(x, alpha):
    """scipy.stats.dirichlet._logpdf: -(sum gammaln(a) - gammaln(sum a)) + sum xlogy(a - 1, x)."""
    lnB = np.sum(gammaln(alpha)) - gammaln(np.sum(alpha))
    return -lnB + np.sum(xlogy(alpha - 1, x))


def dirichlet_proposal(w, precision, tape):
    """zone_sampling.py:537-569 with the Dirichlet draw read from the tape."""
    alpha = 1 + precision * w
    w_new = tape.dirichlet(alpha)
    q = np.exp(dirichlet_logpdf(w_new, alpha))
    alpha_back = 1 + precision * w_new
    q_back = np.exp(dirichlet_logpdf(w, alpha_back))
    return w_new, np.log(q), np.log(q_back)


class Model:
    """Shared data of a replay: observations, families, network, applicable states, config."""

    def __init__(self, fx):
        self.obs = fx["obs"]
        self.fam = fx["fam_of_site"]
        self.states = fx["states"].astype(bool)
        self.inheritance = bool(fx["inheritance"])
        self.warmup = bool(fx["warmup"])
        self.min_size = int(fx["min_size"])
        self.max_size = fx["max_size"]
        self.p_grow = fx["p_grow_connected"]
        self.prec = fx["precision"]
        N = self.obs.shape[0]
        indptr, indices = fx["adj_indptr"], fx["adj_indices"]
        self.adj = [indices[indptr[s]:indptr[s + 1]] for s in range(N)]
        self.n_zones = int(fx["n_zones"])
        self.sample_source = bool(fx["sample_source"]) if "sample_source" in fx else False
        if self.sample_source:
            S = self.states.shape[1]
            self.features = np.zeros(self.obs.shape + (S,), bool)   # data.features (N, F, S)
            n, f = np.nonzero(self.obs >= 0)
            self.features[n, f, self.obs[n, f]] = True
            self.gibbs_counts_global = fx["gibbs_counts_global"]
            self.gibbs_counts_fam = fx.get("gibbs_counts_fam")
            n_fam = 0 if self.gibbs_counts_fam is None else self.gibbs_counts_fam.shape[0]
            self.families = np.stack([self.fam == i for i in range(n_fam)]) if n_fam else None
        self.size_prior = int(fx["prior_size"]) if "prior_size" in fx else 0
        self.alpha_global = fx.get("prior_alpha_global")
        self.alpha_fam = fx.get("prior_alpha_fam")
        self.geo_cost = fx.get("prior_geo_cost")
        self.geo_scale = float(fx["prior_geo_scale"]) if "prior_geo_scale" in fx else None

    def log_prior(self, st):
        """Prior.__call__ (model.py:484-505) for the supported types: zone size 'none' /
        'uniform' / 'quadratic' (model.py:932-971), geo / weights / p_zones uniform (0),
        'counts' on p_global and p_families (prior_p_global_dirichlet model.py:1142-1170,
        prior_p_families_dirichlet :1173-1219, util.dirichlet_logpdf = scipy _logpdf)."""
        zos = st["zos"]
        N = zos.shape[0]
        log_prior = 0
        sizes = np.array([np.count_nonzero(zos == z) for z in range(self.n_zones)], dtype=np.int64)
        if self.size_prior == 1:
            log_prior += -np.sum(-betaln(1 + N - sizes, 1 + sizes) - np.log(N + 1))
        elif self.size_prior == 2:
            log_prior += -np.sum(np.log(sizes ** 2))
        else:
            log_prior += 0.
        if self.geo_cost is not None:  # GeoPrior 'cost_based': the last zone only (model.py:1110-1139)
            log_prior += geo_prior_distance(zos == self.n_zones - 1, self.geo_cost, self.geo_scale)
        else:
            log_prior += 0.  # geo
        log_prior += 0.  # weights
        if self.alpha_global is not None:
            lp = np.zeros(self.states.shape[0])
            for f in range(self.states.shape[0]):
                idx = np.flatnonzero(self.states[f])
                lp[f] = dirichlet_logpdf(st["pg"][f, idx], self.alpha_global[f, idx])
            log_prior += np.sum(lp)
        else:
            log_prior += 0
        log_prior += 0.  # p_zones
        if self.inheritance:
            if self.alpha_fam is not None:
                n_fam = self.alpha_fam.shape[0]
                lp = np.zeros((n_fam, self.states.shape[0]))
                for fam in range(n_fam):
                    for f in range(self.states.shape[0]):
                        idx = np.flatnonzero(self.states[f])
                        lp[fam, f] = dirichlet_logpdf(st["pf"][fam, f, idx], self.alpha_fam[fam, f, idx])
                log_prior += np.sum(lp)
            else:
                log_prior += 0.
        return log_prior

    def neighbours(self, zone, occupied):
        """get_neighbours: sites adjacent to the zone that are in no zone (util.py:152-155)."""
        nb = np.zeros(zone.shape[0], bool)
        for s in np.flatnonzero(zone):
            nb[self.adj[s]] = True
        return nb & ~occupied

    def loglik(self, st):
        return lik_numpy.loglik(self.obs, self.fam, st["zos"], st["w"], st["pg"], st["pz"],
                                st.get("pf"), source=st.get("src"), inheritance=self.inheritance)

    def posterior(self, st):
        """normalize(lh_per_component * weights) (zone_sampling.py:193-202)."""
        return lik_numpy.source_posterior(self.obs, self.fam, st["zos"], st["w"], st["pg"],
                                          st["pz"], st.get("pf"), inheritance=self.inheritance)


REJECT = (None, 0.0, -np.inf)


def op_grow(m, st, c, tape):
    zos = st["zos"]
    z = tape.int(m.n_zones)
    zone = zos == z
    size = int(np.count_nonzero(zone))
    if size >= m.max_size[c]:
        return REJECT
    occupied = zos != NONE
    nb = m.neighbours(zone, occupied)
    p = m.p_grow[c]
    connected = tape.real() < p
    candidates = nb if connected else ~occupied
    if not np.any(candidates):
        return REJECT
    site_new = np.flatnonzero(candidates)[tape.int(np.count_nonzero(candidates))]
    new = dict(st, zos=zos.copy())
    new["zos"][site_new] = z
    q = (1 - p) * (1 / np.count_nonzero(~occupied))
    if nb[site_new]:
        q += p * (1 / np.count_nonzero(nb))
    q_back = 1 / (size + 1)
    return new, np.log(q), np.log(q_back)


def op_shrink(m, st, c, tape):
    zos = st["zos"]
    z = tape.int(m.n_zones)
    zone = zos == z
    size = int(np.count_nonzero(zone))
    if size <= m.min_size:
        return REJECT
    removal = np.flatnonzero(zone)
    site_removed = removal[tape.int(len(removal))]
    new = dict(st, zos=zos.copy())
    new["zos"][site_removed] = NONE
    q = 1 / len(removal)
    occupied_new = new["zos"] != NONE
    back_nb = m.neighbours(new["zos"] == z, occupied_new)
    p = m.p_grow[c]
    q_back = (1 - p) * (1 / np.count_nonzero(~occupied_new))
    if back_nb[site_removed]:
        q_back += p * (1 / np.count_nonzero(back_nb))
    if m.warmup:
        q_back = 1 / (size + 1)  # ZoneMCMCWarmup.shrink_zone overwrites it (zone_sampling.py:1561)
    return new, np.log(q), np.log(q_back)


def op_swap(m, st, c, tape):
    zos = st["zos"]
    occupied = zos != NONE
    z = tape.int(m.n_zones)
    zone = zos == z
    nb = m.neighbours(zone, occupied)
    p = m.p_grow[c]
    connected = tape.real() < p
    candidates = nb if connected else ~occupied
    if not np.any(candidates):
        return REJECT
    site_new = np.flatnonzero(candidates)[tape.int(np.count_nonzero(candidates))]
    new = dict(st, zos=zos.copy())
    new["zos"][site_new] = z
    removal = np.flatnonzero(zone)
    site_removed = removal[tape.int(len(removal))]
    new["zos"][site_removed] = NONE
    back_nb = nb  # get_neighbours(zone_current, occupied) again: the same arguments (:752)
    q = (1 - p) * (1 / np.count_nonzero(~occupied))
    if nb[site_new]:
        q += p * (1 / np.count_nonzero(nb))
    q_back = (1 - p) * (1 / np.count_nonzero(~occupied))
    if back_nb[site_removed]:
        q_back += p * (1 / np.count_nonzero(back_nb))
    return new, np.log(q), np.log(q_back)


def _alter_pair(arr_row, idx, precision, tape):
    """Transform a pair to sum 1, propose, transform back (alter_* :421-438, :470-482)."""
    cur = arr_row[idx]
    t = cur / cur.sum()
    t_new, log_q, log_q_back = dirichlet_proposal(t, precision, tape)
    return t_new * cur.sum(), log_q, log_q_back


def op_weights(m, st, c, tape):
    f = tape.int(st["w"].shape[0])
    new = dict(st, w=st["w"].copy())
    if m.inheritance:
        idx = tape.pair(np.arange(3))
        vals, log_q, log_q_back = _alter_pair(st["w"][f], idx, m.prec[0], tape)
        new["w"][f, idx] = vals
    else:
        vals, log_q, log_q_back = dirichlet_proposal(st["w"][f, :], m.prec[0], tape)
        new["w"][f, :] = vals
    return new, log_q, log_q_back


def _states_pair(m, f, tape):
    return tape.pair(np.flatnonzero(m.states[f]))


def op_p_global(m, st, c, tape):
    f = tape.int(m.states.shape[0])
    idx = _states_pair(m, f, tape)
    new = dict(st, pg=st["pg"].copy())
    vals, log_q, log_q_back = _alter_pair(st["pg"][f], idx, m.prec[1], tape)
    new["pg"][f, idx] = vals
    return new, log_q, log_q_back


def op_p_zones(m, st, c, tape):
    z = tape.int(m.n_zones)
    f = tape.int(m.states.shape[0])
    idx = _states_pair(m, f, tape)
    new = dict(st, pz=st["pz"].copy())
    vals, log_q, log_q_back = _alter_pair(st["pz"][z, f], idx, m.prec[2], tape)
    new["pz"][z, f, idx] = vals
    return new, log_q, log_q_back


def op_p_families(m, st, c, tape):
    fam = tape.int(st["pf"].shape[0])
    f = tape.int(m.states.shape[0])
    idx = _states_pair(m, f, tape)
    new = dict(st, pf=st["pf"].copy())
    vals, log_q, log_q_back = _alter_pair(st["pf"][fam, f], idx, m.prec[3], tape)
    new["pf"][fam, f, idx] = vals
    return new, log_q, log_q_back


def _cells(m, st, zos):
    """feature_lh = sum_c(all_lh * weights) (N, F) of every site under the zone assignment zos
    (gibbsish_sample_zones :644-667; the same cells as combine_lh, model.py:175)."""
    all_lh = lik_numpy.component_lh(m.obs, m.fam, zos, st["pg"], st["pz"], st.get("pf"), m.inheritance)
    weights = lik_numpy.normalized_weights(st["w"], m.fam, zos, m.inheritance)
    return np.sum(all_lh * weights, axis=-1)


def op_gibbsish(m, st, c, tape):
    """gibbsish_sample_zones (zone_sampling.py:619-702): one zone's available sites (free, or in
    the zone; a random subset of ~100 when more) each resampled in / out of the zone from its
    marginal likelihood with and without the zone."""
    zos = st["zos"]
    occupied = zos != NONE
    z = tape.int()                                   # np.random.choice(range(n_zones)) :625
    zone = zos == z
    available = ~occupied | zone
    n_available = np.count_nonzero(available)
    if n_available > 100:                            # :631-633
        available[available] &= tape.reals(n_available) < (100 / n_available)
        n_available = np.count_nonzero(available)
    if n_available == 0:
        return REJECT
    if m.sample_source:                              # :638-643, the current sample's posterior
        log_q_back_s = log_q_sources(m.posterior(st)[available], st["src"][available])
    with_z, without_z = zos.copy(), zos.copy()
    with_z[available] = z
    without_z[available] = NONE
    lh_with = _cells(m, st, with_z)[available]
    lh_without = _cells(m, st, without_z)[available]
    marginal_with = np.exp(np.sum(np.log(lh_with), axis=-1))
    marginal_without = np.exp(np.sum(np.log(lh_without), axis=-1))
    posterior_zone = marginal_with / (marginal_with + marginal_without)
    new_zone = tape.reals(n_available) < posterior_zone
    new = dict(st, zos=zos.copy())
    new["zos"][available] = np.where(new_zone, z, NONE)
    size = np.count_nonzero(new["zos"] == z)
    if not (m.min_size <= size <= m.max_size[c]):  # :678-681
        return REJECT
    q_per_site = posterior_zone * new_zone + (1 - posterior_zone) * (1 - new_zone)
    log_q = np.sum(np.log(q_per_site))
    old = zone[available]
    q_back_per_site = posterior_zone * old + (1 - posterior_zone) * (1 - old)
    if np.any(q_back_per_site == 0):
        return REJECT
    log_q_back = np.sum(np.log(q_back_per_site))
    if m.sample_source:                              # :694-698
        post = m.posterior(new)[available]
        src = new["src"] = st["src"].copy()
        src[available] = sample_categorical(post, tape)
        if m.warmup:  # ZoneMCMCWarmup.gibbs_sample_sources returns Q_GIBBS = -inf (:1293-1296)
            return new, -np.inf, log_q_back + log_q_back_s
        log_q = log_q + log_q_sources(post, src[available])
        log_q_back = log_q_back + log_q_back_s
    return new, log_q, log_q_back


# ---- SAMPLE_SOURCE = true ------------------------------------------------------------------

def sample_categorical(p, tape):
    """preprocessing.sample_categorical (:321-348): argmax(u < cumsum(p)) with one uniform per
    (site, feature) in C order; 0 when no entry of the cdf exceeds u."""
    N, F, _ = p.shape
    cdf = np.cumsum(p, axis=-1)
    z = tape.reals(N * F).reshape(N, F, 1)
    return np.argmax(z < cdf, axis=-1).astype(np.uint8)


def log_q_sources(post, src):
    """sum log posterior[source] over every observation, in ravel order (zone_sampling.py:218)."""
    C = post.shape[-1]
    is_source = np.where(np.eye(C, dtype=bool)[src].ravel())
    return np.sum(np.log(post.ravel()[is_source]))


def with_sources(op):
    """A zone move with source resampling (zone_sampling.py:716-722, 781-784 etc.): log q_back
    gains the current sources' posterior terms, then every source is redrawn from the new
    sample's posterior (gibbs_sample_sources(as_gibbs=False)) and log q gains theirs."""
    def move(m, st, c, tape):
        log_q_back_s = log_q_sources(m.posterior(st), st["src"])
        new, log_q, log_q_back = op(m, st, c, tape)
        if new is None:
            return REJECT
        post = m.posterior(new)
        new = dict(new, src=sample_categorical(post, tape))
        if m.warmup:
            # ZoneMCMCWarmup.gibbs_sample_sources (zone_sampling.py:1293-1296) passes
            # as_gibbs=True whatever it is given: log q_s = Q_GIBBS = -inf, so the move is
            # accepted without an acceptance draw (mcmc_generative.py:310-311)
            return new, -np.inf, log_q_back + log_q_back_s
        return new, log_q + log_q_sources(post, new["src"]), log_q_back + log_q_back_s
    return move


def op_gibbs_sources(m, st, c, tape):
    """gibbs_sample_sources as an operator (zone_sampling.py:180-215): a Gibbs step."""
    return dict(st, src=sample_categorical(m.posterior(st), tape)), -np.inf, 0


def _source_counts(m, st, sites):
    """np.sum(sample.source[sites], axis=0): per feature and component (F, C)."""
    C = 3 if m.inheritance else 2
    return np.sum(np.eye(C, dtype=bool)[st["src"]][sites], axis=0)


def op_gibbs_weights(m, st, c, tape):
    """gibbs_sample_weights (zone_sampling.py:222-331).  With inheritance the per-feature accept
    draw is made and then overridden (sample_new.weights = w_new, :327): always the new weights."""
    w = st["w"]
    w_new = w.copy()
    has_area = st["zos"] != NONE
    F = w.shape[0]
    if not m.inheritance:
        counts = _source_counts(m, st, has_area)
        for f in range(F):
            w_new[f, :] = tape.dirichlet_vec(1 + counts[f])  # np.random.dirichlet(1 + counts[f])
        return dict(st, w=w_new), -np.inf, 0
    fixed = ["inheritance", "contact"][tape.int(2)]
    if fixed == "inheritance":
        counts = _source_counts(m, st, has_area)
        a = tape.beta(1 + counts[..., 1], 1 + counts[..., 0])  # stats.beta(1 + c_contact, 1 + c_univ).rvs()
        w_new[..., 1] = a * w[..., 0] / (1 - a)
    else:
        counts = _source_counts(m, st, np.any(m.families, axis=0) if m.families is not None else has_area)
        a = tape.beta(1 + counts[..., 2], 1 + counts[..., 0])  # stats.beta(1 + c_inherit, 1 + c_univ).rvs()
        w_new[..., 2] = a * w[..., 0] / (1 - a)
    w_new = normalize(w_new)
    tape.reals(F)                        # np.random.random(F) < p_accept (overridden)
    return dict(st, w=w_new), -np.inf, 0


def normalize(x, axis=-1):
    return x / np.sum(x, axis=axis, keepdims=True)


def _gibbs_p(tape, p_row, prior_counts, counts, idx):
    """p[idx] = np.random.dirichlet(prior_counts[idx] + counts) (value from the tape)."""
    p_row = p_row.copy()
    p_row[idx] = tape.dirichlet_vec(prior_counts[idx] + counts)
    return p_row


def _state_counts(m, st, comp, f, idx, sites=None):
    """np.nansum(features[:, f, idx] where source == comp (and the site in `sites`), axis=0)
    (zone_sampling.py:341-352, :366-373, :390-401)."""
    sel = st["src"][:, f] == comp
    if sites is not None:
        sel = sel & sites
    return np.sum(m.features[sel][:, f, idx], axis=0)


def op_gibbs_p_global(m, st, c, tape, fraction_of_features=0.4):
    """gibbs_sample_p_global (zone_sampling.py:334-357)."""
    F = st["pg"].shape[0]
    subset = tape.reals(F) < fraction_of_features
    pg = st["pg"].copy()
    for f in np.flatnonzero(subset):
        idx = np.flatnonzero(m.states[f])
        pg[f] = _gibbs_p(tape, pg[f], m.gibbs_counts_global[f], _state_counts(m, st, 0, f, idx), idx)
    return dict(st, pg=pg), -np.inf, 0


def op_gibbs_p_zones(m, st, c, tape):
    """gibbs_sample_p_zones (zone_sampling.py:359-379)."""
    z = tape.int(m.n_zones)  # np.random.randint(0, n_zones)
    pz = st["pz"].copy()
    ones = np.ones(m.states.shape[1])
    for f in range(pz.shape[1]):
        idx = np.flatnonzero(m.states[f])
        pz[z, f] = _gibbs_p(tape, pz[z, f], ones, _state_counts(m, st, 1, f, idx, st["zos"] == z), idx)
    return dict(st, pz=pz), -np.inf, 0


def op_gibbs_p_families(m, st, c, tape, fraction_of_features=0.4):
    """gibbs_sample_p_families (zone_sampling.py:381-406)."""
    fam = tape.int(st["pf"].shape[0])  # np.random.randint(0, n_families)
    F = st["pf"].shape[1]
    subset = tape.reals(F) < fraction_of_features
    pf = st["pf"].copy()
    for f in np.flatnonzero(subset):
        idx = np.flatnonzero(m.states[f])
        pf[fam, f] = _gibbs_p(tape, pf[fam, f], m.gibbs_counts_fam[fam, f],
                              _state_counts(m, st, 2, f, idx, m.fam == fam), idx)
    return dict(st, pf=pf), -np.inf, 0


OPERATORS = {SHRINK: op_shrink, GROW: op_grow, SWAP: op_swap, WEIGHTS: op_weights,
             P_GLOBAL: op_p_global, P_ZONES: op_p_zones, P_FAMILIES: op_p_families,
             GIBBSISH: op_gibbsish, G_SOURCES: op_gibbs_sources, G_WEIGHTS: op_gibbs_weights,
             G_P_GLOBAL: op_gibbs_p_global, G_P_ZONES: op_gibbs_p_zones,
             G_P_FAMILIES: op_gibbs_p_families}
SOURCE_MOVES = {SHRINK: with_sources(op_shrink), GROW: with_sources(op_grow),
                SWAP: with_sources(op_swap)}


def step(m, st, ll, prior, c, tape):
    """MCMCGenerative.step (mcmc_generative.py:282-329).  Returns (state, ll, prior, op,
    accepted)."""
    op = tape.op()
    fn = SOURCE_MOVES[op] if (m.sample_source and op in SOURCE_MOVES) else OPERATORS[op]
    cand, log_q, log_q_back = fn(m, st, c, tape)
    if log_q_back == -np.inf:
        return st, ll, prior, op, False
    ll_cand = m.loglik(cand)
    prior_cand = m.log_prior(cand)
    if log_q == -np.inf:
        accept = True
    else:
        mh = ((ll_cand - ll) * 1.0) - (log_q - log_q_back) + (prior_cand - prior)
        accept = math.log(tape.real()) < mh
    if accept:
        return cand, ll_cand, prior_cand, op, True
    return st, ll, prior, op, False


def initial_state(fx, c):
    st = {"zos": fx["init_zone_of_site"][c].copy(), "w": fx["init_w"][c].copy(),
          "pg": fx["init_p_global"][c].copy(), "pz": fx["init_p_zones"][c].copy()}
    if bool(fx["inheritance"]):
        st["pf"] = fx["init_p_fam"][c].copy()
    if "init_source" in fx:
        st["src"] = fx["init_source"][c].copy()
    return st


def replay(fx, chain, n_steps=None):
    """Replay chain `chain` of a captured fixture; returns per-step (op, accepted, ll, zos) arrays
    and the final state."""
    m = Model(fx)
    st = initial_state(fx, chain)
    ll = m.loglik(st)
    prior = m.log_prior(st)
    init_prior = prior
    tape = TapeReader(fx["tape"][chain, :int(fx["tape_len"][chain])])
    steps = fx["step_op"].shape[1] if n_steps is None else n_steps
    ops, acc, lls, priors, zos, srcs = [], [], [], [], [], []
    for _ in range(steps):
        st, ll, prior, op, a = step(m, st, ll, prior, chain, tape)
        ops.append(op)
        acc.append(a)
        lls.append(ll)
        priors.append(prior)
        zos.append(st["zos"].copy())
        if "src" in st:
            srcs.append(st["src"].copy())
    return dict(op=np.array(ops), accept=np.array(acc), ll=np.array(lls), prior=np.array(priors),
                init_prior=init_prior, zos=np.array(zos), src=np.array(srcs), state=st,
                tape_used=tape.pos)
