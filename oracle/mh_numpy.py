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
       "alter_p_zones", "alter_p_families", "gibbsish_sample_zones"]
SHRINK, GROW, SWAP, WEIGHTS, P_GLOBAL, P_ZONES, P_FAMILIES = range(7)
NONE = 255


class TapeReader:
    def __init__(self, items):
        self.items = items
        self.pos = 0

    def real(self):
        v = self.items[self.pos]
        self.pos += 1
        return float(v)

    def int(self):
        return int(self.real())


def dirichlet_logpdf(x, alpha):
    """scipy.stats.dirichlet._logpdf: -(sum gammaln(a) - gammaln(sum a)) + sum xlogy(a - 1, x)."""
    lnB = np.sum(gammaln(alpha)) - gammaln(np.sum(alpha))
    return -lnB + np.sum(xlogy(alpha - 1, x))


def dirichlet_proposal(w, precision, tape):
    """zone_sampling.py:537-569 with the Dirichlet draw read from the tape."""
    alpha = 1 + precision * w
    w_new = np.array([tape.real(), tape.real()])
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
        self.size_prior = int(fx["prior_size"]) if "prior_size" in fx else 0
        self.alpha_global = fx.get("prior_alpha_global")
        self.alpha_fam = fx.get("prior_alpha_fam")

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
                                st.get("pf"), inheritance=self.inheritance)


REJECT = (None, 0.0, -np.inf)


def op_grow(m, st, c, tape):
    zos = st["zos"]
    z = tape.int()
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
    site_new = np.flatnonzero(candidates)[tape.int()]
    new = dict(st, zos=zos.copy())
    new["zos"][site_new] = z
    q = (1 - p) * (1 / np.count_nonzero(~occupied))
    if nb[site_new]:
        q += p * (1 / np.count_nonzero(nb))
    q_back = 1 / (size + 1)
    return new, np.log(q), np.log(q_back)


def op_shrink(m, st, c, tape):
    zos = st["zos"]
    z = tape.int()
    zone = zos == z
    size = int(np.count_nonzero(zone))
    if size <= m.min_size:
        return REJECT
    removal = np.flatnonzero(zone)
    site_removed = removal[tape.int()]
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
    z = tape.int()
    zone = zos == z
    nb = m.neighbours(zone, occupied)
    p = m.p_grow[c]
    connected = tape.real() < p
    candidates = nb if connected else ~occupied
    if not np.any(candidates):
        return REJECT
    site_new = np.flatnonzero(candidates)[tape.int()]
    new = dict(st, zos=zos.copy())
    new["zos"][site_new] = z
    removal = np.flatnonzero(zone)
    site_removed = removal[tape.int()]
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
    f = tape.int()
    new = dict(st, w=st["w"].copy())
    if m.inheritance:
        idx = [tape.int(), tape.int()]
        vals, log_q, log_q_back = _alter_pair(st["w"][f], idx, m.prec[0], tape)
        new["w"][f, idx] = vals
    else:
        vals, log_q, log_q_back = dirichlet_proposal(st["w"][f, :], m.prec[0], tape)
        new["w"][f, :] = vals
    return new, log_q, log_q_back


def _states_pair(m, f, tape):
    return [tape.int(), tape.int()]


def op_p_global(m, st, c, tape):
    f = tape.int()
    idx = _states_pair(m, f, tape)
    new = dict(st, pg=st["pg"].copy())
    vals, log_q, log_q_back = _alter_pair(st["pg"][f], idx, m.prec[1], tape)
    new["pg"][f, idx] = vals
    return new, log_q, log_q_back


def op_p_zones(m, st, c, tape):
    z = tape.int()
    f = tape.int()
    idx = _states_pair(m, f, tape)
    new = dict(st, pz=st["pz"].copy())
    vals, log_q, log_q_back = _alter_pair(st["pz"][z, f], idx, m.prec[2], tape)
    new["pz"][z, f, idx] = vals
    return new, log_q, log_q_back


def op_p_families(m, st, c, tape):
    fam = tape.int()
    f = tape.int()
    idx = _states_pair(m, f, tape)
    new = dict(st, pf=st["pf"].copy())
    vals, log_q, log_q_back = _alter_pair(st["pf"][fam, f], idx, m.prec[3], tape)
    new["pf"][fam, f, idx] = vals
    return new, log_q, log_q_back


OPERATORS = {SHRINK: op_shrink, GROW: op_grow, SWAP: op_swap, WEIGHTS: op_weights,
             P_GLOBAL: op_p_global, P_ZONES: op_p_zones, P_FAMILIES: op_p_families}


def step(m, st, ll, prior, c, tape):
    """MCMCGenerative.step (mcmc_generative.py:282-329).  Returns (state, ll, prior, op,
    accepted)."""
    op = tape.int()
    cand, log_q, log_q_back = OPERATORS[op](m, st, c, tape)
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
    ops, acc, lls, priors, zos = [], [], [], [], []
    for _ in range(steps):
        st, ll, prior, op, a = step(m, st, ll, prior, chain, tape)
        ops.append(op)
        acc.append(a)
        lls.append(ll)
        priors.append(prior)
        zos.append(st["zos"].copy())
    return dict(op=np.array(ops), accept=np.array(acc), ll=np.array(lls), prior=np.array(priors),
                init_prior=init_prior, zos=np.array(zos), state=st, tape_used=tape.pos)
