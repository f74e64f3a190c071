"""Batched drop-ins for the sBayes zone samplers: ``BatchedZoneMCMC`` / ``BatchedZoneMCMCWarmup``.

They take the constructor kwargs of ``ZoneMCMC`` / ``ZoneMCMCWarmup``
(sbayes/sampling/zone_sampling.py:117-178, 1272-1291; built by mcmc_setup.py:103-114, 176-188)
and expose ``generate_samples(n_steps, n_samples, warm_up=False, warm_up_steps=None)`` and the
``statistics`` dict of ``MCMCGenerative`` (sbayes/sampling/mcmc_generative.py:56-71, 149-237).
The step loop runs on the GPU (``sbz_mh_run_device``, one wave per chain, all chains of this
rank in one launch); the host only schedules launches between the points where the reference
logs something:
  * sample logging of chain ``chain_idx[0]`` after step i when ``i % steps_per_sample == 0``
    (:213-218), the screen log every 1000 steps (:225-226) and the last sample at step n-1
    (:229-231);
  * the warm-up progress lines and the best-chain arg-max (:185-200).

Initial samples follow ``generate_initial_sample`` (zone_sampling.py:935-1233) draw for draw: the
zones come from the same python ``random`` calls (``random.sample`` of the free-site set, then
``random.choice`` of a neighbour), so with the same seeded ``random`` source they are identical
to the reference's; weights are uniform and p_* the smoothed MLE.  The MH draws themselves come
from Philox4x32-10 keyed by (seed, global chain id) — results do not depend on the GPU count.

Supported model (checked, NotImplementedError otherwise): SAMPLE_SOURCE = false or true (the
Gibbs operators of mcmc_setup.py:80-87 and source-resampling zone moves, sbz_mh_src.hip); the
priors of
contact_zones_amd/priors.py (zero / uniform terms, 'counts' on universal and inheritance,
'uniform' / 'quadratic' zone size), read from the reference Model's Prior or given as
``priors=``.  MC3 (``mc3=True``) and ``sample_from_prior`` are not part of the batched path.

Multi-GPU: one process per GPU.  With ``torch.distributed`` initialised, chains are sharded
contiguously by rank; the only collectives are the per-operator counter sum at the end of a run,
the warm-up arg-max (value, chain id) and the broadcast of the best sample (``parallel.py``).
"""
import math
import os
import random as _random_module
import time
from collections import defaultdict

import numpy as np

from . import packing
from .priors import PriorSpec
from .sampler import OPS, op_probabilities, precisions

Q_REJECT = 0
Q_BACK_REJECT = -np.inf


class ZoneError(Exception):
    """Raised when a zone cannot be grown (zone_sampling.py:1247-1248)."""


class Sample:
    """The state container of the reference (zone_sampling.py:49-115): zones (Z, N) bool,
    weights (F, C), p_global (1, F, S), p_zones (Z, F, S), p_families (Fam, F, S) or None."""

    def __init__(self, zones, weights, p_global, p_zones, p_families=None, source=None, chain=0):
        self.zones = zones
        self.weights = weights
        self.p_global = p_global
        self.p_zones = p_zones
        self.p_families = p_families
        self.source = source
        self.chain = chain
        self.what_changed = {}

    @classmethod
    def empty_sample(cls):
        s = cls(None, None, None, None, None)
        return s

    def copy(self):
        c = lambda a: None if a is None else np.copy(a)  # noqa: E731
        return Sample(c(self.zones), c(self.weights), c(self.p_global), c(self.p_zones),
                      c(self.p_families), c(self.source), self.chain)


def normalize(x, axis=-1):
    """util.py:1087-1105."""
    return x / np.sum(x, axis=axis, keepdims=True)


def get_max_size_list(start, end, n_total, k_groups):
    """util.py:1182-1199: k_groups equal groups of max sizes in [start, end)."""
    n_per_group = math.ceil(n_total / k_groups)
    max_sizes = np.linspace(start=start, stop=end, num=k_groups, endpoint=False, dtype=int)
    return list(np.repeat(max_sizes, n_per_group))[0:n_total]


def adjacency_csr(adj_mat, n_sites):
    """The network's adjacency (scipy sparse or dense, data['network']['adj_mat']) as sorted CSR
    int32 arrays; the neighbour relation is 'adj.dot(zone) != 0' (util.py:152-155)."""
    import scipy.sparse as sp
    # a copy: csr_matrix of a CSR matrix shares its arrays, and sorting them in place would race
    # with another job's sampler reading the same data (experiment.run_jobs runs jobs in threads)
    a = sp.csr_matrix(adj_mat, copy=True)
    a.eliminate_zeros()
    a.sort_indices()
    if a.shape != (n_sites, n_sites):
        raise ValueError(f"adj_mat: expected ({n_sites}, {n_sites}), got {a.shape}")
    return a.indptr.astype(np.int32), a.indices.astype(np.int32)


GIBBS_OPS = set(OPS[8:])  # the SAMPLE_SOURCE = true operators (mcmc_setup.py:80-87)
ALTER_OPS = {"alter_weights", "alter_p_global", "alter_p_zones", "alter_p_families"}


def check_model(model, operators=()):
    """The operators must belong to the model's mode: the Gibbs operators need SAMPLE_SOURCE =
    true; with sources, parameters move by Gibbs steps only (mcmc_setup.py:80-95)."""
    source = bool(getattr(model, "sample_source", False))
    ops = {k for k, v in dict(operators).items() if v} if operators else set()
    if not source and ops & GIBBS_OPS:
        raise ValueError(f"operators {sorted(ops & GIBBS_OPS)} need SAMPLE_SOURCE = true")
    if source and ops & ALTER_OPS:
        raise ValueError(f"operators {sorted(ops & ALTER_OPS)} are not used with SAMPLE_SOURCE = true")


class InitialSamples:
    """generate_initial_sample (zone_sampling.py:935-1233) on the host, draw for draw."""

    def __init__(self, features, applicable_states, adj_indptr, adj_indices, families, n_zones,
                 initial_size, inheritance, initial_sample, rng, sample_source=False, np_random=None):
        self.features = features
        self.applicable_states = applicable_states
        self.adj_indptr, self.adj_indices = adj_indptr, adj_indices
        self.families = families
        self.n_zones = n_zones
        self.initial_size = initial_size
        self.inheritance = inheritance
        self.initial_sample = initial_sample if initial_sample is not None else Sample.empty_sample()
        self.rng = rng
        self.sample_source = sample_source
        # the initial sources' uniforms: np.random.random (the reference's global stream) or a
        # job's own RandomState(seed).random_sample (the same draws as np.random.seed(seed) then
        # np.random.random, without sharing the global stream with concurrent jobs)
        self.np_random = np_random
        self.n_sites, self.n_features = features.shape[:2]

    def neighbours(self, zone, already_in_zone):
        """get_neighbours (util.py:139-155)."""
        nb = np.zeros(self.n_sites, bool)
        for s in np.flatnonzero(zone):
            nb[self.adj_indices[self.adj_indptr[s]:self.adj_indptr[s + 1]]] = True
        return nb & ~already_in_zone

    def grow_zone_of_size_k(self, k, already_in_zone):
        """zone_sampling.py:988-1028; like the reference it marks sites in `already_in_zone` in
        place, also when it then fails."""
        zone = np.zeros(self.n_sites, bool)
        sites_occupied = np.nonzero(already_in_zone)[0]
        sites_free = set(range(self.n_sites)) - set(sites_occupied)
        try:
            # random.sample(set, 1): Python <= 3.10 samples tuple(set) (the reference's call)
            i = self.rng.sample(tuple(sites_free), 1)[0]
            zone[i] = already_in_zone[i] = 1
        except ValueError:
            raise ZoneError
        for _ in range(k - 1):
            nb = self.neighbours(zone, already_in_zone)
            if not np.any(nb):
                raise ZoneError
            site_new = self.rng.choice(nb.nonzero()[0])
            zone[site_new] = already_in_zone[site_new] = 1
        return zone, already_in_zone

    def zones(self):
        """generate_initial_zones (zone_sampling.py:935-986)."""
        if self.n_zones == 0:
            return np.zeros((self.n_zones, self.n_sites), bool)
        occupied = np.zeros(self.n_sites, bool)
        initial_zones = np.zeros((self.n_zones, self.n_sites), bool)
        n_generated = 0
        if self.initial_sample.zones is not None:
            for i in range(len(self.initial_sample.zones)):
                initial_zones[i, :] = self.initial_sample.zones[i]
                occupied += self.initial_sample.zones[i]
                n_generated += 1
        not_initialized = range(n_generated, self.n_zones)
        attempts = 0
        max_attempts = 1000
        while True:
            for i in not_initialized:
                try:
                    g = self.grow_zone_of_size_k(self.initial_size, occupied)
                except ZoneError:
                    if attempts < max_attempts:
                        attempts += 1
                        not_initialized = range(n_generated, self.n_zones)
                        break
                    raise ValueError("Failed to add additional area. Try fewer areas"
                                     "or set initial_sample to None")
                n_generated += 1
                initial_zones[i, :] = g[0]
                occupied = g[1]
            if n_generated == self.n_zones:
                return initial_zones

    def weights(self):
        """zone_sampling.py:1030-1052."""
        if self.initial_sample.weights is not None:
            w = self.initial_sample.weights
        else:
            w = np.full((self.n_features, 3 if self.inheritance else 2), 1.)
        return normalize(w)

    def _smoothed_mle(self, idx):
        sites_per_state = np.nansum(self.features[idx, :, :], axis=0)
        sites_per_state[np.isnan(sites_per_state)] = 0
        sites_per_state[self.applicable_states] += 1
        return sites_per_state / np.sum(sites_per_state, axis=1)[:, np.newaxis]

    def p_global(self):
        """zone_sampling.py:1054-1085."""
        p = np.zeros((1, self.n_features, self.features.shape[2]))
        if self.initial_sample.p_global is not None:
            return self.initial_sample.p_global
        sites_per_state = np.count_nonzero(self.features, axis=0)
        sites_per_state[np.isnan(sites_per_state)] = 0
        sites_per_state[self.applicable_states] += 1
        p[0, :, :] = sites_per_state / np.sum(sites_per_state, axis=1, keepdims=True)
        return p

    def p_zones(self, initial_zones):
        """zone_sampling.py:1105-1147."""
        p = np.zeros((self.n_zones, self.n_features, self.features.shape[2]))
        n_generated = 0
        if self.initial_sample.p_zones is not None:
            for i in range(len(self.initial_sample.p_zones)):
                p[i, :] = self.initial_sample.p_zones[i]
                n_generated += 1
        for i in range(n_generated, self.n_zones):
            p[i, :, :] = self._smoothed_mle(initial_zones[i].nonzero()[0])
        return p

    def p_families(self):
        """zone_sampling.py:1149-1187."""
        p = np.zeros((self.families.shape[0], self.n_features, self.features.shape[2]))
        if self.initial_sample.p_families is not None:
            for i in range(len(self.initial_sample.p_families)):
                p[i, :] = self.initial_sample.p_families[i]
        else:
            for fam in range(len(self.families)):
                p[fam, :, :] = self._smoothed_mle(self.families[fam].nonzero()[0])
        return p

    def __call__(self, c=0):
        """generate_initial_sample (zone_sampling.py:1189-1233); with SAMPLE_SOURCE = true the
        sources get one Gibbs draw from np.random (:1227-1231, contact_zones_amd/sources.py)."""
        zones = self.zones()
        weights = self.weights()
        p_global = self.p_global()
        p_zones = self.p_zones(zones)
        p_families = self.p_families() if self.inheritance else None
        sample = Sample(zones=zones, weights=weights, p_global=p_global, p_zones=p_zones,
                        p_families=p_families, chain=c)
        if self.sample_source:
            from .sources import draw_sources, source_posterior
            if not hasattr(self, "_obs"):
                self._obs = packing.features_to_obs(self.features)
                self._fam = packing.families_to_fam_of_site(
                    self.families if self.inheritance and self.families.shape[0] else None, self.n_sites)
            zos = packing.zones_to_zone_of_site(zones, self.n_sites)
            post = source_posterior(self._obs, self._fam, zos, np.asarray(weights, np.float64),
                                    np.asarray(p_global, np.float64)[0], p_zones, p_families,
                                    self.inheritance)
            draws = draw_sources(post) if self.np_random is None else draw_sources(post, self.np_random)
            sample.source = packing.index_to_source(draws, 3 if self.inheritance else 2)
        return sample


def _dist():
    try:
        import torch.distributed as dist
    except ImportError:  # pragma: no cover
        return None
    return dist if dist.is_available() and dist.is_initialized() else None


class BatchedZoneMCMC:
    """ZoneMCMC (zone_sampling.py:117) with every chain of this rank stepping on the GPU."""

    IS_WARMUP = False
    Q_REJECT = Q_REJECT
    Q_BACK_REJECT = Q_BACK_REJECT
    ZoneError = ZoneError

    def __init__(self, model, data, operators, n_chains, var_proposal, p_grow_connected,
                 initial_size, initial_sample=None, mc3=False, swap_period=None, chain_swaps=None,
                 sample_from_prior=False, show_screen_log=False, logger=None, *, seed=None,
                 rng=None, device=None, group=None, refresh_every_launch=True, priors=None,
                 gibbs_counts=None, log_all_chains=False, chain_params=None, log_window=None,
                 np_random=None, **kwargs):
        if mc3:
            raise NotImplementedError("MC3 chain swaps are not part of the batched sampler")
        if sample_from_prior:
            raise NotImplementedError("sample_from_prior is not supported by the batched sampler")
        check_model(model, operators)
        self.model, self.data = model, data
        self.sample_source = bool(getattr(model, "sample_source", False))
        self.n_chains = int(n_chains)
        self.chain_idx = list(range(self.n_chains))
        self.rng = rng if rng is not None else _random_module  # the reference's `_random`
        self.seed = seed
        self.show_screen_log = show_screen_log
        if logger is None:
            import logging
            logger = logging.getLogger()
        self.logger = logger

        self.features = np.asarray(data.features).astype(bool)
        self.applicable_states = np.asarray(data.states, bool)
        self.n_sites, self.n_features, self.n_states = self.features.shape
        self.adj_indptr, self.adj_indices = adjacency_csr(data.network["adj_mat"], self.n_sites)
        self.inheritance = bool(model.inheritance)
        fams = getattr(data, "families", None)
        self.families = (np.asarray(fams, bool) if self.inheritance and fams is not None
                         else np.zeros((0, self.n_sites), bool))
        self.n_families = self.families.shape[0] if self.inheritance else None
        self.n_sources = 3 if self.inheritance else 2
        self.n_zones = int(model.n_zones)
        self.min_size = int(model.min_size)
        self.max_size = model.max_size
        self.initial_size = initial_size
        self.initial_sample = initial_sample if initial_sample is not None else Sample.empty_sample()
        self.p_grow_connected = p_grow_connected
        self.var_proposal = var_proposal
        self.operators = dict(operators)
        self.p_operators = op_probabilities(self.operators)
        self.fn_operators = [k for k in self.operators]
        self.precision = precisions(var_proposal)
        self.refresh_every_launch = refresh_every_launch
        # the prior terms of the MH ratio: from the reference Model's Prior (model.py:455-505)
        # unless given; unsupported prior types raise NotImplementedError
        self.priors = priors if priors is not None else PriorSpec.from_model(model, self.applicable_states)
        # pseudo-counts of the source-mode Gibbs operators (prior.prior_p_global.counts,
        # prior.prior_p_families.counts: zone_sampling.py:344, 394)
        if gibbs_counts is None and self.sample_source:
            pr = getattr(model, "prior", None)
            cg = getattr(getattr(pr, "prior_p_global", None), "counts", None)
            cf = getattr(getattr(pr, "prior_p_families", None), "counts", None) if self.inheritance else None
            gibbs_counts = (cg, cf)
        self.gibbs_counts = gibbs_counts

        self.statistics = {'sample_id': [], 'sample_likelihood': [], 'sample_prior': [],
                           'sample_zones': [], 'sample_weights': [], 'sample_p_global': [],
                           'sample_p_zones': [], 'sample_p_families': [], 'last_sample': [],
                           'acceptance_ratio': math.nan, 'accepted_steps': 0, 'n_swaps': 0,
                           'accepted_swaps': 0, 'swap_ratio': [],
                           'accept_operator': defaultdict(int), 'reject_operator': defaultdict(int)}
        # independent-chains runs (the runner's --chains): every chain's samples are logged too, in
        # windows gathered to rank 0 as the run goes (ChainLog -> chain_statistics): zones, ll and
        # prior of every chain; the parameters of chain 0 (the logged chain, `statistics`) and of
        # the chains in `chain_params` ("all" or global chain ids)
        self.log_all_chains = bool(log_all_chains)
        self.chain_params = chain_params
        self.log_window = log_window
        self.chain_statistics = None
        self._chain_log = None
        self._ll = np.full(self.n_chains, -np.inf)
        self._prior = np.full(self.n_chains, -np.inf)
        self.t_start = time.time()

        self._group = group
        d = _dist()
        self.rank = d.get_rank(group) if d else 0
        self.world_size = d.get_world_size(group) if d else 1
        from .parallel import shard_range
        self.lo, self.hi = shard_range(self.n_chains, self.rank, self.world_size)
        self._device = device
        self._engine = self._sampler = self._state = None
        self._tape = None  # (tape [n_chains, L], tape_len [n_chains]): replay instead of Philox

        self._init = InitialSamples(self.features, self.applicable_states, self.adj_indptr,
                                    self.adj_indices, self.families, self.n_zones,
                                    self.initial_size, self.inheritance, self.initial_sample,
                                    self.rng, sample_source=self.sample_source, np_random=np_random)

    # ---- reference API ---------------------------------------------------------------
    def generate_initial_sample(self, c=0):
        return self._init(c)

    def get_operators(self, operators):
        return list(operators.keys()), list(operators.values())

    def prior(self, sample, chain):
        """Log prior of `sample` (Prior.__call__, model.py:484-505, for the supported types)."""
        zos, w, pg, pz, pf, _ = self._pack(sample)
        return float(self.priors.log_prior(zos[None], pg[None], None if pf is None else pf[None],
                                           self.applicable_states, self.n_zones,
                                           self.inheritance)[0])

    def likelihood(self, sample, chain):
        """Full log-likelihood of `sample` on the GPU (MCMCGenerative.likelihood, :106-127)."""
        zos, w, pg, pz, pf, src = self._pack(sample)
        eng = self._get_engine()
        return float(eng.loglik(zos[None], w[None], pg[None], pz[None],
                                None if pf is None else pf[None],
                                None if src is None else src[None])[0])

    # ---- device plumbing ---------------------------------------------------------------
    def _get_engine(self):
        if self._engine is None:
            import torch
            from .likelihood import LikelihoodEngine
            from .sampler import Sampler
            dev = self._device
            if dev is None:
                # under torchrun each rank owns GPU LOCAL_RANK (one process per GPU), whether or
                # not the caller bound it with torch.cuda.set_device
                lr = os.environ.get("LOCAL_RANK")
                dev = (int(lr) % torch.cuda.device_count() if _dist() is not None and lr is not None
                       else torch.cuda.current_device())
            dev = int(dev)
            self._device = dev
            obs = packing.features_to_obs(self.features)
            fam = packing.families_to_fam_of_site(self.families if self.inheritance and
                                                  self.families.shape[0] else None, self.n_sites)
            self._engine = LikelihoodEngine(obs, fam, self.n_states, self.n_zones,
                                            self.families.shape[0] if self.inheritance else 0,
                                            self.inheritance, device=dev)
            self._sampler = Sampler(self._engine, self.applicable_states, self.adj_indptr,
                                    self.adj_indices, self.p_operators, self.precision,
                                    self.min_size, warmup=self.IS_WARMUP, priors=self.priors,
                                    sample_source=self.sample_source,
                                    gibbs_counts=self.gibbs_counts)
        return self._engine

    def _pack(self, s):
        zos = packing.zones_to_zone_of_site(np.asarray(s.zones, bool), self.n_sites)
        pg = np.asarray(s.p_global, np.float64)
        pg = pg[0] if pg.ndim == 3 else pg
        pf = np.asarray(s.p_families, np.float64) if self.inheritance else None
        src = (packing.source_to_index(s.source) if self.sample_source and s.source is not None
               else None)
        return zos, np.asarray(s.weights, np.float64), pg, np.asarray(s.p_zones, np.float64), pf, src

    def _unpack(self, st, i, c):
        """Chain i of this rank's device state -> Sample (host copies)."""
        zos = st.zone_of_site[i].cpu().numpy()
        zones = packing.index_to_groups(zos, self.n_zones)
        return Sample(zones=zones, weights=st.w[i].cpu().numpy(),
                      p_global=st.p_global[i].cpu().numpy()[None],
                      p_zones=st.p_zones[i].cpu().numpy(),
                      p_families=st.p_fam[i].cpu().numpy() if st.p_fam is not None else None,
                      source=(packing.index_to_source(st.source_of(i).cpu().numpy(), self.n_sources)
                              if st.source_pm is not None else None),
                      chain=c)

    def _max_size_for(self, lo, hi):
        ms = self.max_size
        return np.asarray(ms[lo:hi] if isinstance(ms, (list, tuple, np.ndarray)) else [ms] * (hi - lo))

    def _p_grow_for(self, lo, hi):
        p = self.p_grow_connected
        return np.asarray(p[lo:hi] if isinstance(p, (list, tuple, np.ndarray)) else [p] * (hi - lo),
                          np.float64)

    def _start(self):
        """Initial samples of every chain (the reference's draw order), this rank's shard on the
        device, the Philox seed agreed across ranks."""
        from .parallel import broadcast_seed
        from .sampler import ChainState
        samples = [self.generate_initial_sample(c) for c in self.chain_idx]
        seed = self.seed if self.seed is not None else self.rng.getrandbits(63)
        self._philox_seed = broadcast_seed(int(seed), self._group)
        self._tape_pos = None
        self._alias = None
        self._alias_logged = []  # logged samples whose p_* still alias chain 0's (source mode)
        if self.hi == self.lo:
            # more ranks than chains: this rank holds no chain but joins every collective
            self._state = None
            self._sync_host_ll()
            return samples
        eng = self._get_engine()
        mine = samples[self.lo:self.hi]
        packed = [self._pack(s) for s in mine]
        stack = lambda k: np.stack([p[k] for p in packed]) if packed else None  # noqa: E731
        pf = stack(4) if self.inheritance else None
        prior0 = self.priors.log_prior(stack(0), stack(2), pf, self.applicable_states,
                                       self.n_zones, self.inheritance)
        self._state = ChainState(eng, stack(0), stack(1), stack(2), stack(3), pf, prior=prior0,
                                 source=stack(5) if self.sample_source else None)
        self._acc0 = self._state.accepted.clone()
        self._prop0 = self._state.proposed.clone()
        if self.sample_source and self.lo == 0 and self.hi > 0:
            import torch
            st = self._state
            z = torch.zeros_like
            self._alias = (torch.zeros(st.B, dtype=torch.int32, device=st.ll.device), z(st.p_global),
                           z(st.p_zones), z(st.p_fam) if st.p_fam is not None else None)
        if self._tape is not None:
            import torch
            self._tape_pos = torch.zeros(self.hi - self.lo, dtype=torch.int64,
                                         device=self._state.ll.device)
        self._sync_host_ll()
        return samples

    def _sync_host_ll(self):
        if self._state is None:
            self._ll[:] = -np.inf
            self._prior[:] = -np.inf
            return
        ll = self._state.ll.cpu().numpy()
        self._ll[:] = -np.inf
        self._ll[self.lo:self.hi] = ll
        self._prior[:] = -np.inf
        self._prior[self.lo:self.hi] = self._state.prior.cpu().numpy()

    def _advance(self, n):
        """n MH steps on every chain of this rank (one launch)."""
        if n <= 0 or self._state is None:
            return
        st = self._state
        kw = {}
        if self._tape is not None:
            tape, tape_len = self._tape
            kw = dict(tape=tape[self.lo:self.hi], tape_len=tape_len[self.lo:self.hi],
                      tape_pos=self._tape_pos)
        out = self._sampler.run(st, n, self._max_size_for(self.lo, self.hi),
                                self._p_grow_for(self.lo, self.hi), seed=self._philox_seed,
                                chain_id0=self.lo, alias=self._alias, **kw)
        status = out["status"].cpu().numpy()
        if self._alias_logged and int(self._alias[0][0].item()) == 0:
            a = self._alias
            self._resolve_alias(a[1][0], a[2][0], a[3][0] if a[3] is not None else None)
        if np.any(status != 0):
            bad = int(np.flatnonzero(status)[0])
            raise RuntimeError(f"sampler: chain {self.lo + bad} stopped with status {status[bad]}")
        if self.refresh_every_launch:
            st.refresh_ll()  # reset the incremental ll to a full evaluation
        self._sync_host_ll()

    def _resolve_alias(self, pg, pz, pf):
        """Give the logged samples still aliasing chain 0's arrays the values those arrays had
        when the reference's Sample was replaced (sbz.h: alias_pending)."""
        stt = self.statistics
        pg, pz = pg.cpu().numpy(), pz.cpu().numpy()
        pf = pf.cpu().numpy() if pf is not None else None
        for k in self._alias_logged:
            stt['sample_p_global'][k][0] = pg
            stt['sample_p_zones'][k][...] = pz
            if pf is not None:
                stt['sample_p_families'][k][...] = pf
        self._alias_logged = []

    def _operator_counts(self):
        from .parallel import all_reduce_sum
        import torch
        if self._state is None:
            from .sampler import N_OPS_MAX
            t = torch.zeros((2, N_OPS_MAX), dtype=torch.int64)
        else:
            acc = (self._state.accepted - self._acc0).sum(0)
            prop = (self._state.proposed - self._prop0).sum(0)
            t = torch.stack([acc, prop]).to(torch.int64)
        t = all_reduce_sum(t, self._group)
        return t[0].cpu().numpy(), t[1].cpu().numpy()

    def _chain0_sample(self):
        """Sample of chain_idx[0] (global chain 0, on rank 0) — rank 0 only."""
        return self._unpack(self._state, 0, 0) if self.rank == 0 else None

    def log_sample_statistics(self, sample, c, sample_id):
        """mcmc_generative.py:353-372."""
        self.statistics['sample_id'].append(sample_id)
        self.statistics['sample_zones'].append(sample.zones)
        self.statistics['sample_weights'].append(sample.weights)
        self.statistics['sample_p_global'].append(sample.p_global)
        self.statistics['sample_p_zones'].append(sample.p_zones)
        self.statistics['sample_p_families'].append(sample.p_families)
        self.statistics['sample_likelihood'].append(self._ll[c])
        self.statistics['sample_prior'].append(self._prior[c])
        if self.show_screen_log:
            print('Log-likelihood: %.2f' % self._ll[c])
            print('Accepted steps: %i' % self.statistics['accepted_steps'])

    def log_last_sample(self, last_sample):
        self.statistics['last_sample'] = last_sample

    def print_screen_log(self, i_step):
        """mcmc_generative.py:380-389 (the log-likelihood of chain_idx[0])."""
        i_step_str = str.ljust(str(i_step), 12)
        likelihood_str = str.ljust('log-likelihood:  %.2f' % self._ll[self.chain_idx[0]], 36)
        time_per_million = (time.time() - self.t_start) / (i_step + 1) * 1000000
        print(i_step_str + likelihood_str + '%i seconds / million steps' % time_per_million)

    # ---- the sampling loop -----------------------------------------------------------------
    def generate_samples(self, n_steps, n_samples, warm_up=False, warm_up_steps=None):
        """mcmc_generative.py:149-237 with the chains batched on the GPU."""
        self._start()
        if warm_up:
            print("Tuning parameters in warm-up...")
            marks = [i for i in range(warm_up_steps) if (i / warm_up_steps) * 100 % 10 == 0]
            done = 0
            for i in marks:
                self._advance(i - done)
                done = i
                print("warm-up", int((i / warm_up_steps) * 100), "%")
            self._advance(warm_up_steps - done)
            self._count_operators()
            return self._best_sample()

        print("Sampling from posterior...")
        steps_per_sample = int(np.ceil(n_steps / n_samples))
        t_start = time.time()
        # steps after which something is logged (i_step = step index, 0-based)
        events = set(range(0, n_steps, steps_per_sample))
        events |= set(range(999, n_steps, 1000))
        if n_steps - 1 == 0:
            raise ZeroDivisionError("integer division or modulo by zero "
                                    "(the reference's last-sample test divides by n_steps - 1)")
        events.add(n_steps - 1)
        done = 0  # steps taken so far
        if self.log_all_chains:
            self._chain_log = ChainLog(self, len(range(0, n_steps, steps_per_sample)), self.chain_params,
                                       self.log_window)
        for i_step in sorted(events):
            self._advance(i_step + 1 - done)
            done = i_step + 1
            if i_step % steps_per_sample == 0:
                if self.log_all_chains:
                    self._chain_log.snap(int(i_step / steps_per_sample))
                s0 = self._chain0_sample()
                if self.rank == 0:
                    # the logged sample's prior evaluated in full (the carried value differs by
                    # rounding only): the reference logs Prior.__call__ of the sample
                    self._prior[self.chain_idx[0]] = self.prior(s0, self.chain_idx[0])
                    self.log_sample_statistics(s0, c=self.chain_idx[0],
                                               sample_id=int(i_step / steps_per_sample))
                    if self._alias is not None:
                        # the reference logs references to the Sample's arrays, which its Gibbs
                        # operators keep changing in place (zone_sampling.py:333-400)
                        self._alias_logged.append(len(self.statistics['sample_id']) - 1)
                        self._alias[0][0] = 1
            if (i_step + 1) % 1000 == 0 and self.rank == 0:
                self.print_screen_log(i_step + 1)
            if i_step % (n_steps - 1) == 0 and i_step != 0 and self.rank == 0:
                self.log_last_sample(self._chain0_sample())
        if self._alias_logged:  # still aliased at the end: the final arrays
            st = self._state
            self._resolve_alias(st.p_global[0], st.p_zones[0],
                                st.p_fam[0] if st.p_fam is not None else None)
        if self.log_all_chains:
            self.chain_statistics = self._chain_log.finish()
            self._chain_log = None
        t_end = time.time()
        self._count_operators()
        self.statistics['sampling_time'] = t_end - t_start
        self.statistics['time_per_sample'] = (t_end - t_start) / n_samples
        self.statistics['acceptance_ratio'] = self.statistics['accepted_steps'] / n_steps
        self.statistics['swap_ratio'] = 0
        return None

    def _count_operators(self):
        acc, prop = self._operator_counts()
        for i, name in enumerate(OPS):
            if name in self.operators:
                self.statistics['accept_operator'][name] += int(acc[i])
                self.statistics['reject_operator'][name] += int(prop[i] - acc[i])
        self.statistics['accepted_steps'] += int(acc.sum())

    def _best_sample(self):
        """Arg-max of ll + prior over all chains of all ranks (first index on ties, as
        list.index(max(...)), mcmc_generative.py:195-200); the winner's Sample on every rank."""
        from .parallel import best_chain, broadcast_arrays
        post = self._ll[self.lo:self.hi] + self._prior[self.lo:self.hi]
        best, _ = best_chain(post, self.lo, self._group)
        owner = None
        arrays = None
        if self.lo <= best < self.hi:
            s = self._unpack(self._state, best - self.lo, best)
            arrays = [s.zones, s.weights, s.p_global, s.p_zones] + \
                     ([s.p_families] if self.inheritance else []) + \
                     ([s.source] if self.sample_source else [])
        from .parallel import owner_of
        owner = owner_of(best, self.n_chains, self.world_size)
        arrays = broadcast_arrays(arrays, owner, self._group)
        k = 4 + int(self.inheritance)
        return Sample(zones=arrays[0], weights=arrays[1], p_global=arrays[2], p_zones=arrays[3],
                      p_families=arrays[4] if self.inheritance else None,
                      source=arrays[k] if self.sample_source else None, chain=best)


class ChainLog:
    """The logged samples of every chain of an independent-chains run (BatchedZoneMCMC with
    log_all_chains), streamed to rank 0 in windows (mcmc_generative.py:205-218 logs one chain;
    util.py:846-907 writes it).

    Each logging point copies, on the device, this rank's chains' zone assignments (u8 [N]), carried
    log-likelihood and carried log prior into slot j of a window of W samples; the parameters
    (w, p_global, p_zones, p_families) only of the chains in `params` ("all", or global chain ids;
    chain 0's are logged by the reference path itself).  A full window is gathered to rank 0 (one
    gather per array, parallel.gather_to_root: RCCL over xGMI with nccl), copied through a pinned
    host buffer into rank 0's host arrays, and the slot counter starts again: device memory is
    O(W), never O(N_SAMPLES), and no rank but 0 ever holds other ranks' samples.

    Bytes: per rank and window B (N + 16) W for every chain, plus P (8 F (C + S (1 + Z + Fam))) W
    for P parameter chains; rank 0's gather output is the same times the ranks; rank 0's host
    arrays n_chains n_log (N + 16) (+ n_log x the parameter bytes per parameter chain).  At the
    north-star run (2048 chains over 8 GPUs, N = 2000, cfg5 parameters 534 KB, 1000 samples,
    W = 64, no parameter chains but chain 0): 33 MB of window per rank, 264 MB of gather output on
    rank 0, 4.1 GB of host arrays on rank 0."""

    WINDOW_BYTES = 256 << 20  # default window: as many samples as fit this per rank (at most 64)

    def __init__(self, smp, n_log, params=None, window=None):
        import torch
        self.smp = smp
        self.n_log = int(n_log)
        n, lo, hi = smp.n_chains, smp.lo, smp.hi
        B = hi - lo
        N, F, S, Z = smp.n_sites, smp.n_features, smp.n_states, smp.n_zones
        self.C = 3 if smp.inheritance else 2
        self.Fam = smp.n_families if smp.inheritance else 0
        if params == "all":
            pc = list(range(1, n))
        else:
            pc = sorted({int(c) for c in (params or []) if 0 < int(c) < n})
        self.pc = pc                                        # global ids with parameters (chain 0 aside)
        self.pc_local = [c - lo for c in pc if lo <= c < hi]
        from .parallel import shard_range
        w = smp.world_size
        self.pc_sizes = [sum(1 for c in pc if shard_range(n, r, w)[0] <= c < shard_range(n, r, w)[1])
                         for r in range(w)]
        st = smp._state
        self.dev = st.ll.device if st is not None else torch.device("cpu")
        pbytes = 8 * F * (self.C + S * (1 + Z + self.Fam))
        per_sample = max(1, B * (N + 16) + max(self.pc_sizes) * pbytes)
        W = int(window) if window else max(1, min(64, self.WINDOW_BYTES // per_sample))
        self.W = max(1, min(W, max(self.n_log, 1)))
        W = self.W
        self.buf = {"zos": torch.empty((B, W, N), dtype=torch.uint8, device=self.dev),
                    "ll": torch.empty((B, W), dtype=torch.float64, device=self.dev),
                    "prior": torch.empty((B, W), dtype=torch.float64, device=self.dev)}
        self.pshape = {"w": (F, self.C), "pg": (F, S), "pz": (Z, F, S)}
        if self.Fam:
            self.pshape["pf"] = (self.Fam, F, S)
        P = len(self.pc_local)
        self.pbuf = {k: torch.empty((P, W) + shp, dtype=torch.float64, device=self.dev)
                     for k, shp in self.pshape.items()} if pc else {}
        self.j = 0          # filled slots of the window
        self.done = 0       # samples already on rank 0
        self.ids = []
        self.host = None
        if smp.rank == 0:
            self.host = {"zos": np.empty((n, self.n_log, N), np.uint8),
                         "ll": np.empty((n, self.n_log)), "prior": np.empty((n, self.n_log))}
            self.phost = {k: np.empty((len(pc), self.n_log) + shp) for k, shp in self.pshape.items()}
            self.pin = None

    def window_bytes(self):
        """Device bytes of this rank's window buffers."""
        return sum(t.numel() * t.element_size() for t in list(self.buf.values()) + list(self.pbuf.values()))

    def snap(self, sample_id):
        """Log this rank's chains at a logging point (device copies into the window)."""
        st, j = self.smp._state, self.j
        if st is not None:
            self.buf["zos"][:, j].copy_(st.zone_of_site)
            self.buf["ll"][:, j].copy_(st.ll)
            self.buf["prior"][:, j].copy_(st.prior)
            if self.pc_local:
                idx = self.pc_local
                self.pbuf["w"][:, j].copy_(st.w[idx])
                self.pbuf["pg"][:, j].copy_(st.p_global[idx])
                self.pbuf["pz"][:, j].copy_(st.p_zones[idx])
                if "pf" in self.pbuf:
                    self.pbuf["pf"][:, j].copy_(st.p_fam[idx])
        self.ids.append(int(sample_id))
        self.j += 1
        if self.j == self.W:
            self.flush()

    def _to_host(self, t, out):
        """Rank 0: a gathered window (device or host tensor) into the host array slice `out`
        (through a pinned staging buffer when it is on the GPU)."""
        import torch
        if t.device.type == "cpu":
            out[...] = t.numpy()
            return
        nb = t.numel() * t.element_size()
        if self.pin is None or self.pin.numel() < nb:
            self.pin = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
        stage = self.pin[:nb].view(t.dtype).view(t.shape)
        stage.copy_(t)
        out[...] = stage.numpy()

    def flush(self):
        """Gather the filled slots of the window to rank 0 and append them to its host arrays."""
        from .parallel import gather_to_root
        n = self.j
        if n == 0:
            return
        smp, s0 = self.smp, self.done
        for k in ("zos", "ll", "prior"):
            full = gather_to_root(self.buf[k][:, :n].contiguous(), smp.n_chains, smp._group)
            if smp.rank == 0:
                self._to_host(full, self.host[k][:, s0:s0 + n])
        for k in self.pbuf:
            full = gather_to_root(self.pbuf[k][:, :n].contiguous(), len(self.pc), smp._group, sizes=self.pc_sizes)
            if smp.rank == 0:
                self._to_host(full, self.phost[k][:, s0:s0 + n])
        self.done += n
        self.j = 0

    def finish(self):
        """The last window; on rank 0 one statistics dict per global chain (chain 0: the logged
        chain's `statistics` itself), None on the other ranks.  Chains without parameters log
        sample_id, sample_likelihood, sample_prior (the carried log prior) and sample_zones; chains
        with parameters also the parameter samples and the prior evaluated in full on the host (as
        the logged chain's)."""
        self.flush()
        smp = self.smp
        if smp.rank != 0:
            return None
        h, Z = self.host, smp.n_zones
        m = self.done
        out = [smp.statistics]
        pidx = {c: i for i, c in enumerate(self.pc)}
        for c in range(1, smp.n_chains):
            zos = h["zos"][c, :m]
            st = {'sample_id': list(self.ids[:m]), 'sample_likelihood': [float(v) for v in h["ll"][c, :m]],
                  'sample_zones': [packing.index_to_groups(z, Z) for z in zos], 'last_sample': [], 'chain': c}
            if c in pidx:
                i = pidx[c]
                pg, pf = self.phost["pg"][i, :m], self.phost["pf"][i, :m] if self.Fam else None
                prior = smp.priors.log_prior(zos, pg, pf, smp.applicable_states, Z, smp.inheritance) if m else []
                st.update({'sample_prior': [float(v) for v in prior],
                           'sample_weights': list(self.phost["w"][i, :m]),
                           'sample_p_global': [p[None] for p in pg],
                           'sample_p_zones': list(self.phost["pz"][i, :m]),
                           'sample_p_families': list(pf) if pf is not None else [None] * m})
            else:
                st['sample_prior'] = [float(v) for v in h["prior"][c, :m]]
            out.append(st)
        return out


class BatchedZoneMCMCWarmup(BatchedZoneMCMC):
    """ZoneMCMCWarmup (zone_sampling.py:1272-1291): per-chain max_size and p_grow_connected."""

    IS_WARMUP = True

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.max_size = get_max_size_list(start=(self.initial_size + self.max_size) / 4,
                                          end=self.max_size, n_total=self.n_chains, k_groups=4)
        self.p_grow_connected = self.rng.choices(population=[0.95, self.p_grow_connected],
                                                 k=self.n_chains)
