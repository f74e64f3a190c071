"""Batched Metropolis-Hastings on the GPU (sbz_mh_run_device) — the sampler side of the hot path.

``Sampler`` runs many independent chains of the sBayes zone model on one MI355X: each chain is
one wave that executes ``MCMCGenerative.step`` (sbayes/sampling/mcmc_generative.py:282-351)
with the ZoneMCMC / ZoneMCMCWarmup operators (sbayes/sampling/zone_sampling.py:408-933,
1272-1577) for n steps per launch.  Chain state stays resident in HBM (torch tensors);
``ChainState`` holds it.  Draws come from Philox (production) or from a replay tape of the
reference's own decisions (parity tests).

Supported models: SAMPLE_SOURCE = false (sbz_mh.hip) and true (sbz_mh_src.hip, ``sample_source=True``:
Gibbs operators, source-resampling zone moves); zero (uniform) priors, 'counts' priors on
p_global / p_families and 'uniform' / 'quadratic' zone-size priors (contact_zones_amd/priors.py).  Operator names and their canonical order follow
``include/sbz.h`` (sbz_op).
"""
import ctypes

import numpy as np

from ._lib import SBZ_SOURCE_BY_POSITION, check, sbz_chains, sbz_mh_config, sbz_state, sbz_tape, sbz_trace

OPS = ["shrink_zone", "grow_zone", "swap_zone", "alter_weights", "alter_p_global",
       "alter_p_zones", "alter_p_families", "gibbsish_sample_zones",
       # SAMPLE_SOURCE = true operators (mcmc_setup.py:80-87)
       "gibbs_sample_sources", "gibbs_sample_weights", "gibbs_sample_p_global",
       "gibbs_sample_p_zones", "gibbs_sample_p_families"]
N_OPS_MAX = 16  # sbz_mh_config.op_prob / per-chain counter width


def _torch():
    import torch
    return torch


def op_probabilities(operators):
    """Operator weights (dict name -> weight, as MCMC.steps_per_operator builds them,
    mcmc_setup.py:70-95) -> float64[N_OPS_MAX] in canonical order."""
    p = np.zeros(N_OPS_MAX)
    for name, v in operators.items():
        if name not in OPS:
            raise ValueError(f"unknown operator {name!r} (sampler supports {OPS})")
        p[OPS.index(name)] = float(v)
    return p


def precisions(var_proposal):
    """PROPOSAL_PRECISION dict (weights, universal, contact, inheritance) -> float64[4]."""
    if isinstance(var_proposal, dict):
        inh = var_proposal.get("inheritance")
        return np.array([var_proposal["weights"], var_proposal["universal"],
                         var_proposal["contact"], 0.0 if inh is None else inh], np.float64)
    return np.asarray(var_proposal, np.float64)


class ChainState:
    """Device-resident state of B chains (torch tensors on the engine's GPU)."""

    def __init__(self, engine, zone_of_site, w, p_global, p_zones, p_fam=None, prior=None,
                 source=None):
        torch = _torch()
        dev = torch.device("cuda", engine.device)
        self.engine = engine
        f64 = torch.float64
        self.zone_of_site = torch.as_tensor(np.ascontiguousarray(zone_of_site, np.uint8), device=dev)
        self.B = int(self.zone_of_site.shape[0])
        self.w = torch.as_tensor(np.ascontiguousarray(w, np.float64), device=dev, dtype=f64)
        self.p_global = torch.as_tensor(np.ascontiguousarray(p_global, np.float64), device=dev, dtype=f64)
        self.p_zones = torch.as_tensor(np.ascontiguousarray(p_zones, np.float64), device=dev, dtype=f64)
        self.p_fam = (torch.as_tensor(np.ascontiguousarray(p_fam, np.float64), device=dev, dtype=f64)
                      if engine.inheritance else None)
        engine._check_shapes(self.B, self.zone_of_site, self.w, self.p_global, self.p_zones,
                             self.p_fam, None)
        self.ll = torch.empty(self.B, dtype=f64, device=dev)
        # log prior of each chain (carried by the sampler; 0 when every prior term is zero)
        self.prior = (torch.zeros(self.B, dtype=f64, device=dev) if prior is None else
                      torch.as_tensor(np.broadcast_to(np.asarray(prior, np.float64), (self.B,)).copy(),
                                      device=dev))
        self.accepted = torch.zeros((self.B, N_OPS_MAX), dtype=torch.int64, device=dev)
        self.proposed = torch.zeros((self.B, N_OPS_MAX), dtype=torch.int64, device=dev)
        # SAMPLE_SOURCE = true: component of every observation (Sample.source), kept on the device
        # by POSITION, uint8 [B][F][Np] (include/sbz.h source_pm): the layout the likelihood's
        # source branch reads in place and the sampler updates; `source` gives it by site
        self.source_pm = None
        if source is not None:
            src = np.ascontiguousarray(source, np.uint8)
            if src.shape != (self.B, engine.n_sites, engine.n_features):
                raise ValueError(f"source: expected {(self.B, engine.n_sites, engine.n_features)}, "
                                 f"got {src.shape}")
            self.source_pm = torch.as_tensor(engine.sources_to_positions(src), device=dev)
        self.counter = torch.zeros(self.B, dtype=torch.int64, device=dev)
        # the kernels trust the index bytes (include/sbz.h): range-check them once here, on the
        # stream that produced the tensors
        engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        engine.check_indices_device(self.B, self.zone_of_site.data_ptr(),
                                    self.source_pm.data_ptr() if self.source_pm is not None else 0,
                                    source_pm=True)
        self.refresh_ll()

    @property
    def source(self):
        """The sources by site, uint8 [B][N][F] (a device tensor computed from source_pm)."""
        if self.source_pm is None:
            return None
        pos = _torch().as_tensor(self.engine.position_of_site, device=self.source_pm.device)
        return self.source_pm[:, :, pos].transpose(1, 2).contiguous()

    def source_of(self, i):
        """Chain i's sources by site, uint8 [N][F] (device tensor)."""
        pos = _torch().as_tensor(self.engine.position_of_site, device=self.source_pm.device)
        return self.source_pm[i][:, pos].t().contiguous()

    def refresh_ll(self):
        """Recompute every chain's log-likelihood from scratch (the likelihood kernel; the source
        branch when the chains carry sources)."""
        torch = _torch()
        eng = self.engine
        eng.set_stream(torch.cuda.current_stream(self.ll.device).cuda_stream)
        eng.loglik_device(self.B, self.zone_of_site.data_ptr(), self.w.data_ptr(),
                          self.p_global.data_ptr(), self.p_zones.data_ptr(),
                          self.p_fam.data_ptr() if self.p_fam is not None else 0,
                          self.source_pm.data_ptr() if self.source_pm is not None else 0,
                          self.ll.data_ptr(), validate=False,  # checked at construction
                          source_pm=True)
        return self.ll

    def to_numpy(self):
        out = {"zone_of_site": self.zone_of_site.cpu().numpy(), "w": self.w.cpu().numpy(),
               "p_global": self.p_global.cpu().numpy(), "p_zones": self.p_zones.cpu().numpy(),
               "ll": self.ll.cpu().numpy(), "prior": self.prior.cpu().numpy()}
        if self.source_pm is not None:
            out["source"] = self.source.cpu().numpy()
        if self.p_fam is not None:
            out["p_fam"] = self.p_fam.cpu().numpy()
        return out


class Sampler:
    """MH sampler over a LikelihoodEngine's context (same data, same GPU)."""

    def __init__(self, engine, applicable_states, adj_indptr, adj_indices, operators, var_proposal,
                 min_size, warmup=False, priors=None, sample_source=False, gibbs_counts=None):
        self.engine = engine
        states = np.ascontiguousarray(applicable_states, dtype=np.uint8)
        if states.shape != (engine.n_features, engine.n_states):
            raise ValueError(f"applicable_states: expected {(engine.n_features, engine.n_states)}")
        if np.any(states.sum(axis=1) < 2):
            raise ValueError("every feature needs at least 2 applicable states (random.sample(., 2))")
        indptr = np.ascontiguousarray(adj_indptr, dtype=np.int32)
        indices = np.ascontiguousarray(adj_indices, dtype=np.int32)
        lib = engine._lib
        check(lib.sbz_set_network(engine.ctx, states.ctypes.data_as(ctypes.c_void_p),
                                  int(indices.size), indptr.ctypes.data_as(ctypes.c_void_p),
                                  indices.ctypes.data_as(ctypes.c_void_p)), engine.ctx)
        self.cfg = sbz_mh_config()
        probs = operators if isinstance(operators, np.ndarray) else op_probabilities(operators)
        for i in range(min(N_OPS_MAX, len(probs))):
            self.cfg.op_prob[i] = float(probs[i])
        self.cfg.sample_source = int(bool(sample_source))
        self.sample_source = bool(sample_source)
        prec = precisions(var_proposal)
        for i in range(4):
            self.cfg.precision[i] = float(prec[i])
        self.cfg.min_size = int(min_size)
        self.cfg.warmup = int(bool(warmup))
        self.set_priors(priors)
        if sample_source:
            cg, cf = gibbs_counts if gibbs_counts is not None else (None, None)
            self.set_gibbs_counts(cg, cf)

    def set_gibbs_counts(self, counts_global=None, counts_fam=None):
        """Prior pseudo-counts of the source-mode Gibbs operators (PGlobalPrior.counts [F][S],
        PFamiliesPrior.counts [Fam][F][S]; None = 1, the 'uniform' priors' counts)."""
        eng = self.engine
        F, S = eng.n_features, eng.n_states
        cg = None if counts_global is None else np.ascontiguousarray(counts_global, np.float64)
        cf = None if counts_fam is None else np.ascontiguousarray(counts_fam, np.float64)
        if cg is not None and cg.shape != (F, S):
            raise ValueError(f"counts_global: expected {(F, S)}, got {cg.shape}")
        if cf is not None and cf.shape != (eng.n_families, F, S):
            raise ValueError(f"counts_fam: expected {(eng.n_families, F, S)}, got {cf.shape}")
        vp = ctypes.c_void_p
        check(eng._lib.sbz_set_gibbs_counts(eng.ctx, vp(cg.ctypes.data) if cg is not None else None,
                                            vp(cf.ctypes.data) if cf is not None else None), eng.ctx)
        self._gibbs_counts = (cg, cf)

    def set_priors(self, priors):
        """The prior terms of the MH ratio (contact_zones_amd.priors.PriorSpec; None = zero)."""
        from .priors import PriorSpec
        p = priors if priors is not None else PriorSpec()
        eng = self.engine
        F, S = eng.n_features, eng.n_states
        ag = af = None
        if p.alpha_global is not None:
            ag = np.ascontiguousarray(p.alpha_global, np.float64)
            if ag.shape != (F, S):
                raise ValueError(f"alpha_global: expected {(F, S)}, got {ag.shape}")
        if p.alpha_fam is not None:
            af = np.ascontiguousarray(p.alpha_fam, np.float64)
            if af.shape != (eng.n_families, F, S):
                raise ValueError(f"alpha_fam: expected {(eng.n_families, F, S)}, got {af.shape}")
        vp = ctypes.c_void_p
        check(eng._lib.sbz_set_priors(eng.ctx, vp(ag.ctypes.data) if ag is not None else None,
                                      vp(af.ctypes.data) if af is not None else None,
                                      int(p.size_prior)), eng.ctx)
        cost = None
        if p.geo_cost is not None:
            cost = np.ascontiguousarray(p.geo_cost, np.float64)
            N = eng.n_sites
            if cost.shape != (N, N):
                raise ValueError(f"geo_cost: expected {(N, N)}, got {cost.shape}")
        check(eng._lib.sbz_set_geo_prior(eng.ctx, vp(cost.ctypes.data) if cost is not None else None,
                                         float(p.geo_scale) if cost is not None else 0.0), eng.ctx)
        self.priors = p

    def run(self, state, n_steps, max_size, p_grow_connected, seed=0, chain_id0=0, tape=None,
            tape_len=None, tape_pos=None, trace=False, trace_zones=False, alias=None):
        """Run n_steps MH steps on every chain of `state` (in place).

        max_size / p_grow_connected: scalars or per-chain arrays (warm-up: get_max_size_list and
        the 0.95 / configured mix, zone_sampling.py:1276-1291).  With `tape` (float64 [B, L]),
        the chains replay recorded decisions; `tape_pos` (int64 [B] device tensor) carries the
        cursor between calls.  Returns a dict of device tensors (traces when requested)."""
        torch = _torch()
        eng = self.engine
        dev = state.ll.device
        B = state.B
        ms = torch.as_tensor(np.broadcast_to(np.asarray(max_size, np.int32), (B,)).copy(), device=dev)
        pg = torch.as_tensor(np.broadcast_to(np.asarray(p_grow_connected, np.float64), (B,)).copy(),
                             device=dev)
        ch = sbz_chains()
        ch.zone_of_site = state.zone_of_site.data_ptr()
        ch.w = state.w.data_ptr()
        ch.p_global = state.p_global.data_ptr()
        ch.p_zones = state.p_zones.data_ptr()
        ch.p_fam = state.p_fam.data_ptr() if state.p_fam is not None else None
        ch.ll = state.ll.data_ptr()
        ch.prior = state.prior.data_ptr()
        if self.sample_source:
            if state.source_pm is None:
                raise ValueError("SAMPLE_SOURCE sampler needs chains with sources (ChainState(source=...))")
            ch.source = state.source_pm.data_ptr()
            ch.source_layout = SBZ_SOURCE_BY_POSITION
        if alias is not None:  # (pending [B] int32, p_global, p_zones, p_fam) device tensors
            pend, apg, apz, apf = alias
            ch.alias_pending = pend.data_ptr()
            ch.alias_p_global = apg.data_ptr()
            ch.alias_p_zones = apz.data_ptr()
            ch.alias_p_fam = apf.data_ptr() if apf is not None else None
        ch.max_size = ms.data_ptr()
        ch.p_grow_connected = pg.data_ptr()
        out = {"status": torch.zeros(B, dtype=torch.int32, device=dev)}
        ch.status = out["status"].data_ptr()
        keep = [ms, pg]
        if tape is not None:
            t = torch.as_tensor(np.ascontiguousarray(tape, np.float64), device=dev)
            tl = torch.as_tensor(np.asarray(tape_len, np.int64), device=dev)
            tp = tape_pos if tape_pos is not None else torch.zeros(B, dtype=torch.int64, device=dev)
            ch.tape = t.data_ptr()
            ch.tape_stride = int(t.shape[1])
            ch.tape_len = tl.data_ptr()
            ch.tape_pos = tp.data_ptr()
            out["tape_pos"] = tp
            keep += [t, tl]
        ch.seed = int(seed) & (2**64 - 1)
        ch.chain_id0 = int(chain_id0)
        ch.counter = state.counter.data_ptr()
        ch.accepted = state.accepted.data_ptr()
        ch.proposed = state.proposed.data_ptr()
        if trace:
            out["op"] = torch.empty((B, n_steps), dtype=torch.int8, device=dev)
            out["accept"] = torch.empty((B, n_steps), dtype=torch.uint8, device=dev)
            out["ll"] = torch.empty((B, n_steps), dtype=torch.float64, device=dev)
            ch.trace_op = out["op"].data_ptr()
            ch.trace_accept = out["accept"].data_ptr()
            ch.trace_ll = out["ll"].data_ptr()
        if trace_zones:
            out["zone_of_site"] = torch.empty((B, n_steps, eng.n_sites), dtype=torch.uint8, device=dev)
            ch.trace_zos = out["zone_of_site"].data_ptr()
        eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        check(eng._lib.sbz_mh_run_device(eng.ctx, B, int(n_steps), ctypes.byref(self.cfg),
                                         ctypes.byref(ch)), eng.ctx)
        out["_keep"] = keep  # the launch is asynchronous: keep its inputs alive
        return out


def run_host(sampler, state, n_steps, max_size, p_grow_connected, seed=0, chain_id0=0, tape=None,
             tape_len=None, trace=False):
    """The host-form sampler entry (sbz_mh_run): `state` is a dict of numpy arrays (zone_of_site,
    w, p_global, p_zones, p_fam, source, prior, counter, accepted, proposed), updated in place
    except for 'll' and 'status', which are (re)filled.  No torch tensors are involved: this is
    what a reference-side ctypes binding without a device allocator calls."""
    eng = sampler.engine
    B = int(np.asarray(state["zone_of_site"]).shape[0])
    keep = []

    def arr(name, dtype, shape=None, fill=None):
        a = state.get(name)
        if a is None:
            if fill is None:
                return None
            a = np.full(shape, fill, dtype)
        a = np.ascontiguousarray(a, dtype)
        state[name] = a
        keep.append(a)
        return a.ctypes.data

    st = sbz_state()
    st.zone_of_site = arr("zone_of_site", np.uint8)
    st.w = arr("w", np.float64)
    st.p_global = arr("p_global", np.float64)
    st.p_zones = arr("p_zones", np.float64)
    st.p_fam = arr("p_fam", np.float64) if eng.inheritance else None
    st.source = arr("source", np.uint8) if sampler.sample_source else None
    st.ll = arr("ll", np.float64, (B,), 0.0)
    st.prior = arr("prior", np.float64)
    ms = np.ascontiguousarray(np.broadcast_to(np.asarray(max_size, np.int32), (B,)))
    pg = np.ascontiguousarray(np.broadcast_to(np.asarray(p_grow_connected, np.float64), (B,)))
    keep += [ms, pg]
    st.max_size = ms.ctypes.data
    st.p_grow_connected = pg.ctypes.data
    st.chain_id0 = int(chain_id0)
    st.counter = arr("counter", np.uint64, (B,), 0)
    st.accepted = arr("accepted", np.int64, (B, N_OPS_MAX), 0)
    st.proposed = arr("proposed", np.int64, (B, N_OPS_MAX), 0)
    st.status = arr("status", np.int32, (B,), 0)
    tp = None
    if tape is not None:
        tv = np.ascontiguousarray(tape, np.float64)
        tl = np.ascontiguousarray(tape_len, np.int64)
        pos = arr("tape_pos", np.int64, (B,), 0)
        keep += [tv, tl]
        tp = sbz_tape(tv.ctypes.data, int(tv.shape[1]), tl.ctypes.data, pos)
    tr = None
    out = {}
    if trace:
        out = {"op": np.zeros((B, n_steps), np.int8), "accept": np.zeros((B, n_steps), np.uint8),
               "ll": np.zeros((B, n_steps), np.float64)}
        tr = sbz_trace(out["op"].ctypes.data, out["accept"].ctypes.data, out["ll"].ctypes.data)
    check(eng._lib.sbz_mh_run(eng.ctx, B, int(n_steps), ctypes.byref(sampler.cfg),
                              int(seed) & (2**64 - 1), ctypes.byref(tp) if tp is not None else None,
                              ctypes.byref(st), ctypes.byref(tr) if tr is not None else None), eng.ctx)
    return out
