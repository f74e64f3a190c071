"""Capture seeded Metropolis-Hastings trajectories from the reference sampler (BUILD CONTAINER ONLY).

For each case the reference's own ZoneMCMC / ZoneMCMCWarmup (sbayes/sampling/zone_sampling.py)
runs `generate_samples` with np.random and python `random` seeded.  Every random decision the
step loop consumes is recorded per chain, in consumption order, as a "tape" of float64 items:

  op          operator id (OPS below), from np.random.choice(fn_operators, p=...)
                                          (mcmc_generative.py:294)
  z / f / fam np.random.choice(range(n))  (zone_sampling.py:417, 466, 506-507, 584-585, 729, 810, 889)
  u_conn      random.random()             (connected step, zone_sampling.py:733, 817)
  k           random.choice(seq) index    (the k-th candidate / member in ascending order, 742, 825, 896)
  a, b        random.sample(pop, 2)       (the two altered weights / states, 421, 470, 510, 588)
  d0, d1      np.random.dirichlet(alpha)  (the two components of the proposal, dirichlet_proposal :555)
  u_acc       random.random()             (accept, mcmc_generative.py:318)

The outcome of every step is recorded too: operator, accepted flag, the chain's log-likelihood
after the step, and its zone assignment (zone_of_site).  The replay (oracle/mh_numpy.py on the
CPU, the HIP sampler on the GPU) consumes the same tape and must reproduce the outcomes.
Writes tests/golden/mh_<case>.npz.  Run: python tests/golden/make_golden_mh.py
"""
import os
import random
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import refenv  # noqa: E402
from contact_zones_amd import packing  # noqa: E402

refenv.setup()

# canonical operator ids (contact_zones_amd/sampler.py OPS uses the same order)
OPS = ["shrink_zone", "grow_zone", "swap_zone", "alter_weights", "alter_p_global",
       "alter_p_zones", "alter_p_families", "gibbsish_sample_zones",
       # SAMPLE_SOURCE = true operators (mcmc_setup.py:80-87)
       "gibbs_sample_sources", "gibbs_sample_weights", "gibbs_sample_p_global",
       "gibbs_sample_p_zones", "gibbs_sample_p_families"]


class Tape:
    """Per-chain record of the decisions, in consumption order."""

    def __init__(self):
        self.chain = None
        self.items = {}

    def put(self, *vals):
        if self.chain is None:  # initial-sample generation: not part of the step tape
            return
        self.items.setdefault(self.chain, []).extend(float(v) for v in vals)


TAPE = Tape()


class RecordingRandom:
    """Stand-in for the `random` module as used by the samplers (`_random`), recording draws."""

    def __init__(self, seed):
        self._rng = random.Random(seed)

    def random(self):
        u = self._rng.random()
        TAPE.put(u)
        return u

    def choice(self, seq):
        k = self._rng._randbelow(len(seq))  # random.choice (Python 3.10): seq[_randbelow(len(seq))]
        TAPE.put(k)
        return seq[k]

    def sample(self, population, k):
        out = self._rng.sample(population, k)
        TAPE.put(*out)
        return out

    def choices(self, population, weights=None, *, cum_weights=None, k=1):
        return self._rng.choices(population, weights, cum_weights=cum_weights, k=k)


def install_recorders(seed, zs_mod, mg_mod):
    rec = RecordingRandom(seed)
    zs_mod._random = rec
    mg_mod._random = rec
    orig_choice = np.random.choice
    orig_dirichlet = np.random.dirichlet
    orig_random = np.random.random
    orig_randint = np.random.randint
    from scipy.stats._continuous_distns import beta_gen
    from scipy.stats._distn_infrastructure import rv_generic
    orig_beta_rvs = beta_gen.__dict__.get("rvs")

    def choice(a, size=None, replace=True, p=None):
        out = orig_choice(a, size, replace, p)
        if p is not None:  # operator choice: record the canonical id of the chosen operator
            TAPE.put(OPS.index(out[0].__name__))
        else:
            TAPE.put(out)
        return out

    def dirichlet(alpha, size=None):
        out = orig_dirichlet(alpha, size)
        TAPE.put(*out)
        return out

    def random_(size=None):
        # np.random.random: the categorical draws of sample_categorical (preprocessing.py:337,
        # C order) and the feature subsets of the Gibbs operators (zone_sampling.py:335, 383)
        out = orig_random(size)
        TAPE.put(*np.ravel(out))
        return out

    def randint(low, high=None, size=None, dtype=int):
        out = orig_randint(low, high, size, dtype)
        TAPE.put(*np.ravel(out))
        return out

    def beta_rvs(self, *args, **kwds):
        # scipy.stats.beta(...).rvs() in gibbs_sample_weights (zone_sampling.py:263, 291)
        out = rv_generic.rvs(self, *args, **kwds)
        TAPE.put(*np.ravel(out))
        return out

    np.random.choice = choice
    np.random.dirichlet = dirichlet
    np.random.random = random_
    np.random.randint = randint
    beta_gen.rvs = beta_rvs

    def restore():
        np.random.choice = orig_choice
        np.random.dirichlet = orig_dirichlet
        np.random.random = orig_random
        np.random.randint = orig_randint
        if orig_beta_rvs is None:
            del beta_gen.rvs
        else:
            beta_gen.rvs = orig_beta_rvs

    return restore


def run_case(name, data, model_cfg, mcmc_cfg, steps, seed, warmup, n_chains, gibbsish=0.0):
    from sbayes.model import Model
    from sbayes.sampling import zone_sampling as zs
    from sbayes.sampling import mcmc_generative as mg

    np.random.seed(seed)
    restore = install_recorders(seed, zs, mg)
    TAPE.chain, TAPE.items = None, {}
    try:
        model = Model(data=data, config=model_cfg)
        a = mcmc_cfg["STEPS"]
        ops = {"shrink_zone": a["area"] * 0.4, "grow_zone": a["area"] * 0.4,
               "swap_zone": a["area"] * 0.2, "gibbsish_sample_zones": a["area"] * gibbsish}
        if model_cfg["SAMPLE_SOURCE"]:  # MCMC.steps_per_operator (mcmc_setup.py:80-87)
            ops.update({"gibbs_sample_sources": a.get("source", 0.0),
                        "gibbs_sample_weights": a["weights"],
                        "gibbs_sample_p_global": a["universal"],
                        "gibbs_sample_p_zones": a["contact"]})
            if model_cfg["INHERITANCE"]:
                ops["gibbs_sample_p_families"] = a["inheritance"]
        else:
            ops.update({"alter_weights": a["weights"], "alter_p_global": a["universal"],
                        "alter_p_zones": a["contact"]})
            if model_cfg["INHERITANCE"]:
                ops["alter_p_families"] = a["inheritance"]
        tot = sum(ops.values())
        ops = {k: v / tot for k, v in ops.items()}
        cls = zs.ZoneMCMCWarmup if warmup else zs.ZoneMCMC
        sampler = cls(data=data, model=model, n_chains=n_chains, operators=ops,
                      var_proposal=mcmc_cfg["PROPOSAL_PRECISION"],
                      p_grow_connected=mcmc_cfg["P_GROW_CONNECTED"],
                      initial_size=mcmc_cfg["M_INITIAL"], logger=None)

        N = data.features.shape[0]
        init, final, steps_out = {}, {}, {c: [] for c in range(n_chains)}
        orig_step = sampler.step
        orig_init = sampler.generate_initial_sample

        def gen_init(c=0):
            TAPE.chain = None
            s = orig_init(c)
            init[c] = s.copy()
            return s

        init_prior = {}

        def step(sample, c):
            init_prior.setdefault(c, float(sampler._prior[c]))  # the chain's prior at its start
            TAPE.chain = c
            acc0 = sampler.statistics["accepted_steps"]
            n0 = len(TAPE.items.get(c, []))
            new = orig_step(sample, c)
            TAPE.chain = None
            op = int(TAPE.items[c][n0])
            steps_out[c].append((op, sampler.statistics["accepted_steps"] > acc0,
                                 float(sampler._ll[c]),
                                 packing.zones_to_zone_of_site(new.zones, N),
                                 float(sampler._prior[c]),
                                 None if new.source is None else packing.source_to_index(new.source)))
            final[c] = new
            return new

        sampler.step = step
        sampler.generate_initial_sample = gen_init
        if warmup:
            best = sampler.generate_samples(n_steps=0, n_samples=0, warm_up=True, warm_up_steps=steps)
        else:
            sampler.generate_samples(steps, max(1, steps // 10))
            best = None
    finally:
        restore()

    C = 3 if model_cfg["INHERITANCE"] else 2
    out = {}
    out["obs"] = packing.features_to_obs(data.features)
    out["states"] = np.asarray(data.states, bool)
    adj = data.network["adj_mat"].tocsr()
    adj.sort_indices()
    assert np.all(adj.data != 0)
    out["adj_indptr"] = adj.indptr.astype(np.int32)
    out["adj_indices"] = adj.indices.astype(np.int32)
    fam_of_site = (packing.families_to_fam_of_site(data.families, N) if model_cfg["INHERITANCE"]
                   else np.full(N, 255, np.uint8))
    out["fam_of_site"] = fam_of_site
    out["inheritance"] = np.array(model_cfg["INHERITANCE"])
    out["warmup"] = np.array(warmup)
    out["n_zones"] = np.array(model_cfg["N_AREAS"])
    out["min_size"] = np.array(model_cfg["MIN_M"])
    max_size = sampler.max_size if warmup else [model_cfg["MAX_M"]] * n_chains
    p_grow = sampler.p_grow_connected if warmup else [mcmc_cfg["P_GROW_CONNECTED"]] * n_chains
    out["max_size"] = np.asarray(max_size, np.int32)
    out["p_grow_connected"] = np.asarray(p_grow, np.float64)
    prec = mcmc_cfg["PROPOSAL_PRECISION"]
    out["precision"] = np.array([prec["weights"], prec["universal"], prec["contact"],
                                 prec["inheritance"] if prec["inheritance"] is not None else 0.0])
    probs = np.zeros(len(OPS))
    for k, v in ops.items():
        probs[OPS.index(k)] = v
    out["op_probs"] = probs
    out["init_zone_of_site"] = np.stack([packing.zones_to_zone_of_site(init[c].zones, N)
                                         for c in range(n_chains)])
    out["init_w"] = np.stack([init[c].weights for c in range(n_chains)])
    out["init_p_global"] = np.stack([init[c].p_global[0] for c in range(n_chains)])
    out["init_p_zones"] = np.stack([init[c].p_zones for c in range(n_chains)])
    if model_cfg["INHERITANCE"]:
        out["init_p_fam"] = np.stack([init[c].p_families for c in range(n_chains)])
    L = max(len(TAPE.items.get(c, [])) for c in range(n_chains))
    tape = np.full((n_chains, L), np.nan)
    for c in range(n_chains):
        tape[c, :len(TAPE.items[c])] = TAPE.items[c]
    out["tape"] = tape
    out["tape_len"] = np.array([len(TAPE.items[c]) for c in range(n_chains)])
    out["step_op"] = np.array([[s[0] for s in steps_out[c]] for c in range(n_chains)], np.int8)
    out["step_accept"] = np.array([[s[1] for s in steps_out[c]] for c in range(n_chains)], bool)
    out["step_ll"] = np.array([[s[2] for s in steps_out[c]] for c in range(n_chains)])
    out["step_zone_of_site"] = np.array([[s[3] for s in steps_out[c]] for c in range(n_chains)],
                                        np.uint8)
    out["step_prior"] = np.array([[s[4] for s in steps_out[c]] for c in range(n_chains)])
    out["sample_source"] = np.array(bool(model_cfg["SAMPLE_SOURCE"]))
    if model_cfg["SAMPLE_SOURCE"]:
        # source assignments (component index per site and feature) at the start and after
        # every step; the Gibbs operators' prior counts (zone_sampling.py:342-343, 391-392)
        out["init_source"] = np.stack([packing.source_to_index(init[c].source)
                                       for c in range(n_chains)])
        out["step_source"] = np.array([[s[5] for s in steps_out[c]] for c in range(n_chains)],
                                      np.uint8)
        pr0 = sampler.posterior_per_chain[0].prior
        out["gibbs_counts_global"] = np.asarray(pr0.prior_p_global.counts, np.float64)
        if model_cfg["INHERITANCE"]:
            out["gibbs_counts_fam"] = np.asarray(pr0.prior_p_families.counts, np.float64)
    # final parameters of every chain
    out["final_w"] = np.stack([final[c].weights for c in range(n_chains)])
    out["final_p_global"] = np.stack([final[c].p_global[0] for c in range(n_chains)])
    out["final_p_zones"] = np.stack([final[c].p_zones for c in range(n_chains)])
    if model_cfg["INHERITANCE"]:
        out["final_p_fam"] = np.stack([final[c].p_families for c in range(n_chains)])
    # priors as the chains used them (Prior, model.py:455-505): Dirichlet concentrations of the
    # 'counts' priors scattered to [F][S] / [Fam][F][S] (0 at inapplicable states), size prior.
    # Taken from a chain's model copy (mcmc_generative.py:80): every copy re-parses the config and
    # rescales data.prior_inheritance['counts'] in place (model.py:654-660), which moves the
    # family concentrations by an ulp from the first model's.
    pr = sampler.posterior_per_chain[0].prior
    if model_cfg["INHERITANCE"] and pr.prior_p_families.prior_type.value == "counts":
        for c in range(1, n_chains):  # every copy after the first carries the same values
            other = sampler.posterior_per_chain[c].prior.prior_p_families.dirichlet
            for fam_a, fam_b in zip(pr.prior_p_families.dirichlet, other):
                assert all(np.array_equal(x, y) for x, y in zip(fam_a, fam_b))
    states = np.asarray(data.states, bool)
    F, S = states.shape
    out["prior_size"] = np.array({"none": 0, "uniform": 1, "quadratic": 2}[
        model_cfg["PRIOR"]["area_size"]["type"]])
    if pr.prior_p_global.prior_type.value == "counts":
        ag = np.zeros((F, S))
        for f in range(F):
            ag[f, states[f]] = pr.prior_p_global.dirichlet[f]
        out["prior_alpha_global"] = ag
    if model_cfg["INHERITANCE"] and pr.prior_p_families.prior_type.value == "counts":
        n_fam = len(pr.prior_p_families.dirichlet)
        af = np.zeros((n_fam, F, S))
        for fam in range(n_fam):
            for f in range(F):
                af[fam, f, states[f]] = pr.prior_p_families.dirichlet[fam][f]
        out["prior_alpha_fam"] = af
    if model_cfg["PRIOR"]["geo"]["type"] == "cost_based":  # GeoPrior (model.py:979-1139)
        out["prior_geo_cost"] = np.asarray(data.geo_prior["cost_matrix"], np.float64)
        out["prior_geo_scale"] = np.array(float(model_cfg["PRIOR"]["geo"]["scale"]))
    out["init_prior"] = np.array([init_prior[c] for c in range(n_chains)])
    if warmup:
        out["best_zone_of_site"] = packing.zones_to_zone_of_site(best.zones, N)
        out["best_w"] = np.asarray(best.weights)
        out["best_p_global"] = np.asarray(best.p_global)[0]
        out["best_p_zones"] = np.asarray(best.p_zones)
        if model_cfg["INHERITANCE"]:
            out["best_p_fam"] = np.asarray(best.p_families)
    else:
        # the reference's own statistics dict (mcmc_generative.py:56-71, 205-237)
        st = sampler.statistics
        out["stat_n_samples"] = np.array(max(1, steps // 10))
        out["stat_sample_id"] = np.asarray(st["sample_id"], np.int64)
        out["stat_sample_likelihood"] = np.asarray(st["sample_likelihood"], np.float64)
        out["stat_sample_prior"] = np.asarray(st["sample_prior"], np.float64)
        out["stat_sample_zones"] = np.asarray(st["sample_zones"], bool)
        out["stat_sample_weights"] = np.asarray(st["sample_weights"], np.float64)
        out["stat_sample_p_global"] = np.asarray(st["sample_p_global"], np.float64)
        out["stat_sample_p_zones"] = np.asarray(st["sample_p_zones"], np.float64)
        if model_cfg["INHERITANCE"]:
            out["stat_sample_p_families"] = np.asarray(st["sample_p_families"], np.float64)
        out["stat_accepted_steps"] = np.array(st["accepted_steps"])
        out["stat_acceptance_ratio"] = np.array(st["acceptance_ratio"])
        out["stat_accept_operator"] = np.array([st["accept_operator"].get(k, 0) for k in OPS])
        out["stat_reject_operator"] = np.array([st["reject_operator"].get(k, 0) for k in OPS])
        out["stat_last_zones"] = np.asarray(st["last_sample"].zones, bool)
        out["stat_last_weights"] = np.asarray(st["last_sample"].weights, np.float64)
        # the reference's per-zone contributions of every logged sample (postprocessing.py:271-313)
        if not model_cfg["SAMPLE_SOURCE"]:  # (the reference's single-zone samples carry no source)
            from sbayes.postprocessing import contribution_per_area
            contribution_per_area(sampler)
            out["stat_lh_single_zones"] = np.asarray(sampler.statistics["sample_lh_single_zones"])
            out["stat_prior_single_zones"] = np.asarray(sampler.statistics["sample_prior_single_zones"])
    # run metadata (for the host-side drop-in tests: initial samples, warm-up lists)
    out["seed"] = np.array(seed)
    out["initial_size"] = np.array(mcmc_cfg["M_INITIAL"])
    out["max_m"] = np.array(model_cfg["MAX_M"])
    out["p_grow_base"] = np.array(mcmc_cfg["P_GROW_CONNECTED"])
    path = os.path.join(HERE, f"mh_{name}.npz")
    np.savez_compressed(path, **out)
    acc = out["step_accept"].mean()
    print(f"{name:22s} chains={n_chains} steps={steps} tape={L} accept={acc:.3f} "
          f"ops={np.bincount(out['step_op'].ravel(), minlength=len(OPS))} -> {os.path.getsize(path)} B")
    assert C in (2, 3)


def sim_data(inheritance_families=0, seed=1):
    """sim_exp1 simulated by the reference (as make_golden_lik.case_cfg1_sim); optional
    synthetic families (the simulation config has none) for the inheritance model."""
    from sbayes.experiment_setup import Experiment
    from sbayes.simulation import Simulation
    exp_dir = refenv.scratch_copy("experiments/simulation/sim_exp1")
    np.random.seed(seed)
    random.seed(seed)
    exp = Experiment(experiment_name="golden", config_file=os.path.join(exp_dir, "config.json"), log=False)
    exp.load_config(os.path.join(exp_dir, "config.json"), custom_settings={
        "simulation": {"I_CONTACT": 3, "E_CONTACT": 0.5, "STRENGTH": 1, "AREA": 4}})
    sim = Simulation(experiment=exp)
    sim.run_simulation()
    N = sim.features.shape[0]
    fams = None
    if inheritance_families:
        rng = np.random.default_rng(seed + 100)
        lab = rng.integers(0, inheritance_families + 1, size=N)  # label 0: no family
        fams = np.stack([lab == i + 1 for i in range(inheritance_families)])
    return types.SimpleNamespace(features=sim.features, states=sim.states, network=sim.network,
                                 families=fams)


def small_data(seed=7, N=40, F=12, S=4, fam=2):
    """A small random network (Delaunay of random points, the reference's compute_network) that
    hits the size bounds and the no-candidate rejections often."""
    from sbayes.preprocessing import compute_network
    rng = np.random.default_rng(seed)
    sites = {"id": list(range(N)), "locations": rng.random((N, 2)) * 100,
             "names": [f"s{i}" for i in range(N)]}
    net = compute_network(sites)
    states = np.ones((F, S), bool)
    states[rng.random((F, S)) < 0.25] = False
    states[:, :2] = True
    x = np.zeros((N, F, S), bool)
    for f in range(F):
        st = np.flatnonzero(states[f])
        xs = rng.choice(st, size=N)
        x[np.arange(N), f, xs] = True
    x[rng.random((N, F)) < 0.05] = False  # NA cells
    lab = rng.integers(0, fam + 1, size=N)
    fams = np.stack([lab == i + 1 for i in range(fam)])
    return types.SimpleNamespace(features=x, states=states, network=net, families=fams)


def model_cfg(Z, inheritance, min_m=3, max_m=50, counts=False, size="none", source=False, geo=None):
    prior = {"geo": {"type": "cost_based", "scale": geo} if geo else {"type": "uniform"},
             "area_size": {"type": size},
             "weights": {"type": "uniform"}, "universal": {"type": "uniform"},
             "inheritance": {"type": "uniform"}, "contact": {"type": "uniform"}}
    if counts:  # as experiments/balkan/config.json:34-50
        prior["universal"] = {"type": "counts", "scale_counts": None}
        prior["inheritance"] = {"type": "counts", "scale_counts": 10}
    return {"N_AREAS": Z, "MIN_M": min_m, "MAX_M": max_m, "INHERITANCE": inheritance,
            "SAMPLE_SOURCE": source, "PRIOR": prior}


def with_counts(d, seed=11):
    """Attach prior counts (load_data.py:86, 113 layouts: 'counts' [F][S], [Fam][F][S]) drawn for
    the applicable states."""
    rng = np.random.default_rng(seed)
    st = np.asarray(d.states, bool)
    cu = np.where(st, rng.integers(0, 40, size=st.shape), 0).astype(float)
    n_fam = d.families.shape[0]
    ci = np.where(st[None], rng.integers(0, 25, size=(n_fam,) + st.shape), 0).astype(float)
    return types.SimpleNamespace(features=d.features, states=d.states, network=d.network,
                                 families=d.families, prior_universal={"counts": cu},
                                 prior_inheritance={"counts": ci})


def with_geo(d, cost=None):
    """Attach the geo prior's cost matrix (load_data.py:106-121: the network's distance matrix
    when no cost file is given)."""
    c = d.network["dist_mat"] if cost is None else cost
    return types.SimpleNamespace(**{**vars(d), "geo_prior": {"cost_matrix": np.asarray(c, np.float64)}})


def mcmc_cfg(area=0.4, m_initial=5, p_grow=0.85, inheritance=0.1, source=0.0):
    return {"P_GROW_CONNECTED": p_grow, "M_INITIAL": m_initial,
            "PROPOSAL_PRECISION": {"weights": 15, "universal": 40, "contact": 20, "inheritance": 20},
            "STEPS": {"area": area, "weights": 0.2, "universal": 0.1, "contact": 0.2,
                      "inheritance": inheritance, "source": source}}


def geo_cases():
    """Cost-based geo prior (experiments/simulation/sim_exp2/config.json:50-53): only the last
    zone's MST enters the prior (model.py:1110-1139 overwrites log_prior in its zone loop)."""
    s = small_data()
    run_case("small_geo", with_geo(s), model_cfg(2, True, min_m=3, max_m=8, geo=30.0),
             mcmc_cfg(area=0.8, m_initial=4), steps=300, seed=15, warmup=False, n_chains=3)
    # integer costs with ties and zeros (zero-cost edges leave the MST's nonzero count)
    rng = np.random.default_rng(16)
    n = s.features.shape[0]
    c = rng.integers(0, 6, size=(n, n)).astype(float)
    c = np.triu(c, 1)
    c = c + c.T
    run_case("small_geo_ties_warmup", with_geo(s, c), model_cfg(2, True, min_m=3, max_m=8, geo=2.0),
             mcmc_cfg(area=0.8, m_initial=4), steps=200, seed=17, warmup=True, n_chains=4)
    run_case("src_geo", with_geo(s), model_cfg(2, True, min_m=3, max_m=8, source=True, geo=30.0),
             mcmc_cfg(area=0.4, m_initial=4, source=0.05), steps=150, seed=18, warmup=False,
             n_chains=2)


def real_data(name, n_zones):
    """The reference's own Experiment -> Data for experiments/<name>/config.json (features,
    counts priors, network), N_AREAS = n_zones, from a scratch copy (load_universal_counts writes
    into the CWD); South America with CRS = None.  Returns (data, model config,
    mcmc config) as the reference's MCMC would use them."""
    import json
    from sbayes.experiment_setup import Experiment
    from sbayes.load_data import Data
    d = refenv.scratch_copy(f"experiments/{name}")
    cwd = os.getcwd()
    os.chdir(d)
    try:
        with open("config.json") as f:
            raw = json.load(f)
        custom = {"model": {"N_AREAS": n_zones}}
        for low, up in (("features", "FEATURES"), ("feature_states", "FEATURE_STATES")):
            if low in raw.get("data", {}):
                custom.setdefault("data", {})[up] = raw["data"][low]
        if name == "south_america":
            custom.setdefault("data", {})["CRS"] = None
        exp = Experiment(experiment_name="golden", log=False)
        exp.load_config(config_file="config.json", custom_settings=custom)
        data = Data(experiment=exp)
        data.load_features()
        data.load_universal_counts()
        data.load_inheritance_counts()
        return data, exp.config["model"], exp.config["mcmc"]
    finally:
        os.chdir(cwd)


def real_cases():
    """SAMPLE_SOURCE = true runs of the reference's own real-data configs (BASELINE configs[2]
    and [3]): Balkan with 3 zones, South America with 1 and 6 zones, their counts priors,
    STEPS, PROPOSAL_PRECISION, MIN_M / MAX_M / M_INITIAL, 2 chains x 100 steps."""
    for name, z, seed in (("balkan", 3, 31), ("south_america", 1, 32), ("south_america", 6, 33)):
        data, model, mcmc = real_data(name, z)
        tag = "balkan" if name == "balkan" else "sa"
        run_case(f"src_{tag}_z{z}", data, model, mcmc, steps=100, seed=seed, warmup=False, n_chains=2)


def sa_sweep_cases():
    """South America with K = 2..5 zones (BASELINE configs[3] sweeps K = 1..6; real_cases holds
    K = 1 and 6): the same capture, 2 chains x 100 steps each."""
    for z, seed in ((2, 34), (3, 35), (4, 36), (5, 37)):
        data, model, mcmc = real_data("south_america", z)
        run_case(f"src_sa_z{z}", data, model, mcmc, steps=100, seed=seed, warmup=False, n_chains=2)


def gibbsish_cases():
    """gibbsish_sample_zones (zone_sampling.py:619-702) with a non-zero operator weight.  The
    reference's own operator table gives it weight 0 (mcmc_setup.py:77, 'area' * 0.0), so these
    captures set the weight in the capture's table only (run_case(gibbsish=...)); the reference
    files are not touched.  Mixture and SAMPLE_SOURCE, ZoneMCMC and ZoneMCMCWarmup, a small network
    (every free site available) and the 951-site simulation (more than 100 available sites: the
    random subset of :631-633)."""
    s = small_data()
    run_case("gibbsish_small", s, model_cfg(2, True, min_m=3, max_m=25), mcmc_cfg(area=0.6, m_initial=4),
             steps=300, seed=41, warmup=False, n_chains=3, gibbsish=0.6)
    run_case("gibbsish_small_warmup", s, model_cfg(2, True, min_m=3, max_m=25),
             mcmc_cfg(area=0.6, m_initial=4), steps=200, seed=42, warmup=True, n_chains=4, gibbsish=0.6)
    d3 = sim_data(inheritance_families=3)
    run_case("gibbsish_sim", d3, model_cfg(2, True, min_m=3, max_m=120), mcmc_cfg(area=0.6),
             steps=200, seed=43, warmup=False, n_chains=2, gibbsish=0.6)
    run_case("src_gibbsish_small", s, model_cfg(2, True, min_m=3, max_m=25, source=True),
             mcmc_cfg(area=0.4, m_initial=4, source=0.05), steps=200, seed=44, warmup=False,
             n_chains=3, gibbsish=0.6)
    run_case("src_gibbsish_warmup", s, model_cfg(2, True, min_m=3, max_m=25, source=True),
             mcmc_cfg(area=0.4, m_initial=4, source=0.05), steps=150, seed=45, warmup=True,
             n_chains=3, gibbsish=0.6)
    run_case("src_gibbsish_noinh", s, model_cfg(2, False, min_m=3, max_m=25, source=True),
             mcmc_cfg(area=0.4, m_initial=4, inheritance=0.0, source=0.05), steps=150, seed=46,
             warmup=False, n_chains=2, gibbsish=0.6)
    # zone moves redraw all 951 x 35 sources (33 k tape items each): few steps, mostly gibbsish
    run_case("src_gibbsish_sim", d3, model_cfg(2, True, min_m=3, max_m=120, source=True),
             mcmc_cfg(area=0.5, source=0.0), steps=24, seed=47, warmup=False, n_chains=1,
             gibbsish=6.0)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "gibbsish":
        gibbsish_cases()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "geo":
        geo_cases()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "real":
        real_cases()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "sa_sweep":
        sa_sweep_cases()
        return
    d = sim_data()
    run_case("cfg1_sim", d, model_cfg(1, False), mcmc_cfg(inheritance=0.0), steps=300, seed=3,
             warmup=False, n_chains=2)
    d3 = sim_data(inheritance_families=3)
    run_case("cfg1_sim_inh_z2", d3, model_cfg(2, True), mcmc_cfg(), steps=300, seed=4,
             warmup=False, n_chains=2)
    run_case("cfg1_sim_warmup", d3, model_cfg(2, True), mcmc_cfg(), steps=200, seed=5,
             warmup=True, n_chains=4)
    s = small_data()
    run_case("small_bounds", s, model_cfg(3, True, min_m=3, max_m=6), mcmc_cfg(area=0.8, m_initial=4),
             steps=400, seed=6, warmup=False, n_chains=3)
    run_case("small_warmup", s, model_cfg(2, True, min_m=3, max_m=8), mcmc_cfg(area=0.8, m_initial=4),
             steps=300, seed=8, warmup=True, n_chains=4)
    sc = with_counts(s)
    run_case("small_priors", sc, model_cfg(3, True, min_m=3, max_m=6, counts=True, size="uniform"),
             mcmc_cfg(area=0.6, m_initial=4), steps=400, seed=9, warmup=False, n_chains=3)
    # SAMPLE_SOURCE = true (the reference default, config/default_config.json:32)
    run_case("src_small", s, model_cfg(2, True, min_m=3, max_m=8, source=True),
             mcmc_cfg(area=0.25, m_initial=4, source=0.05), steps=200, seed=12, warmup=False,
             n_chains=3)
    run_case("src_small_noinh", s, model_cfg(2, False, min_m=3, max_m=8, source=True),
             mcmc_cfg(area=0.25, m_initial=4, inheritance=0.0, source=0.05), steps=200, seed=13,
             warmup=False, n_chains=2)
    run_case("src_priors_warmup", sc,
             model_cfg(2, True, min_m=3, max_m=8, counts=True, size="uniform", source=True),
             mcmc_cfg(area=0.25, m_initial=4), steps=150, seed=14, warmup=True, n_chains=3)
    run_case("small_priors_warmup", sc,
             model_cfg(2, True, min_m=3, max_m=8, counts=True, size="quadratic"),
             mcmc_cfg(area=0.6, m_initial=4), steps=300, seed=10, warmup=True, n_chains=4)
    geo_cases()
    real_cases()


if __name__ == "__main__":
    main()
