"""Run an sBayes experiment config end to end on the GPU: the reference's CLI path
(sbayes/cli.py:13-87: Experiment -> Data -> MCMC.warm_up -> MCMC.sample -> save_samples) with
the batched GPU sampler in place of ZoneMCMCWarmup / ZoneMCMC, and no dependency on the
reference package.

  config        sbayes/experiment_setup.py:62-90 (load_config), :124-260 (verify_config),
                defaults of sbayes/config/default_config.json (DEFAULT_CONFIG below)
  data          sbayes/load_data.py:63-121 via contact_zones_amd.io (packed features, Delaunay
                network, prior counts)
  operators     sbayes/mcmc_setup.py:70-95 (steps_per_operator)
  priors        sbayes/model.py:538-680: 'counts' priors on p_global / p_families
                (initial count 1 + scale_counts), zone-size prior, 'cost_based' geo prior
                (cost file or the distance matrix, model.py:979-1139); weights / contact
                must be 'uniform' (NotImplementedError otherwise, as the batched sampler)
  sampling      warm-up: BatchedZoneMCMCWarmup, N_WARM_UP_CHAINS chains in one launch; main:
                BatchedZoneMCMC from the warm-up's best sample (mcmc_setup.py:97-121, 174-187)
  results       contribution_per_area (GPU batch), match_areas, rank_areas, samples2file
                (mcmc_setup.py:189-260) -> <RESULTS_PATH>/<name>/<file_info>/stats_*.txt, areas_*.txt

Simulation configs ('simulation' key) are not supported here.
Usage: python -m contact_zones_amd <config.json> [--name NAME] [--seed S] [--device D]
"""
import copy
import json
import logging
import os
import random
import time
import types

import numpy as np

REQUIRED = "<REQUIRED>"

# sbayes/config/default_config.json
DEFAULT_CONFIG = {
    "mcmc": {
        "N_STEPS": 1000000, "N_SAMPLES": 1000, "N_RUNS": 1, "P_GROW_CONNECTED": 0.85,
        "PROPOSAL_PRECISION": {"weights": 15, "universal": 40, "contact": 20, "inheritance": 20},
        "STEPS": {"area": 0.05, "weights": 0.4, "universal": 0.05, "contact": 0.4,
                  "inheritance": 0.1, "source": 0.0},
        "M_INITIAL": 5,
        "WARM_UP": {"N_WARM_UP_STEPS": 100000, "N_WARM_UP_CHAINS": 15},
    },
    "model": {
        "N_AREAS": REQUIRED, "MIN_M": 3, "MAX_M": 50, "INHERITANCE": REQUIRED, "SAMPLE_SOURCE": True,
        "PRIOR": {"geo": {"type": "uniform"}, "area_size": {"type": "none"},
                  "weights": {"type": "uniform"}, "universal": {"type": "uniform"},
                  "inheritance": {"type": "uniform"}, "contact": {"type": "uniform"}},
    },
    "data": {"FEATURES": REQUIRED, "FEATURE_STATES": REQUIRED},
}


def set_defaults(cfg, default):
    """experiment_setup.py:263-281: fill missing keys recursively."""
    for k, v in default.items():
        if k not in cfg:
            cfg[k] = copy.deepcopy(v)
        elif isinstance(v, dict) and isinstance(cfg[k], dict):
            set_defaults(cfg[k], v)
    return cfg


def update_recursive(cfg, new):
    for k, v in new.items():
        if isinstance(v, dict) and isinstance(cfg.get(k), dict):
            update_recursive(cfg[k], v)
        else:
            cfg[k] = v
    return cfg


def _iter_items(d, prefix=""):
    for k, v in d.items():
        if isinstance(v, dict):
            yield from _iter_items(v, prefix + k + ".")
        else:
            yield prefix + k, v


def load_config(config_file, custom_settings=None, simulated=False):
    """The reference's load_config + verify_config: returns the verified config (paths made
    relative to the config's directory) and that directory.  A simulation config (a 'simulation'
    section, experiments/simulation/*/config.json) needs `simulated=True`: its data then come as
    SimulatedData (the runner's --sim-data), since simulating them is not part of this path."""
    base = os.path.dirname(os.path.abspath(config_file))
    with open(config_file) as f:
        cfg = json.load(f)
    if "simulation" in cfg and not simulated:
        raise NotImplementedError("simulation config: pass the simulated data (--sim-data, SimulatedData)")
    data = cfg.setdefault("data", {})
    for low, up in (("features", "FEATURES"), ("feature_states", "FEATURE_STATES")):
        if low in data and up not in data:  # experiments/balkan/config.json spells them lowercase
            data[up] = data.pop(low)
    set_defaults(cfg, DEFAULT_CONFIG)
    if custom_settings:
        update_recursive(cfg, custom_settings)
    if simulated:  # the data come from the simulation (Simulation, not read from files)
        for k in ("FEATURES", "FEATURE_STATES"):
            if data.get(k) == REQUIRED:
                del data[k]

    def fix(p):
        return p if os.path.isabs(p) else os.path.join(base, p)

    for k, v in _iter_items(cfg):
        if v == REQUIRED:
            raise NameError(f"{k} is not defined in {config_file}")
    model, mcmc = cfg["model"], cfg["mcmc"]
    inh = bool(model["INHERITANCE"])
    pri = model["PRIOR"]
    if not inh:
        pri["inheritance"] = None
    for key in ["geo", "area_size", "weights", "universal", "contact"] + (["inheritance"] if inh else []):
        prior = pri[key]
        if "type" not in prior:
            raise NameError(f"type for prior '{key}' is not defined in {config_file}.")
        if prior["type"] == "counts":
            if "file_type" not in prior:
                raise NameError(f"counts file for prior '{key}' is not defined in {config_file}.")
            prior.setdefault("scale_counts", None)
            if key == "universal":
                prior["file"] = fix(prior["file"])
            elif key == "inheritance":
                prior["files"] = {fam: fix(p) for fam, p in prior["files"].items()}
        if prior["type"] == "cost_based":
            if "scale" not in prior:
                raise NameError(f"scale for geo prior is not defined in {config_file}.")
            if "file" in prior:
                prior["file"] = fix(prior["file"])
    mcmc["N_CHAINS"] = 1  # MC3 is disabled in the reference (experiment_setup.py:200-206)
    # independent main-run chains (an extension, MC3 still off): chain 0 is the reference's logged
    # chain; chains 1.. get results files of their own (run_experiment)
    k = mcmc.setdefault("INDEPENDENT_CHAINS", 1)
    if not isinstance(k, int) or k < 1:
        raise ValueError(f"INDEPENDENT_CHAINS must be a positive integer, got {k!r}")
    if mcmc["N_STEPS"] % mcmc["N_SAMPLES"] != 0:
        raise ValueError("Non-consistent spacing between samples. Set N_STEPS to be a multiple of N_SAMPLES. ")
    steps = mcmc["STEPS"]
    if not inh:
        steps["inheritance"] = 0.0
    if not model["SAMPLE_SOURCE"]:
        steps["source"] = 0.0
    total = sum(steps.values())
    for k in steps:
        steps[k] = steps[k] / total
    res = cfg.setdefault("results", {})
    res.setdefault("RESULTS_PATH", "results")
    res.setdefault("FILE_INFO", "n")
    for k in ("FEATURES", "FEATURE_STATES"):
        if k in data:
            data[k] = fix(data[k])
    res["RESULTS_PATH"] = fix(res["RESULTS_PATH"])
    return cfg, base


def operators(config):
    """mcmc_setup.py:70-95 (steps_per_operator)."""
    steps = config["mcmc"]["STEPS"]
    ops = {"shrink_zone": steps["area"] * 0.4, "grow_zone": steps["area"] * 0.4,
           "swap_zone": steps["area"] * 0.2, "gibbsish_sample_zones": steps["area"] * 0.0}
    if config["model"]["SAMPLE_SOURCE"]:
        ops.update({"gibbs_sample_sources": steps["source"], "gibbs_sample_weights": steps["weights"],
                    "gibbs_sample_p_global": steps["universal"], "gibbs_sample_p_zones": steps["contact"],
                    "gibbs_sample_p_families": steps["inheritance"]})
    else:
        ops.update({"alter_weights": steps["weights"], "alter_p_global": steps["universal"],
                    "alter_p_zones": steps["contact"], "alter_p_families": steps["inheritance"]})
    return ops


EPS = np.finfo(float).eps  # sbayes/util.py:EPS


def scale_counts(counts, scale_to):
    """util.py:569-586."""
    s = np.sum(counts, axis=-1)
    s = np.where(s == 0, EPS, s)
    factor = scale_to / s
    factor = np.where(factor < 1, factor, 1)
    return counts * factor[..., None]


class ExperimentData:
    """The attributes of the reference's Data (load_data.py:25-61) the batched sampler and the
    results writer use, from contact_zones_amd.io."""

    def __init__(self, config):
        from . import io
        import scipy.sparse as sp
        d = config["data"]
        self.table = io.read_features_packed(d["FEATURES"], d["FEATURE_STATES"])
        t = self.table
        self.features = t.one_hot()
        self.states = t.applicable
        self.families = t.families
        self.feature_names = {"external": t.feature_names, "internal": list(range(t.n_features))}
        self.state_names = {"external": t.state_names,
                            "internal": [list(range(len(s))) for s in t.state_names]}
        self.family_names = {"external": t.family_names, "internal": list(range(len(t.family_names)))}
        indptr, indices, dist = io.compute_network(t.locations)
        N = t.n_sites
        self.network = {"adj_mat": sp.csr_matrix((np.ones(indices.size, int), indices, indptr), shape=(N, N)),
                        "dist_mat": dist, "locations": t.locations}
        self.is_simulated = False
        self.log = [t.log]
        pri = config["model"]["PRIOR"]
        self.universal_counts = self.inheritance_counts = None
        if pri["universal"]["type"] == "counts":
            self.universal_counts, lg = io.read_universal_counts(
                t, pri["universal"]["file"], pri["universal"]["file_type"], d["FEATURE_STATES"])
            self.log.append(lg)
        self.geo_cost = None
        if pri["geo"]["type"] == "cost_based":  # load_geo_cost_matrix (load_data.py:106-121)
            if "file" in pri["geo"]:
                self.geo_cost, lg = io.read_geo_cost_matrix([str(x) for x in t.site_ids], pri["geo"]["file"])
                self.log.append(lg)
            else:
                self.geo_cost = dist
        if config["model"]["INHERITANCE"] and pri["inheritance"]["type"] == "counts":
            self.inheritance_counts, lg = io.read_inheritance_counts(
                t, pri["inheritance"]["files"], pri["inheritance"]["file_type"], d["FEATURE_STATES"])
            self.log.append(lg)


class SimulatedData:
    """Simulated data with its ground truth, in the attributes of the reference's Simulation
    (simulation.py:30-160) that MCMC, eval_ground_truth and samples2file read: features, states,
    names, network, is_simulated = True, and the truth — areas (Z_true, N), weights (F, C),
    p_universal (F, S), p_contact (Z_true, F, S), p_inheritance (Fam, F, S) or None, families.
    The simulation itself (simulate_features etc.) is not part of the hot path: the arrays come
    from the reference's own Simulation or any other source (see from_npz)."""

    def __init__(self, obs, states, locations, areas, weights, p_universal, p_contact,
                 p_inheritance=None, fam_of_site=None, feature_names=None, state_names=None,
                 family_names=None, geo_cost=None):
        import scipy.sparse as sp
        from . import io, packing
        obs = np.asarray(obs, np.int8)
        N, F = obs.shape
        states = np.asarray(states, bool)
        S = states.shape[1]
        fam = np.full(N, 255, np.uint8) if fam_of_site is None else np.asarray(fam_of_site, np.uint8)
        Fam = int(fam[fam != 255].max()) + 1 if np.any(fam != 255) else 0
        feature_names = list(feature_names) if feature_names is not None else [f"f{f + 1}" for f in range(F)]
        state_names = ([list(x) for x in state_names] if state_names is not None else
                       [[f"s{x + 1}" for x in range(int(states[f].sum()))] for f in range(F)])
        family_names = list(family_names) if family_names is not None else [f"fam{i + 1}" for i in range(Fam)]
        self.table = types.SimpleNamespace(
            obs=obs, applicable=states, fam_of_site=fam, n_sites=N, n_features=F, n_states=S,
            feature_names=feature_names, state_names=state_names, family_names=family_names,
            locations=np.asarray(locations, np.float64))
        self.features = packing.obs_to_features(obs, S)
        self.states = states
        self.families = packing.index_to_groups(fam, Fam) if Fam else np.zeros((0, N), bool)
        self.feature_names = {"external": feature_names, "internal": list(range(F))}
        self.state_names = {"external": state_names, "internal": [list(range(len(x))) for x in state_names]}
        self.family_names = {"external": family_names, "internal": list(range(Fam))}
        indptr, indices, dist = io.compute_network(self.table.locations)
        self.network = {"adj_mat": sp.csr_matrix((np.ones(indices.size, int), indices, indptr), shape=(N, N)),
                        "dist_mat": dist, "locations": self.table.locations}
        self.is_simulated = True
        self.log = [f"simulated data: {N} sites, {F} features, {np.asarray(areas).shape[0]} true areas"]
        self.universal_counts = self.inheritance_counts = None
        self.geo_cost = dist if geo_cost is None else np.asarray(geo_cost, np.float64)
        self.areas = np.asarray(areas, bool)
        self.weights = np.asarray(weights, np.float64)
        self.p_universal = np.asarray(p_universal, np.float64)
        self.p_contact = np.asarray(p_contact, np.float64)
        self.p_inheritance = None if p_inheritance is None else np.asarray(p_inheritance, np.float64)

    @classmethod
    def from_npz(cls, path):
        """Arrays saved with keys obs, states, locations, areas, weights, p_universal, p_contact
        [, p_inheritance, fam_of_site, geo_cost] and optional JSON-encoded names ('names':
        {"features": [...], "states": [[...]], "families": [...]})."""
        import json
        with np.load(path, allow_pickle=False) as z:
            d = {k: z[k] for k in z.files}
        names = json.loads(str(d.pop("names"))) if "names" in d else {}
        return cls(d["obs"], d["states"], d["locations"], d["areas"], d["weights"], d["p_universal"],
                   d["p_contact"], d.get("p_inheritance"), d.get("fam_of_site"), names.get("features"),
                   names.get("states"), names.get("families"), d.get("geo_cost"))


def build_priors(config, data):
    """The prior terms the batched sampler uses (model.py:538-680): Dirichlet concentrations
    alpha [F][S] / [Fam][F][S] (1 + scaled counts on the applicable states) and, in source mode,
    the Gibbs pseudo-counts (prior.prior_p_*.counts)."""
    from .priors import PriorSpec
    model = config["model"]
    pri = model["PRIOR"]
    for key in ("weights", "contact"):
        if pri[key]["type"] != "uniform":
            raise NotImplementedError(f"{key} prior of type '{pri[key]['type']}' is not supported")
    if pri["geo"]["type"] not in ("uniform", "cost_based"):
        raise NotImplementedError(f"geo prior of type '{pri['geo']['type']}' is not supported")
    F, S = data.states.shape
    Fam = data.families.shape[0]
    cg = np.ones((F, S))
    ag = None
    if pri["universal"]["type"] == "counts":
        c = data.universal_counts.astype(float)
        if pri["universal"]["scale_counts"] is not None:
            c = scale_counts(c, pri["universal"]["scale_counts"])
        cg = 1.0 + c                                    # prior.counts (model.py:585)
        ag = np.where(data.states, cg + 1.0, 0.0)       # counts_to_dirichlet adds 1 (util.py:618)
    elif pri["universal"]["type"] != "uniform":
        raise NotImplementedError(f"universal prior of type '{pri['universal']['type']}' is not supported")
    cf, af = None, None
    if model["INHERITANCE"]:
        cf = np.ones((Fam, F, S))
        t = pri["inheritance"]["type"]
        if t == "counts":
            c = data.inheritance_counts.astype(float)
            if pri["inheritance"]["scale_counts"] is not None:
                c = scale_counts(c, pri["inheritance"]["scale_counts"])
            cf = 1.0 + c                                # model.py:664
            af = np.where(data.states[None], cf + 1.0, 0.0)  # util.py:547-566, 618
        elif t != "uniform":
            raise NotImplementedError(f"inheritance prior of type '{t}' is not supported")
    size = pri["area_size"]["type"]
    geo_cost = data.geo_cost if pri["geo"]["type"] == "cost_based" else None
    geo_scale = pri["geo"]["scale"] if geo_cost is not None else None
    return PriorSpec(ag, af, size, geo_cost, geo_scale), (cg, cf)


def model_spec(config, n_zones):
    m = config["model"]
    return types.SimpleNamespace(n_zones=int(n_zones), min_size=int(m["MIN_M"]), max_size=int(m["MAX_M"]),
                                 inheritance=bool(m["INHERITANCE"]), sample_source=bool(m["SAMPLE_SOURCE"]))


def derive_seeds(seed, run, n_zones):
    """Independent seeds for the phases of one (run, n_zones) job from the experiment seed.

    The reference draws everything from the global `random` / `np.random` streams, so its warm-up,
    main run and every N_RUNS / N_AREAS job consume different draws.  The GPU sampler keys its
    Philox streams by (seed, global chain id) with the counter starting at 0 in every ChainState,
    so reusing one seed would hand each main chain exactly the uniforms its warm-up chain used, and
    make every replicate of N_RUNS bit-identical.  SeedSequence([seed, run, n_zones]).spawn(3)
    gives the host draws (initial samples, initial sources), the warm-up Philox key and the
    main-run Philox key, pairwise independent and reproducible from `seed`."""
    ss = np.random.SeedSequence([int(seed) & (2**63 - 1), int(run), int(n_zones)])
    host, warm, main = (int(c.generate_state(1, np.uint64)[0]) & (2**63 - 1) for c in ss.spawn(3))
    return {"host": host, "warmup": warm, "sample": main}


def agree_seed(seed=None, group=None):
    """The experiment seed every rank uses: `seed` if given, else one drawn from OS entropy on
    rank 0; broadcast from rank 0 of `group` when torch.distributed is initialised, so that all
    ranks build the same initial samples (the chains are sharded, their initial states are not)."""
    from .parallel import broadcast_seed
    if seed is None:
        seed = int(np.random.SeedSequence().entropy) & (2**63 - 1)
    return broadcast_seed(int(seed), group)


def run_experiment(config, data, n_zones, run=0, name="experiment", seed=None, device=None,
                   logger=None, warmup_chains=None, group=None):
    """One run for one number of zones (cli.py:13-27): warm-up, sampling, results files.
    Returns (statistics, paths).  `seed` is the experiment seed (None: fresh entropy, agreed
    across the ranks of `group`); the phases draw from independent streams derived from
    (seed, run, n_zones), so a job's files do not depend on which rank or thread runs it or on
    what runs beside it.  `group`: the ranks whose GPUs share this job's chains (None: all ranks;
    a one-rank group when the runner shards the jobs themselves, run_jobs)."""
    from . import io
    from .mcmc import BatchedZoneMCMC, BatchedZoneMCMCWarmup
    from .postprocessing import contribution_per_area, eval_ground_truth, match_areas, rank_areas
    logger = logger or logging.getLogger("sbz")
    mc = config["mcmc"]
    cfg = copy.deepcopy(config)
    cfg["model"]["N_AREAS"] = int(n_zones)
    priors, gibbs = build_priors(cfg, data)
    model = model_spec(cfg, n_zones)
    ops = operators(cfg)
    seeds = derive_seeds(agree_seed(seed, group), run, n_zones)
    rng = random.Random(seeds["host"])
    # the initial sources' draws: the reference's np.random stream seeded per job, as a RandomState
    # of the job's own (the same draws as np.random.seed + np.random.random)
    nps = np.random.RandomState(seeds["host"] % 2**32)
    common = dict(model=model, data=data, operators=ops, var_proposal=mc["PROPOSAL_PRECISION"],
                  p_grow_connected=mc["P_GROW_CONNECTED"], initial_size=mc["M_INITIAL"],
                  logger=logger, rng=rng, device=device, priors=priors,
                  gibbs_counts=gibbs if model.sample_source else None, group=group,
                  np_random=nps.random_sample)
    t0 = time.time()
    warm = BatchedZoneMCMCWarmup(n_chains=warmup_chains or mc["WARM_UP"]["N_WARM_UP_CHAINS"],
                                 seed=seeds["warmup"], **common)
    best = warm.generate_samples(n_steps=0, n_samples=0, warm_up=True,
                                 warm_up_steps=mc["WARM_UP"]["N_WARM_UP_STEPS"])
    logger.info("warm-up: %d chains x %d steps in %.2f s", warm.n_chains, mc["WARM_UP"]["N_WARM_UP_STEPS"],
                time.time() - t0)
    # the main run: N_CHAINS (1, MC3 off) or INDEPENDENT_CHAINS chains, all starting from the
    # warm-up's best sample, sharded over the ranks; with more than one, every chain's samples are
    # gathered to rank 0 at the end of the run (BatchedZoneMCMC.chain_statistics)
    n_main = max(int(mc["N_CHAINS"]), int(mc.get("INDEPENDENT_CHAINS", 1)))
    smp = BatchedZoneMCMC(n_chains=n_main, initial_sample=best, seed=seeds["sample"],
                          log_all_chains=n_main > 1, chain_params=mc.get("CHAIN_PARAMS"),
                          log_window=mc.get("LOG_WINDOW"), **common)
    smp.generate_samples(mc["N_STEPS"], mc["N_SAMPLES"])
    if getattr(smp, "rank", 0) != 0:
        # chain_idx[0] (the logged chain) lives on rank 0: the other ranks have nothing to write
        return smp.statistics, None
    per_chain = smp.chain_statistics or [smp.statistics]
    info = cfg["results"]["FILE_INFO"]
    if info == "n":
        fi = f"n{n_zones}"
    elif info == "s":
        fi = f"s{cfg['simulation']['STRENGTH']}a{cfg['simulation']['AREA']}"
    elif info == "i":
        fi = f"i{int(cfg['model']['INHERITANCE'])}"
    elif info == "p":
        # mcmc_setup.py:208 compares the PRIOR['universal'] dict with the string "uniform", which
        # is never equal: the reference always names these results p1
        fi = "p1"
    else:
        raise ValueError("file_info must be 'n', 's', 'i' or 'p'")
    pth = os.path.join(cfg["results"]["RESULTS_PATH"], name, fi)
    os.makedirs(pth, exist_ok=True)
    out = None
    truth = None  # eval_ground_truth once per run (its true_* keys copied into every chain's stats)
    for c, chain_stats in enumerate(per_chain):
        # chain 0: the reference's files; chain c > 0: the same files with a _chain<c> suffix
        sfx = "" if c == 0 else f"_chain{c}"
        paths = {"parameters": os.path.join(pth, f"stats_{fi}_{run}{sfx}.txt"),
                 "areas": os.path.join(pth, f"areas_{fi}_{run}{sfx}.txt")}
        if c == 0:  # the ground-truth files: once per run
            paths.update({"gt": os.path.join(pth, "ground_truth", "stats.txt"),
                          "gt_areas": os.path.join(pth, "ground_truth", "areas.txt")})
        main_stats = smp.statistics
        smp.statistics = chain_stats
        try:
            if "sample_weights" in chain_stats:
                contribution_per_area(smp)
                stats = rank_areas(match_areas(smp.statistics))
            else:
                # a chain logged without its parameters (ChainLog): zones matched, no per-zone
                # contributions to rank them by, no parameter columns (io.samples2file)
                stats = match_areas(dict(smp.statistics, acceptance_ratio=main_stats["acceptance_ratio"]))
        finally:
            smp.statistics = main_stats
        if getattr(data, "is_simulated", False):  # MCMC.save_samples (mcmc_setup.py:227-229)
            if truth is None:
                truth = eval_ground_truth(smp, data, bool(cfg["model"]["INHERITANCE"]), {})
                os.makedirs(os.path.dirname(paths["gt"]), exist_ok=True)
            stats.update(truth)
        io.samples2file(stats, data, cfg, paths)
        if c == 0:
            out = (stats, paths)
    stats = out[0]
    logger.info("sampling: %d steps x %d chain(s), acceptance %.3f, %.2f s; results in %s", mc["N_STEPS"],
                len(per_chain), stats["acceptance_ratio"], stats["sampling_time"], pth)
    return out


def main(argv=None):
    import argparse
    p = argparse.ArgumentParser(description="sBayes experiment on the GPU (batched sampler)")
    p.add_argument("config")
    p.add_argument("--name", default=None, help="experiment name (results sub-directory)")
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--device", type=int, default=None)
    p.add_argument("--set", default=None, help="JSON object merged into the config (custom settings)")
    p.add_argument("--chains", type=int, default=None,
                   help="independent main-run chains (mcmc.INDEPENDENT_CHAINS; MC3 stays off): chain 0 "
                        "writes the reference's results files, chain c > 0 the same files with a _chain<c> "
                        "suffix; the chains are sharded over the ranks and gathered to rank 0 at the end")
    p.add_argument("--chain-params", default=None,
                   help="with --chains: the chains (besides chain 0) whose parameters are logged too, "
                        "'all' or comma-separated global chain ids (mcmc.CHAIN_PARAMS); the others log "
                        "zones, log-likelihood and log prior only")
    p.add_argument("--log-window", type=int, default=None, help=argparse.SUPPRESS)
    p.add_argument("--jobs", choices=["concurrent", "sequential"], default="concurrent",
                   help="the N_RUNS x N_AREAS jobs: all at once, each on a thread and HIP stream of its own "
                        "(default), or one after another as the reference's cli.py; the files are the same")
    p.add_argument("--shard", choices=["auto", "jobs", "chains"], default="auto",
                   help="under torchrun: give each rank whole jobs ('jobs': job i on rank i %% world) or "
                        "split every job's chains over the ranks ('chains'); auto: jobs when there are at "
                        "least as many jobs as ranks")
    p.add_argument("--sim-data", default=None,
                   help="simulation config: the simulated data and its ground truth (.npz, SimulatedData.from_npz)")
    a = p.parse_args(argv)
    rank, device = init_distributed(a.device)
    logging.basicConfig(level=logging.INFO if rank == 0 else logging.WARNING, format="%(message)s")
    logger = logging.getLogger("sbz")
    custom = json.loads(a.set) if a.set else {}
    if a.chains is not None:
        custom.setdefault("mcmc", {})["INDEPENDENT_CHAINS"] = a.chains
    if a.chain_params is not None:
        custom.setdefault("mcmc", {})["CHAIN_PARAMS"] = (
            "all" if a.chain_params == "all" else [int(c) for c in a.chain_params.split(",") if c])
    if a.log_window is not None:
        custom.setdefault("mcmc", {})["LOG_WINDOW"] = a.log_window
    config, _ = load_config(a.config, custom or None, simulated=a.sim_data is not None)
    name = a.name or time.strftime("%Y%m%d-%H%M%S")
    data = SimulatedData.from_npz(a.sim_data) if a.sim_data else ExperimentData(config)
    for line in data.log:
        logger.info(line)
    n_areas = config["model"]["N_AREAS"]
    sweep = n_areas if isinstance(n_areas, list) else [n_areas]
    if not all(isinstance(n, int) for n in sweep):
        raise ValueError(f"N_AREAS must be an integer or a list of integers, got {n_areas!r} "
                         "(set it with --set '{\"model\": {\"N_AREAS\": 3}}')")
    name = _broadcast_name(name)
    seed = agree_seed(a.seed)
    jobs = [(run, int(n)) for run in range(config["mcmc"]["N_RUNS"]) for n in sweep]
    try:
        run_jobs(config, data, jobs, name, seed, device, logger, shard=a.shard,
                 concurrent=a.jobs == "concurrent")
    except BaseException:
        # no barrier: the other ranks may be waiting in a different collective; leave the group
        # and exit non-zero so the launcher tears the job down
        _finish_distributed(ok=False)
        raise
    _finish_distributed(ok=True)
    return 0


def run_jobs(config, data, jobs, name, seed, device=None, logger=None, shard="auto", concurrent=True):
    """The (run, n_zones) jobs of an experiment (cli.py:71-84 runs them one after another).

    concurrent: every job of this process at once, each on a thread of its own with its own HIP
    stream (torch's current stream is per thread, and every launch of a job goes to it), so the
    jobs' launches share the GPU (one chain per job occupies one CU of 256).  Under torchrun
    (WORLD_SIZE > 1) with shard 'jobs' (or 'auto' and at least as many jobs as ranks) job i runs
    whole on rank i % world in a one-rank group (no collective inside a job); with 'chains' every
    job's chains are split over all ranks (the jobs then run one after another: their collectives
    must not interleave).  A job's files do not depend on any of this (run_experiment).  Returns
    this process's results in job order (None for another rank's jobs)."""
    from .parallel import _dist
    d = _dist()
    world = d.get_world_size() if d is not None else 1
    rank = d.get_rank() if d is not None else 0
    group = None
    mine = list(range(len(jobs)))
    if world > 1 and (shard == "jobs" or (shard == "auto" and len(jobs) >= world)):
        groups = [d.new_group([r]) for r in range(world)]  # every rank creates every group
        group = groups[rank]
        mine = [i for i in range(len(jobs)) if i % world == rank]
    elif world > 1:
        concurrent = False
    results = [None] * len(jobs)

    def job(i):
        run, n = jobs[i]
        return run_experiment(config, data, n, run=run, name=name, seed=seed, device=device,
                              logger=logger, group=group)

    if not concurrent or len(mine) <= 1:
        for i in mine:
            results[i] = job(i)
        return results
    import threading
    import torch
    dev = device if device is not None else torch.cuda.current_device()
    errors = []

    def work(i):
        try:
            with torch.cuda.device(dev), torch.cuda.stream(torch.cuda.Stream(dev)):
                results[i] = job(i)
                torch.cuda.current_stream().synchronize()
        except BaseException as e:  # re-raised in the calling thread
            errors.append((i, e))

    threads = [threading.Thread(target=work, args=(i,), name=f"sbz-job-{i}") for i in mine]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0][1]
    return results


def init_distributed(device=None):
    """One process per GPU under torchrun (WORLD_SIZE > 1): bind this rank's GPU from LOCAL_RANK
    and join the process group (nccl = RCCL over xGMI; gloo when no GPU is visible) before any GPU
    call.  The batched samplers then shard the chains over the ranks.  Returns (rank, device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, device
    import torch
    import torch.distributed as dist
    gpu = torch.cuda.is_available()
    # more ranks than GPUs (a rehearsal on a one-GPU box) share the GPUs round-robin; RCCL
    # refuses two ranks on one device, so such a run sets SBZ_DIST_BACKEND=gloo
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count() if gpu else 1)
    if device is None:
        device = local
    if not dist.is_initialized():
        if gpu:
            torch.cuda.set_device(device)
        dist.init_process_group(os.environ.get("SBZ_DIST_BACKEND", "nccl" if gpu else "gloo"))
    return dist.get_rank(), device


def _broadcast_name(name):
    """Rank 0's experiment name (the default is a timestamp, which ranks may disagree on)."""
    from .parallel import _dist
    d = _dist()
    if d is None or d.get_world_size() == 1:
        return name
    box = [name]
    d.broadcast_object_list(box, src=0)
    return box[0]


def _finish_distributed(ok=True):
    """Leave the process group: after a barrier on success; without one after a failure (a
    barrier could pair with a peer's pending all_reduce / broadcast and hang or mismatch)."""
    from .parallel import _dist
    d = _dist()
    if d is not None and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        if ok:
            d.barrier()
        d.destroy_process_group()
