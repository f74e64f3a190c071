"""Time the reference's own sampler (sbayes ZoneMCMC, one chain, one CPU core) on the Balkan and
South America configs — BUILD CONTAINER ONLY (imports /root/reference through
tests/golden/refenv.py).  Prints MH steps/s per core; the numbers are recorded in DESIGN.md next
to the GPU's (bench.py real-data legs)."""
import json
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import refenv  # noqa: E402


def run(name, n_zones, steps, seed=1):
    from sbayes.experiment_setup import Experiment
    from sbayes.load_data import Data
    from sbayes.mcmc_setup import MCMC
    from sbayes.sampling.zone_sampling import ZoneMCMC
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
        exp = Experiment(experiment_name="timing", log=False)
        exp.load_config(config_file="config.json", custom_settings=custom)
        data = Data(experiment=exp)
        data.load_features()
        data.load_universal_counts()
        data.load_inheritance_counts()
        mcmc = MCMC(data=data, experiment=exp)
        mc = exp.config["mcmc"]
        np.random.seed(seed)
        random.seed(seed)
        smp = ZoneMCMC(data=data, model=mcmc.model, n_chains=1, operators=mcmc.ops,
                       var_proposal=mc["PROPOSAL_PRECISION"], p_grow_connected=mc["P_GROW_CONNECTED"],
                       initial_size=mc["M_INITIAL"], logger=None)
        t0 = time.perf_counter()
        smp.generate_samples(steps, max(1, steps // 10))
        el = time.perf_counter() - t0
        return {"config": name, "n_zones": n_zones, "steps": steps, "seconds": el,
                "steps_per_sec_per_core": steps / el}
    finally:
        os.chdir(cwd)


def run_cfg5(seconds=20.0, seed=5):
    """The bench's sampler workload (bench.py sampler_leg: cfg5 2000 x 500 x 10, Z = 8, Fam = 4,
    SAMPLE_SOURCE = false, default STEPS / PROPOSAL_PRECISION / MIN_M / MAX_M / M_INITIAL /
    P_GROW_CONNECTED, the same synthetic data) on the reference's own ZoneMCMC (one chain, one
    core, caching likelihood) and on the numpy restatement bench.py's CPU baseline times
    (oracle/mh_numpy.step with drawn decisions), each for about `seconds`: steps/s per core and
    their ratio."""
    import types
    import bench
    from contact_zones_amd import packing
    from sbayes.model import Model
    from sbayes.preprocessing import compute_network
    from sbayes.sampling.zone_sampling import ZoneMCMC
    a = types.SimpleNamespace(sites=2000, features=500, states=10, zones=8, families=4, zone_size=50)
    obs, fam = bench.make_shared(a, np.random.default_rng(seed))
    N, F, S, Z, Fam = a.sites, a.features, a.states, a.zones, a.families
    indptr, indices = bench.make_network(N, np.random.default_rng(seed + 17))
    import scipy.sparse as sp
    adj = sp.csr_matrix((np.ones(indices.size), indices, indptr), shape=(N, N))
    net = compute_network({"id": list(range(N)), "locations": np.random.default_rng(1).random((N, 2)),
                           "names": [str(i) for i in range(N)]})
    net["adj_mat"] = adj  # the bench's network
    data = types.SimpleNamespace(features=packing.obs_to_features(obs, S), states=np.ones((F, S), bool),
                                 network=net, families=packing.index_to_groups(fam, Fam))
    prior = {"geo": {"type": "uniform"}, "area_size": {"type": "none"}, "weights": {"type": "uniform"},
             "universal": {"type": "uniform"}, "inheritance": {"type": "uniform"}, "contact": {"type": "uniform"}}
    cfg = {"N_AREAS": Z, "MIN_M": bench.MH_MIN_M, "MAX_M": bench.MH_MAX_M, "INHERITANCE": True,
           "SAMPLE_SOURCE": False, "PRIOR": prior}
    np.random.seed(seed)
    random.seed(seed)
    model = Model(data=data, config=cfg)
    smp = ZoneMCMC(data=data, model=model, n_chains=1, operators=bench.mh_operators(),
                   var_proposal=bench.MH_PRECISION, p_grow_connected=bench.MH_P_GROW,
                   initial_size=bench.MH_M_INITIAL, logger=None)
    steps = 50
    t0 = time.perf_counter()
    smp.generate_samples(steps, 10)  # (initial sample, first evaluations, the caches filled)
    warm = time.perf_counter() - t0
    steps = max(steps, int(steps * seconds / max(warm, 1e-3)))  # a run of about `seconds`
    np.random.seed(seed)
    random.seed(seed)
    smp = ZoneMCMC(data=data, model=model, n_chains=1, operators=bench.mh_operators(),
                   var_proposal=bench.MH_PRECISION, p_grow_connected=bench.MH_P_GROW,
                   initial_size=bench.MH_M_INITIAL, logger=None)
    t0 = time.perf_counter()
    smp.generate_samples(steps, max(1, steps // 10))
    el = time.perf_counter() - t0
    ref = steps / el
    shape = {"sites": N, "features": F, "states": S, "zones": Z, "families": Fam, "zone_size": 50, "seed": seed}
    port = bench._cpu_sampler_worker(shape, seconds, seed * 7919)
    por = port["n"] / port["seconds"]
    return {"case": "cfg5 2000x500x10 Z8 Fam4, SAMPLE_SOURCE = false, bench sampler operators",
            "reference_steps_per_sec_per_core": ref, "reference_steps": steps, "reference_seconds": el,
            "restatement_steps_per_sec_per_core": por, "restatement_steps": port["n"],
            "restatement_over_reference": por / ref,
            "threads": {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS")},
            "host_cpu_count": os.cpu_count(),
            "where": "build container CPU, 1 thread each (tools/time_reference_sampler.py cfg5)"}


def run_cfg5src(seconds=20.0, seed=5):
    """The bench's source-mode leg workload (bench.py source_sampler_leg: cfg5 2000 x 500 x 10, Z = 8,
    Fam = 4, SAMPLE_SOURCE = true, config/default_config.json STEPS with source 0, the same synthetic
    data and network) on the reference's own ZoneMCMC, one chain on one core, for about `seconds`:
    MH steps/s per core.  The reference never travels to the GPU box, so this is the build
    container's figure (no restatement of the source-mode Gibbs operators is timed on the box)."""
    import types
    import bench
    from contact_zones_amd import packing
    from sbayes.model import Model
    from sbayes.preprocessing import compute_network
    from sbayes.sampling.zone_sampling import ZoneMCMC
    N, F, S, Z, Fam = 2000, 500, 10, 8, 4
    rng = np.random.default_rng(seed)  # as source_sampler_leg draws its data and network
    obs = rng.integers(0, S, size=(N, F)).astype(np.int8)
    obs[rng.random((N, F)) < 0.02] = -1
    fam = rng.integers(0, Fam, size=N).astype(np.uint8)
    fam[rng.random(N) < 0.2] = 255
    from scipy.spatial import Delaunay
    indptr, indices = Delaunay(rng.random((N, 2))).vertex_neighbor_vertices
    import scipy.sparse as sp
    adj = sp.csr_matrix((np.ones(indices.size), indices, indptr), shape=(N, N))
    net = compute_network({"id": list(range(N)), "locations": np.random.default_rng(1).random((N, 2)),
                           "names": [str(i) for i in range(N)]})
    net["adj_mat"] = adj
    data = types.SimpleNamespace(features=packing.obs_to_features(obs, S), states=np.ones((F, S), bool),
                                 network=net, families=packing.index_to_groups(fam, Fam))
    prior = {"geo": {"type": "uniform"}, "area_size": {"type": "none"}, "weights": {"type": "uniform"},
             "universal": {"type": "uniform"}, "inheritance": {"type": "uniform"}, "contact": {"type": "uniform"}}
    cfg = {"N_AREAS": Z, "MIN_M": bench.MH_MIN_M, "MAX_M": bench.MH_MAX_M, "INHERITANCE": True,
           "SAMPLE_SOURCE": True, "PRIOR": prior}
    ops = {k: v for k, v in bench.src_operators(True).items() if v > 0}

    def sampler():
        np.random.seed(seed)
        random.seed(seed)
        model = Model(data=data, config=cfg)
        return ZoneMCMC(data=data, model=model, n_chains=1, operators=ops, var_proposal=bench.MH_PRECISION,
                        p_grow_connected=bench.MH_P_GROW, initial_size=bench.MH_M_INITIAL, logger=None)
    steps = 20
    smp = sampler()
    t0 = time.perf_counter()
    smp.generate_samples(steps, 10)  # (initial sample with its sources, the caches filled)
    warm = time.perf_counter() - t0
    steps = max(steps, int(steps * seconds / max(warm, 1e-3)))
    smp = sampler()
    t0 = time.perf_counter()
    smp.generate_samples(steps, max(1, steps // 10))
    el = time.perf_counter() - t0
    return {"case": "cfg5 2000x500x10 Z8 Fam4, SAMPLE_SOURCE = true, default STEPS with source 0 "
                    "(bench.py sampler_source_mode's workload)",
            "reference_steps_per_sec_per_core": steps / el, "reference_steps": steps,
            "reference_seconds": el, "includes": "the run's initial sample (generate_initial_sample "
            "with its source draw) inside the timed generate_samples call",
            "threads": {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS")},
            "host_cpu_count": os.cpu_count(),
            "where": "build container CPU, 1 thread (tools/time_reference_sampler.py cfg5src)"}


if __name__ == "__main__":
    refenv.setup()
    if len(sys.argv) > 1 and sys.argv[1] == "cfg5src":
        sys.path.insert(0, ROOT)
        import contextlib
        with contextlib.redirect_stdout(sys.stderr):  # the reference's own progress prints
            res = run_cfg5src()
        print(json.dumps(res, indent=1), flush=True)
    elif len(sys.argv) > 1 and sys.argv[1] == "cfg5":
        sys.path.insert(0, ROOT)
        import contextlib
        with contextlib.redirect_stdout(sys.stderr):  # the reference's own progress prints
            res = run_cfg5()
        print(json.dumps(res, indent=1), flush=True)
    else:
        for name, z, steps in (("balkan", 3, 2000), ("south_america", 6, 1000)):
            print(json.dumps(run(name, z, steps)), flush=True)
