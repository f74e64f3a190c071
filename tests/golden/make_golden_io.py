"""Capture golden vectors for the I/O row (contact_zones_amd/io.py, postprocessing.match_areas /
rank_areas) from the reference itself — BUILD CONTAINER ONLY (imports /root/reference via
refenv; writes tests/golden/io/*).

Inputs are data files the reference ships (experiments/balkan, experiments/south_america,
test/test_files), copied under tests/golden/io/data/ so the tests read the same bytes without
the reference.  Outputs:
  io_expected.npz   per dataset: what sbayes.util.read_features_from_csv returns (features as
                    obs codes, applicable states, names, families, locations, NA count, log),
                    the counts of read_universal_counts / read_inheritance_counts, and the
                    Delaunay network of compute_network (CSR + distance matrix)
  samples_in.npz    a seeded statistics dict (balkan names, 3 zones, 12 logged samples)
  stats_expected.txt / areas_expected.txt
                    the files sbayes.util.samples2file writes for it after
                    sbayes.postprocessing.match_areas and rank_areas (MCMC.save_samples order)
Run: python tests/golden/make_golden_io.py
"""
import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refenv  # noqa: E402

OUT = os.path.join(HERE, "io")
DATA = os.path.join(OUT, "data")

DATASETS = {
    "balkan": ("experiments/balkan/data/features/features.csv",
               "experiments/balkan/data/features/feature_states.csv",
               "experiments/balkan/data/prior_universal/universal_counts.csv",
               {"Greek": "experiments/balkan/data/prior_inheritance/greek_counts.csv",
                "Romance": "experiments/balkan/data/prior_inheritance/romance_counts.csv",
                "Slavic": "experiments/balkan/data/prior_inheritance/slavic_counts.csv",
                "Turkish": "experiments/balkan/data/prior_inheritance/turkish_counts.csv"}),
    "south_america": ("experiments/south_america/data/features/features.csv",
                      "experiments/south_america/data/features/feature_states.csv",
                      "experiments/south_america/data/prior_universal/universal_counts.csv",
                      {"Arawak": "experiments/south_america/data/prior_inheritance/arawak_counts.csv",
                       "Panoan": "experiments/south_america/data/prior_inheritance/panoan_counts.csv",
                       "Quechuan": "experiments/south_america/data/prior_inheritance/quechuan_counts.csv",
                       "Tucanoan": "experiments/south_america/data/prior_inheritance/tucanoan_counts.csv",
                       "Tupian": "experiments/south_america/data/prior_inheritance/tupian_counts.csv"}),
    "test_files": ("test/test_files/features.csv", "test/test_files/feature_states_expected.csv",
                   None, {}),
}


def local(rel):
    """Copy a reference data file under io/data/ (same relative path) and return the copy."""
    dst = os.path.join(DATA, rel)
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    shutil.copyfile(os.path.join(refenv.REFERENCE, rel), dst)
    return dst


def rel(path):
    return os.path.relpath(path, DATA)


def capture_readers(out):
    from sbayes import preprocessing, util
    for name, (feat, states, uni, inh) in DATASETS.items():
        feat_l, states_l = local(feat), local(states)
        (sites, site_names, features, feature_names, state_names, applicable, families,
         family_names, log) = util.read_features_from_csv(feat_l, states_l)
        features = np.asarray(features, bool)
        obs = np.where(features.any(-1), features.argmax(-1), -1).astype(np.int8)
        p = name + "_"
        out[p + "obs"] = obs
        out[p + "applicable"] = np.asarray(applicable, bool)
        out[p + "locations"] = np.asarray(sites["locations"], np.float64)
        out[p + "families"] = np.asarray(families, np.int64).reshape(len(family_names["external"]), -1)
        meta = {"feature_names": [str(x) for x in feature_names["external"]],
                "state_names": [[str(s) for s in st] for st in state_names["external"]],
                "family_names": [str(x) for x in family_names["external"]],
                "site_ids": [str(x) for x in site_names["external"]],
                "site_names": [str(x) for x in sites["names"]],
                "log": log.replace(feat_l, "<FEATURES>"),
                "files": {"features": rel(feat_l), "feature_states": rel(states_l)}}
        if uni is not None:
            uni_l = local(uni)
            counts, ulog = preprocessing.read_universal_counts(
                feature_names=feature_names, state_names=state_names, file=uni_l,
                file_type="counts_file", feature_states_file=states_l)
            out[p + "universal_counts"] = np.asarray(counts)
            inh_l = {k: local(v) for k, v in inh.items()}
            icounts, ilog = preprocessing.read_inheritance_counts(
                family_names=family_names, feature_names=feature_names, state_names=state_names,
                files=inh_l, file_type="counts_file", feature_states_file=states_l)
            out[p + "inheritance_counts"] = np.asarray(icounts)
            meta["files"]["universal"] = rel(uni_l)
            meta["files"]["inheritance"] = {k: rel(v) for k, v in inh_l.items()}
        net = preprocessing.compute_network(sites)
        adj = net["adj_mat"].tocsr()
        out[p + "adj_indptr"] = adj.indptr.astype(np.int64)
        out[p + "adj_indices"] = adj.indices.astype(np.int64)
        out[p + "dist_mat"] = np.asarray(net["dist_mat"], np.float64)
        out[p + "meta"] = np.array(json.dumps(meta))


def capture_results_files():
    """samples2file after match_areas + rank_areas on a seeded statistics dict."""
    import types

    from sbayes import postprocessing, util
    rng = np.random.default_rng(11)
    feat, states = DATASETS["balkan"][0], DATASETS["balkan"][1]
    (_, _, features, feature_names, state_names, applicable, families, family_names,
     _) = util.read_features_from_csv(os.path.join(DATA, feat), os.path.join(DATA, states))
    N, F, S = np.asarray(features).shape
    Z, n, Fam = 3, 12, len(family_names["external"])
    stats = {"sample_zones": [], "sample_weights": [], "sample_p_global": [], "sample_p_zones": [],
             "sample_p_families": [], "sample_likelihood": [], "sample_prior": [],
             "sample_lh_single_zones": [], "sample_prior_single_zones": [],
             "sample_posterior_single_zones": []}
    for _ in range(n):
        lab = rng.integers(0, Z + 2, size=N)
        stats["sample_zones"].append(np.stack([lab == z for z in range(Z)]))
        stats["sample_weights"].append(rng.dirichlet(np.ones(3), size=F))
        stats["sample_p_global"].append(rng.dirichlet(np.ones(S), size=(1, F)))
        stats["sample_p_zones"].append(rng.dirichlet(np.ones(S), size=(Z, F)))
        stats["sample_p_families"].append(rng.dirichlet(np.ones(S), size=(Fam, F)))
        stats["sample_likelihood"].append(float(-rng.random() * 1000))
        stats["sample_prior"].append(float(-rng.random() * 10))
        lh, pr = list(-rng.random(Z) * 500), list(-rng.random(Z) * 5)
        stats["sample_lh_single_zones"].append(lh)
        stats["sample_prior_single_zones"].append(pr)
        stats["sample_posterior_single_zones"].append([a + b for a, b in zip(lh, pr)])
    np.savez_compressed(os.path.join(OUT, "samples_in.npz"),
                        **{k: np.asarray(v) for k, v in stats.items()})
    config = {"model": {"INHERITANCE": True, "N_AREAS": Z}, "mcmc": {"N_STEPS": 1200, "N_SAMPLES": n}}
    data = types.SimpleNamespace(feature_names=feature_names, state_names=state_names,
                                 family_names=family_names, is_simulated=False)
    stats = postprocessing.match_areas(stats)
    stats = postprocessing.rank_areas(stats)
    paths = {"parameters": os.path.join(OUT, "stats_expected.txt"),
             "areas": os.path.join(OUT, "areas_expected.txt")}
    util.samples2file(stats, data, config, paths)


def capture_model_setup(out):
    """The reference's Experiment -> Data -> MCMC setup for the Balkan and South America configs
    (N_AREAS set to 3): the verified config's operator table (MCMC.steps_per_operator) and the
    'counts' priors' pseudo-counts and Dirichlet concentrations (model.py:538-680)."""
    from sbayes.experiment_setup import Experiment
    from sbayes.load_data import Data
    from sbayes.mcmc_setup import MCMC
    cwd = os.getcwd()
    for name, rel_dir in (("balkan", "experiments/balkan"), ("south_america", "experiments/south_america")):
        local(rel_dir + "/config.json")  # the config the tests load (data paths relative to it)
        d = refenv.scratch_copy(rel_dir)
        os.chdir(d)  # load_universal_counts writes universal_counts.csv into the CWD
        try:
            custom = {"model": {"N_AREAS": 3}}
            cfg_path = os.path.join(d, "config.json")
            with open(cfg_path) as f:
                raw = json.load(f)
            data_cfg = raw.get("data", {})
            for low, up in (("features", "FEATURES"), ("feature_states", "FEATURE_STATES")):
                if low in data_cfg:
                    custom.setdefault("data", {})[up] = data_cfg[low]
            if name == "south_america":
                custom.setdefault("data", {})["CRS"] = None
            exp = Experiment(experiment_name="golden", log=False)
            exp.load_config(config_file=cfg_path, custom_settings=custom)
            data = Data(experiment=exp)
            data.load_features()
            data.load_universal_counts()
            data.load_inheritance_counts()
            mcmc = MCMC(data=data, experiment=exp)
            p = "setup_" + name + "_"
            out[p + "ops"] = np.array(json.dumps(mcmc.ops))
            out[p + "steps"] = np.array(json.dumps(exp.config["mcmc"]["STEPS"]))
            pr = mcmc.model.prior
            F, S = data.states.shape
            ag = np.zeros((F, S))
            for f in range(F):
                ag[f, data.states[f]] = pr.prior_p_global.dirichlet[f]
            out[p + "alpha_global"] = ag
            out[p + "counts_global"] = np.asarray(pr.prior_p_global.counts, np.float64)
            fam = pr.prior_p_families
            n_fam = len(fam.dirichlet)
            af = np.zeros((n_fam, F, S))
            for k in range(n_fam):
                for f in range(F):
                    af[k, f, data.states[f]] = fam.dirichlet[k][f]
            out[p + "alpha_fam"] = af
            out[p + "counts_fam"] = np.asarray(fam.counts, np.float64)
        finally:
            os.chdir(cwd)


SIM_CASES = {  # simulated-data result files: (experiment, simulation overrides, model config)
    "sim1": ("experiments/simulation/sim_exp1",
             {"I_CONTACT": 3, "E_CONTACT": 0.5, "STRENGTH": 1, "AREA": 4},
             {"N_AREAS": 2, "INHERITANCE": False}),
    "sim2": ("experiments/simulation/sim_exp2", {}, {"N_AREAS": 1, "INHERITANCE": True}),
}


def capture_results_files_simulated():
    """samples2file on simulated data (util.py:846-907): the ground-truth stats and areas files
    (collect_gt_for_writing / collect_gt_areas_for_writing, util.py:657-742) and the stats file's
    recall / precision columns (:811-825), for the reference's own simulations sim_exp1 (no
    inheritance; model with 2 zones against 1 true zone) and sim_exp2 (simulated inheritance),
    with a seeded statistics dict and the simulation's true parameters."""
    import random
    import types
    from sbayes import util
    from sbayes.experiment_setup import Experiment
    from sbayes.simulation import Simulation
    for case, (rel_dir, sim_over, model) in SIM_CASES.items():
        exp_dir = refenv.scratch_copy(rel_dir)
        np.random.seed(1)
        random.seed(1)
        exp = Experiment(experiment_name="golden", config_file=os.path.join(exp_dir, "config.json"), log=False)
        exp.load_config(os.path.join(exp_dir, "config.json"), custom_settings={"simulation": sim_over} if sim_over else None)
        sim = Simulation(experiment=exp)
        sim.run_simulation()
        Z, inh = model["N_AREAS"], model["INHERITANCE"]
        sim_inh = bool(exp.config["simulation"]["INHERITANCE"])
        N, F = np.asarray(sim.features).shape[:2]
        S = np.asarray(sim.features).shape[2]
        fam_names = sim.family_names if sim_inh else {"external": [], "internal": []}
        Fam = len(fam_names["external"])
        rng = np.random.default_rng(21 if case == "sim1" else 22)
        n = 9
        C = 3 if inh else 2
        stats = {k: [] for k in ("sample_zones", "sample_weights", "sample_p_global", "sample_p_zones",
                                 "sample_p_families", "sample_likelihood", "sample_prior")}
        true_z = np.any(sim.areas, axis=0)
        for i in range(n):
            if i == 0:  # an empty sample: precision 0 / 0 = nan
                zones = np.zeros((Z, N), bool)
            else:  # zones that partly overlap the true one
                lab = np.where(true_z & (rng.random(N) < 0.7), rng.integers(0, Z, N), -1)
                lab[rng.random(N) < 0.02] = Z - 1
                zones = np.stack([lab == z for z in range(Z)])
            stats["sample_zones"].append(zones)
            stats["sample_weights"].append(rng.dirichlet(np.ones(C), size=F))
            stats["sample_p_global"].append(rng.dirichlet(np.ones(S), size=(1, F)))
            stats["sample_p_zones"].append(rng.dirichlet(np.ones(S), size=(Z, F)))
            stats["sample_p_families"].append(rng.dirichlet(np.ones(S), size=(max(Fam, 1), F))[:Fam])
            stats["sample_likelihood"].append(float(-rng.random() * 1000))
            stats["sample_prior"].append(float(-rng.random() * 10))
        if not inh:
            del stats["sample_p_families"]
        w = np.asarray(sim.weights, np.float64)
        stats["true_zones"] = sim.areas
        stats["true_weights"] = w.copy() if inh else w[:, :2] / w[:, :2].sum(-1, keepdims=True)
        stats["true_p_global"] = sim.p_universal[np.newaxis, ...]
        stats["true_p_zones"] = sim.p_contact
        if sim_inh:
            stats["true_p_families"] = sim.p_inheritance
        stats["true_ll"] = float(-rng.random() * 1e4)
        stats["true_prior"] = float(-rng.random() * 10)
        Zt = np.asarray(sim.areas).shape[0]
        stats["true_lh_single_zones"] = list(-rng.random(Zt) * 500)
        stats["true_prior_single_zones"] = list(-rng.random(Zt) * 5)
        stats["true_posterior_single_zones"] = [a + b for a, b in zip(stats["true_lh_single_zones"],
                                                                      stats["true_prior_single_zones"])]
        np.savez_compressed(os.path.join(OUT, f"samples_{case}_in.npz"),
                            **{k: np.asarray(v) for k, v in stats.items()})
        meta = {"feature_names": [str(x) for x in sim.feature_names["external"]],
                "state_names": [[str(s) for s in st] for st in sim.state_names["external"]],
                "family_names": [str(x) for x in fam_names["external"]],
                "config": {"model": model, "simulation": {"INHERITANCE": sim_inh},
                           "mcmc": {"N_STEPS": 900, "N_SAMPLES": n}}}
        with open(os.path.join(OUT, f"samples_{case}_meta.json"), "w") as f:
            json.dump(meta, f)
        config = {"model": dict(model), "simulation": {"INHERITANCE": sim_inh},
                  "mcmc": {"N_STEPS": 900, "N_SAMPLES": n}}
        data = types.SimpleNamespace(feature_names=sim.feature_names, state_names=sim.state_names,
                                     family_names=fam_names, areas=sim.areas, is_simulated=True)
        paths = {"parameters": os.path.join(OUT, f"stats_{case}_expected.txt"),
                 "areas": os.path.join(OUT, f"areas_{case}_expected.txt"),
                 "gt": os.path.join(OUT, f"gt_stats_{case}_expected.txt"),
                 "gt_areas": os.path.join(OUT, f"gt_areas_{case}_expected.txt")}
        util.samples2file(stats, data, config, paths)


def main():
    refenv.setup()
    os.makedirs(OUT, exist_ok=True)
    out = {}
    capture_readers(out)
    capture_model_setup(out)
    np.savez_compressed(os.path.join(OUT, "io_expected.npz"), **out)
    capture_results_files()
    capture_results_files_simulated()
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__" and sys.argv[1:] == ["simulated"]:
    refenv.setup()
    capture_results_files_simulated()
elif __name__ == "__main__":
    main()
