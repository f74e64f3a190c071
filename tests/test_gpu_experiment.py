"""An sBayes experiment config end to end on the GPU (contact_zones_amd/experiment.py): the
Balkan config (tests/golden/io/data, the reference's data files) through warm-up, sampling,
per-zone contributions, match / rank and the results files."""
import os

import numpy as np
import pytest

from contact_zones_amd import experiment, io

pytestmark = pytest.mark.gpu
CFG = os.path.join(os.path.dirname(__file__), "golden", "io", "data", "experiments", "balkan", "config.json")


def _short(tmp_path, **model):
    return {"model": {"N_AREAS": 2, **model},
            "mcmc": {"N_STEPS": 2000, "N_SAMPLES": 20, "WARM_UP": {"N_WARM_UP_STEPS": 400, "N_WARM_UP_CHAINS": 6}},
            "results": {"RESULTS_PATH": str(tmp_path)}}


def _read_stats(path):
    with open(path) as f:
        head = f.readline().rstrip("\r\n").split("\t")
        rows = [line.rstrip("\r\n").split("\t") for line in f]
    return head, rows


@pytest.mark.parametrize("source", [True, False])
def test_balkan_experiment_end_to_end(gpu_available, tmp_path, source):
    cfg, _ = experiment.load_config(CFG, _short(tmp_path, SAMPLE_SOURCE=source))
    data = experiment.ExperimentData(cfg)
    stats, paths = experiment.run_experiment(cfg, data, 2, name="t", seed=3)
    head, rows = _read_stats(paths["parameters"])
    t = data.table
    assert head == io.stats_columns(t.feature_names, t.state_names, t.family_names, 2, True, False, True)
    assert len(rows) == 20 and all(len(r) == len(head) for r in rows)
    assert [int(r[0]) for r in rows] == [100 * i for i in range(20)]
    with open(paths["areas"]) as f:
        areas = [line.rstrip("\n").split("\t") for line in f]
    assert len(areas) == 20 and all(len(a) == 2 and len(a[0]) == t.n_sites for a in areas)
    zones = np.array([[[c == "1" for c in z] for z in a] for a in areas])
    assert not np.any(zones.sum(axis=1) > 1)                          # disjoint zones
    sizes = zones.sum(axis=2)
    assert np.all((sizes >= cfg["model"]["MIN_M"]) & (sizes <= cfg["model"]["MAX_M"]))
    np.testing.assert_array_equal(sizes, np.array([[int(r[4]), int(r[5])] for r in rows]))
    ll = np.array([float(r[2]) for r in rows])
    assert np.all(np.isfinite(ll))
    if not source:
        # mixture mode: every logged likelihood equals the oracle's full evaluation of that sample
        from oracle import lik_numpy
        for s in range(20):
            zos = np.full(t.n_sites, 255, np.uint8)
            for z in range(2):
                zos[stats["sample_zones"][s][z]] = z
            ref = lik_numpy.loglik(t.obs, t.fam_of_site, zos, stats["sample_weights"][s],
                                   stats["sample_p_global"][s][0], stats["sample_p_zones"][s],
                                   stats["sample_p_families"][s], inheritance=True)
            assert ll[s] == pytest.approx(ref, rel=1e-9)


def test_balkan_experiment_geo_prior(gpu_available, tmp_path):
    """A 'cost_based' geo prior (the distance matrix as costs): every logged prior equals the host
    restatement of the reference's Prior (PriorSpec.log_prior, scipy MST) on that sample."""
    cfg, _ = experiment.load_config(CFG, {**_short(tmp_path, SAMPLE_SOURCE=False),
                                          "model": {"N_AREAS": 2, "SAMPLE_SOURCE": False,
                                                    "PRIOR": {"geo": {"type": "cost_based", "scale": 2.0}}}})
    data = experiment.ExperimentData(cfg)
    spec, _ = experiment.build_priors(cfg, data)
    stats, _ = experiment.run_experiment(cfg, data, 2, name="g", seed=5)
    t = data.table
    # match_areas / rank_areas relabel the zones after sampling (the logged priors keep the
    # sampling-time labels, as the reference's), and only the last zone enters the geo prior:
    # the logged prior is the prior of one of the two labelings
    n_geo = 0
    for s in range(len(stats["sample_zones"])):
        refs = []
        for order in ((0, 1), (1, 0)):
            zos = np.full((1, t.n_sites), 255, np.uint8)
            for z in range(2):
                zos[0, stats["sample_zones"][s][order[z]]] = z
            refs.append(spec.log_prior(zos, stats["sample_p_global"][s][0][None],
                                       stats["sample_p_families"][s][None], data.states, 2, True)[0])
        assert any(stats["sample_prior"][s] == pytest.approx(r, rel=1e-9, abs=1e-9) for r in refs)
        n_geo += refs[0] != refs[1]
    assert n_geo > 0  # the geo term differs between the zones


def test_runs_are_independent_and_reproducible(gpu_available, tmp_path):
    """With --seed, the N_RUNS replicates draw from different streams (run index in the seed
    derivation) and the main run's draws differ from its warm-up's; the same (seed, run) is
    reproducible."""
    cfg, _ = experiment.load_config(CFG, _short(tmp_path, SAMPLE_SOURCE=False))
    data = experiment.ExperimentData(cfg)
    a, _ = experiment.run_experiment(cfg, data, 2, run=0, name="r", seed=11)
    b, _ = experiment.run_experiment(cfg, data, 2, run=1, name="r", seed=11)
    c, _ = experiment.run_experiment(cfg, data, 2, run=0, name="r2", seed=11)
    assert a["sample_likelihood"] != b["sample_likelihood"]
    assert a["sample_likelihood"] == c["sample_likelihood"]


SIM_CFG = os.path.join(os.path.dirname(__file__), "golden", "io", "data", "experiments", "simulation",
                       "sim_exp1", "config.json")


@pytest.mark.parametrize("source", [False, True])
def test_simulated_experiment_ground_truth(gpu_available, tmp_path, source):
    """The reference's sim_exp1 config on its own simulation (tests/golden/data_cfg1_sim.npz, the
    truth of tests/golden/truth_sim.npz): MCMC.save_samples' simulated branch writes the
    ground-truth stats / areas files, whose likelihood and prior equal the reference's
    eval_ground_truth values, and the stats file carries recall / precision against the truth."""
    from conftest import load_golden
    d, t = load_golden("data_cfg1_sim"), load_golden("truth_sim")
    data = experiment.SimulatedData(d["obs"], d["states"], d["locations"], t["areas"], t["data_weights"],
                                    t["p_universal"], t["p_contact"])
    np.testing.assert_array_equal(data.network["adj_mat"].indptr, d["adj_indptr"])
    np.testing.assert_array_equal(data.network["adj_mat"].indices, d["adj_indices"])
    cfg, _ = experiment.load_config(SIM_CFG, {
        "simulation": {"I_CONTACT": 3, "E_CONTACT": 0.5, "STRENGTH": 1, "AREA": 4},
        "model": {"SAMPLE_SOURCE": source},
        "mcmc": {"N_STEPS": 1500, "N_SAMPLES": 15, "WARM_UP": {"N_WARM_UP_STEPS": 300, "N_WARM_UP_CHAINS": 4}},
        "results": {"RESULTS_PATH": str(tmp_path)}}, simulated=True)
    stats, paths = experiment.run_experiment(cfg, data, 1, name="sim", seed=4)
    assert os.path.dirname(paths["parameters"]).endswith(os.path.join("sim", "s1a4"))
    head, rows = _read_stats(paths["gt"])
    assert len(rows) == 1 and len(rows[0]) == len(head)
    gt = dict(zip(head, rows[0]))
    assert float(gt["likelihood"]) == pytest.approx(float(t["true_ll"]), rel=1e-9)
    assert float(gt["prior"]) == float(t["true_prior"])
    assert float(gt["lh_a1"]) == pytest.approx(float(t["true_lh_single_zones"][0]), rel=1e-9)
    with open(paths["gt_areas"]) as f:
        assert f.read() == io.format_area_columns(t["areas"])
    head, rows = _read_stats(paths["parameters"])
    assert head[-5:-3] == ["recall", "precision"] and len(rows) == 15
    for s, r in enumerate(rows):
        rec, prec = io.recall_precision(stats["sample_zones"][s], t["areas"])
        assert float(r[-5]) == rec and float(r[-4]) == prec
