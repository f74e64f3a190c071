"""The I/O row against the reference's own outputs captured by
tests/golden/make_golden_io.py: the features / counts readers, the Delaunay network, the
feature-states tool (the reference's test fixture), and the results files of
MCMC.save_samples (match_areas, rank_areas, samples2file) byte for byte."""
import json
import os
import types

import numpy as np
import pytest

from contact_zones_amd import io, postprocessing

GOLD = os.path.join(os.path.dirname(__file__), "golden", "io")
DATA = os.path.join(GOLD, "data")
DATASETS = ["balkan", "south_america", "test_files"]


@pytest.fixture(scope="module")
def gold():
    with np.load(os.path.join(GOLD, "io_expected.npz")) as z:
        return {k: z[k] for k in z.files}


def meta_of(gold, name):
    return json.loads(str(gold[name + "_meta"]))


@pytest.mark.parametrize("name", DATASETS)
def test_read_features_packed_matches_reference(gold, name):
    m = meta_of(gold, name)
    f = os.path.join(DATA, m["files"]["features"])
    tab = io.read_features_packed(f, os.path.join(DATA, m["files"]["feature_states"]))
    np.testing.assert_array_equal(tab.obs, gold[name + "_obs"])
    np.testing.assert_array_equal(tab.applicable, gold[name + "_applicable"])
    np.testing.assert_array_equal(tab.locations, gold[name + "_locations"])
    np.testing.assert_array_equal(tab.families.astype(int), gold[name + "_families"])
    assert tab.feature_names == m["feature_names"]
    assert tab.state_names == m["state_names"]
    assert tab.family_names == m["family_names"]
    assert [str(x) for x in tab.site_ids] == m["site_ids"]
    assert [str(x) for x in tab.site_names] == m["site_names"]
    assert tab.log.replace(f, "<FEATURES>") == m["log"]
    assert tab.na_number == int(np.count_nonzero(gold[name + "_obs"] < 0))


@pytest.mark.parametrize("name", DATASETS)
def test_read_features_from_csv_drop_in(gold, name):
    m = meta_of(gold, name)
    (sites, site_names, features, feature_names, state_names, applicable, families, family_names,
     log) = io.read_features_from_csv(os.path.join(DATA, m["files"]["features"]),
                                      os.path.join(DATA, m["files"]["feature_states"]))
    obs = gold[name + "_obs"]
    assert features.shape == obs.shape + (applicable.shape[1],) and features.dtype == bool
    np.testing.assert_array_equal(np.where(features.any(-1), features.argmax(-1), -1), obs)
    np.testing.assert_array_equal(families, gold[name + "_families"])
    assert list(feature_names["external"]) == m["feature_names"]
    assert [list(s) for s in state_names["internal"]] == [list(range(len(s))) for s in m["state_names"]]
    assert sites["id"] == list(range(obs.shape[0])) and sites["cz"] is None


@pytest.mark.parametrize("name", ["balkan", "south_america"])
def test_prior_counts_match_reference(gold, name):
    m = meta_of(gold, name)
    fs = os.path.join(DATA, m["files"]["feature_states"])
    tab = io.read_features_packed(os.path.join(DATA, m["files"]["features"]), fs)
    uni, _ = io.read_universal_counts(tab, os.path.join(DATA, m["files"]["universal"]), "counts_file", fs)
    np.testing.assert_array_equal(uni, gold[name + "_universal_counts"])
    files = {k: os.path.join(DATA, v) for k, v in m["files"]["inheritance"].items()}
    inh, log = io.read_inheritance_counts(tab, files, "counts_file", fs)
    np.testing.assert_array_equal(inh, gold[name + "_inheritance_counts"])
    missing = [f for f in tab.family_names if f not in files]
    assert all(f"No prior information for {f}" in log for f in missing)


@pytest.mark.parametrize("name", ["balkan", "south_america"])
def test_network_matches_reference(gold, name):
    indptr, indices, dist = io.compute_network(gold[name + "_locations"])
    np.testing.assert_array_equal(indptr, gold[name + "_adj_indptr"])
    np.testing.assert_array_equal(indices, gold[name + "_adj_indices"])
    np.testing.assert_array_equal(dist, gold[name + "_dist_mat"])


def test_extract_feature_states_reference_fixture(tmp_path):
    """The reference's own test (test/test_extract_feature_states.py) and its expected file."""
    out = tmp_path / "feature_states.csv"
    io.extract_feature_states([os.path.join(DATA, "test/test_files/features.csv")], out)
    with open(os.path.join(DATA, "test/test_files/feature_states_expected.csv")) as f:
        assert out.read_text() == f.read()


def test_reader_errors(tmp_path):
    f = tmp_path / "f.csv"
    s = tmp_path / "s.csv"
    s.write_text("F1\nA\nB\n")
    f.write_text("id,name,family,x,y,F1\nl1,a,,0,0,C\n")
    with pytest.raises(AssertionError):
        io.read_features_packed(f, s)
    f.write_text("id,name,x,y,F1\nl1,a,0,0,A\n")
    with pytest.raises(KeyError):
        io.read_features_packed(f, s)
    f.write_text("id,name,family,x,y,F1\nl1,a,,0,0, A \nl2,b,fam,1,1,\n")
    tab = io.read_features_packed(f, s)
    assert tab.obs.tolist() == [[0], [-1]] and tab.na_number == 1
    assert tab.fam_of_site.tolist() == [255, 0] and tab.family_names == ["fam"]


def test_results_files_match_reference(gold, tmp_path):
    """match_areas -> rank_areas -> samples2file (MCMC.save_samples) on the captured statistics:
    the stats and areas files equal the reference's byte for byte."""
    m = meta_of(gold, "balkan")
    with np.load(os.path.join(GOLD, "samples_in.npz")) as z:
        stats = {k: list(z[k]) for k in z.files}
    for k in ("sample_lh_single_zones", "sample_prior_single_zones", "sample_posterior_single_zones"):
        stats[k] = [list(v) for v in stats[k]]
    stats["sample_likelihood"] = [float(v) for v in stats["sample_likelihood"]]
    stats["sample_prior"] = [float(v) for v in stats["sample_prior"]]
    n, Z = len(stats["sample_zones"]), stats["sample_zones"][0].shape[0]
    stats = postprocessing.rank_areas(postprocessing.match_areas(stats))
    data = types.SimpleNamespace(feature_names=m["feature_names"], state_names=m["state_names"],
                                 family_names=m["family_names"], is_simulated=False)
    config = {"model": {"INHERITANCE": True, "N_AREAS": Z}, "mcmc": {"N_STEPS": 1200, "N_SAMPLES": n}}
    paths = {"parameters": tmp_path / "stats.txt", "areas": tmp_path / "areas.txt"}
    io.samples2file(stats, data, config, paths)
    for mine, ref in (("stats.txt", "stats_expected.txt"), ("areas.txt", "areas_expected.txt")):
        with open(tmp_path / mine, "rb") as a, open(os.path.join(GOLD, ref), "rb") as b:
            assert a.read() == b.read(), mine


@pytest.mark.parametrize("case", ["sim1", "sim2"])
def test_simulated_results_files_match_reference(tmp_path, case):
    """samples2file on the reference's own simulations (sim_exp1: no inheritance, a 2-zone model
    against 1 true area; sim_exp2: simulated inheritance): the ground-truth stats and areas files
    (util.py:657-742) and the stats file with its recall / precision columns (:811-825, NaN
    precision for an empty sample) equal the reference's byte for byte."""
    with open(os.path.join(GOLD, f"samples_{case}_meta.json")) as f:
        m = json.load(f)
    with np.load(os.path.join(GOLD, f"samples_{case}_in.npz")) as z:
        d = {k: z[k] for k in z.files}
    stats = {k: list(d[k]) for k in d if k.startswith("sample_")}
    stats["sample_likelihood"] = [float(v) for v in stats["sample_likelihood"]]
    stats["sample_prior"] = [float(v) for v in stats["sample_prior"]]
    for k in ("true_zones", "true_weights", "true_p_global", "true_p_zones", "true_p_families"):
        if k in d:
            stats[k] = d[k]
    stats["true_ll"], stats["true_prior"] = float(d["true_ll"]), float(d["true_prior"])
    for k in ("true_lh_single_zones", "true_prior_single_zones", "true_posterior_single_zones"):
        stats[k] = [float(v) for v in d[k]]
    data = types.SimpleNamespace(feature_names=m["feature_names"], state_names=m["state_names"],
                                 family_names=m["family_names"], areas=d["true_zones"], is_simulated=True)
    paths = {"parameters": tmp_path / "stats.txt", "areas": tmp_path / "areas.txt",
             "gt": tmp_path / "gt_stats.txt", "gt_areas": tmp_path / "gt_areas.txt"}
    io.samples2file(stats, data, m["config"], paths)
    for mine, ref in (("stats.txt", f"stats_{case}_expected.txt"), ("areas.txt", f"areas_{case}_expected.txt"),
                      ("gt_stats.txt", f"gt_stats_{case}_expected.txt"),
                      ("gt_areas.txt", f"gt_areas_{case}_expected.txt")):
        with open(tmp_path / mine, "rb") as a, open(os.path.join(GOLD, ref), "rb") as b:
            assert a.read() == b.read(), mine


# ---- experiment setup (contact_zones_amd/experiment.py) vs the reference's Experiment/Data/MCMC ----
@pytest.mark.parametrize("name", ["balkan", "south_america"])
def test_experiment_setup_matches_reference(gold, name):
    from contact_zones_amd import experiment
    cfg_path = os.path.join(DATA, "experiments", name, "config.json")
    cfg, _ = experiment.load_config(cfg_path, {"model": {"N_AREAS": 3}})
    p = "setup_" + name + "_"
    assert cfg["mcmc"]["STEPS"] == json.loads(str(gold[p + "steps"]))
    assert experiment.operators(cfg) == json.loads(str(gold[p + "ops"]))
    data = experiment.ExperimentData(cfg)
    spec, (cg, cf) = experiment.build_priors(cfg, data)
    np.testing.assert_array_equal(spec.alpha_global, gold[p + "alpha_global"])
    np.testing.assert_array_equal(spec.alpha_fam, gold[p + "alpha_fam"])
    np.testing.assert_array_equal(cg, gold[p + "counts_global"])
    np.testing.assert_array_equal(cf, gold[p + "counts_fam"])
    np.testing.assert_array_equal(data.network["adj_mat"].indices, gold[name + "_adj_indices"])


def test_experiment_config_errors(tmp_path):
    from contact_zones_amd import experiment
    c = tmp_path / "c.json"
    c.write_text(json.dumps({"model": {"N_AREAS": 2}, "data": {"FEATURES": "f.csv", "FEATURE_STATES": "s.csv"}}))
    with pytest.raises(NameError):  # INHERITANCE is required
        experiment.load_config(c)
    c.write_text(json.dumps({"model": {"N_AREAS": 2, "INHERITANCE": False},
                             "mcmc": {"N_STEPS": 10, "N_SAMPLES": 3},
                             "data": {"FEATURES": "f.csv", "FEATURE_STATES": "s.csv"}}))
    with pytest.raises(ValueError):  # uneven sample spacing
        experiment.load_config(c)
    c.write_text(json.dumps({"simulation": {}, "model": {}}))
    with pytest.raises(NotImplementedError):
        experiment.load_config(c)


def test_geo_cost_matrix_reader(tmp_path):
    """read_geo_cost_matrix (preprocessing.py:677-700): rows / columns ordered by the features
    file's site ids, symmetrised by averaging when the file is not symmetric."""
    import pandas as pd
    ids = ["b", "a", "c"]
    raw = pd.DataFrame([[0, 1, 4], [3, 0, 2], [4, 2, 0]], index=["a", "b", "c"], columns=["a", "b", "c"])
    raw.to_csv(tmp_path / "cost.csv")
    cost, log = io.read_geo_cost_matrix(ids, tmp_path / "cost.csv")
    sym = (raw.values + raw.values.T) / 2
    order = [1, 0, 2]
    np.testing.assert_array_equal(cost, sym[np.ix_(order, order)])
    assert "made symmetric" in log
