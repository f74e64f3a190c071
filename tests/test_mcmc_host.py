"""Host side of the batched sampler drop-in (CPU): initial samples, warm-up chain lists and the
model checks, pinned to the reference's own values captured in tests/golden/mh_*.npz."""
import random
import types

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import prior_spec, golden_cases, load_golden, mh_cases
from contact_zones_amd import packing
from contact_zones_amd.mcmc import (BatchedZoneMCMC, BatchedZoneMCMCWarmup, InitialSamples,
                                    check_model, get_max_size_list)
from contact_zones_amd.priors import PriorSpec
from contact_zones_amd.sampler import OPS

MH_CASES = mh_cases(source=False)
SRC_CASES = mh_cases(source=True)


def objects_from_fixture(fx):
    """Reference-shaped (model, data, kwargs) for a captured case."""
    N = fx["obs"].shape[0]
    S = fx["states"].shape[1]
    inh = bool(fx["inheritance"])
    n_fam = fx["init_p_fam"].shape[1] if inh else 0
    adj = sp.csr_matrix((np.ones(fx["adj_indices"].size), fx["adj_indices"], fx["adj_indptr"]),
                        shape=(N, N))
    data = types.SimpleNamespace(
        features=packing.obs_to_features(fx["obs"], S), states=fx["states"],
        network={"adj_mat": adj},
        families=packing.index_to_groups(fx["fam_of_site"], n_fam) if inh else None)
    model = types.SimpleNamespace(n_zones=int(fx["n_zones"]), min_size=int(fx["min_size"]),
                                  max_size=int(fx["max_m"]), inheritance=inh,
                                  sample_source=bool(fx.get("sample_source", False)))
    ops = {OPS[i]: float(p) for i, p in enumerate(fx["op_probs"]) if p > 0 or OPS[i] == "gibbsish_sample_zones"}
    prec = fx["precision"]
    var_proposal = {"weights": prec[0], "universal": prec[1], "contact": prec[2],
                    "inheritance": prec[3] if inh else None}
    kw = dict(model=model, data=data, operators=ops, n_chains=fx["init_w"].shape[0],
              var_proposal=var_proposal, p_grow_connected=float(fx["p_grow_base"]),
              initial_size=int(fx["initial_size"]),
              priors=prior_spec(fx))
    if bool(fx.get("sample_source", False)):
        kw["gibbs_counts"] = (fx["gibbs_counts_global"], fx.get("gibbs_counts_fam"))
    return kw


def make_sampler(fx, **extra):
    kw = objects_from_fixture(fx)
    cls = BatchedZoneMCMCWarmup if bool(fx["warmup"]) else BatchedZoneMCMC
    return cls(rng=random.Random(int(fx["seed"])), **kw, **extra)


@pytest.mark.parametrize("case", MH_CASES + SRC_CASES)
def test_initial_samples_match_reference(case):
    """generate_initial_sample for every chain, in the reference's draw order, from the same
    seeded python random source (and np.random for the initial sources): zones, weights, p_*
    and sources identical to the reference's."""
    fx = load_golden(case)
    smp = make_sampler(fx)
    N = fx["obs"].shape[0]
    np.random.seed(int(fx["seed"]))
    for c in range(fx["init_w"].shape[0]):
        s = smp.generate_initial_sample(c)
        if bool(fx.get("sample_source", False)):
            np.testing.assert_array_equal(packing.source_to_index(s.source), fx["init_source"][c])
        np.testing.assert_array_equal(packing.zones_to_zone_of_site(s.zones, N), fx["init_zone_of_site"][c])
        np.testing.assert_array_equal(s.weights, fx["init_w"][c])
        np.testing.assert_array_equal(s.p_global[0], fx["init_p_global"][c])
        np.testing.assert_array_equal(s.p_zones, fx["init_p_zones"][c])
        if bool(fx["inheritance"]):
            np.testing.assert_array_equal(s.p_families, fx["init_p_fam"][c])


@pytest.mark.parametrize("case", [c for c in MH_CASES if "warmup" in c])
def test_warmup_chain_lists_match_reference(case):
    """ZoneMCMCWarmup: max_size list (util.get_max_size_list) and p_grow_connected choices."""
    fx = load_golden(case)
    smp = make_sampler(fx)
    np.testing.assert_array_equal(np.asarray(smp.max_size), fx["max_size"])
    np.testing.assert_array_equal(np.asarray(smp.p_grow_connected), fx["p_grow_connected"])


def test_max_size_list():
    assert get_max_size_list(2.25, 6, 3, 4) == [2, 3, 4]
    assert get_max_size_list(13.75, 50, 15, 4) == [13] * 4 + [22] * 4 + [31] * 4 + [40] * 3


def test_initial_sample_reuses_previous_sample():
    """initial_sample (the warm-up winner) is taken as is; missing zones are grown."""
    fx = load_golden("mh_small_bounds")
    kw = objects_from_fixture(fx)
    s0 = make_sampler(fx).generate_initial_sample(0)
    init = InitialSamples(kw["data"].features.astype(bool), fx["states"], fx["adj_indptr"],
                          fx["adj_indices"], kw["data"].families, 3, 4, True,
                          s0, random.Random(1))
    s = init(0)
    np.testing.assert_array_equal(s.zones, s0.zones)
    np.testing.assert_array_equal(s.p_zones, s0.p_zones)
    np.testing.assert_array_equal(s.p_families, s0.p_families)
    assert s.p_global is s0.p_global  # the reference does not copy it (zone_sampling.py:1068)


def test_model_checks():
    check_model(types.SimpleNamespace(sample_source=False, inheritance=True), {"grow_zone": 1.0})
    check_model(types.SimpleNamespace(sample_source=True, inheritance=False),
                {"grow_zone": 0.5, "gibbs_sample_sources": 0.5})
    with pytest.raises(ValueError):
        check_model(types.SimpleNamespace(sample_source=False), {"gibbs_sample_weights": 1.0})
    with pytest.raises(ValueError):
        check_model(types.SimpleNamespace(sample_source=True), {"alter_weights": 1.0})


def test_unsupported_options_raise():
    fx = load_golden("mh_cfg1_sim")
    kw = objects_from_fixture(fx)
    with pytest.raises(NotImplementedError):
        BatchedZoneMCMC(mc3=True, **kw)
    with pytest.raises(NotImplementedError):
        BatchedZoneMCMC(sample_from_prior=True, **kw)
    kw2 = dict(kw, operators={"grow_zone": 1.0, "gibbs_sample_sources": 0.5})
    with pytest.raises(ValueError):
        BatchedZoneMCMC(**kw2)


@pytest.mark.parametrize("case", ["lik_cfg3_balkan", "lik_cfg4_sa_z6", "lik_cfg2", "lik_edge_na"])
def test_gpu_likelihood_host_component_arrays(case):
    """GpuLikelihood's update_component_likelihoods / update_weights (the arrays the reference's
    own CPU operators read, model.py:230-294) reproduce the reference's likelihood:
    sum log sum_c lh * w equals the captured Likelihood(..., caching=False) value, and the source
    branch with the captured sources too (host only, no GPU)."""
    from contact_zones_amd.likelihood import GpuLikelihood
    fx = load_golden(case)
    inh = bool(fx["inheritance"])
    S = fx["p_global"].shape[-1]
    obs, fam = fx["obs"], fx["fam_of_site"]
    n_fam = fx["p_fam"].shape[1] if inh else 0
    data = types.SimpleNamespace(features=packing.obs_to_features(obs, S),
                                 families=packing.index_to_groups(fam, n_fam) if inh else np.zeros((0, obs.shape[0]), bool))
    lik = GpuLikelihood(data, inh)
    for b in range(fx["w"].shape[0]):
        Z = fx["p_zones"].shape[1]
        zones = packing.index_to_groups(fx["zone_of_site"][b], Z)
        sample = types.SimpleNamespace(
            zones=zones, weights=fx["w"][b], p_global=fx["p_global"][b][None], p_zones=fx["p_zones"][b],
            p_families=fx["p_fam"][b] if inh else None, source=None)
        lh = lik.update_component_likelihoods(sample, caching=False)
        w = lik.update_weights(sample)
        ll = np.sum(np.log(np.sum(lh * w, axis=-1)))
        assert ll == pytest.approx(float(fx["ll_mixture"][b]), rel=1e-12)
        src = fx["source"][b]
        sel = np.take_along_axis(lh * w, src[..., None].astype(np.intp), axis=-1)[..., 0]
        with np.errstate(divide="ignore"):
            lls = np.sum(np.log(sel))
        ref = float(fx["ll_source"][b])
        assert (lls == ref) if np.isinf(ref) else lls == pytest.approx(ref, rel=1e-12)
        np.testing.assert_array_equal(lik.get_zone_assignment(sample), fx["zone_of_site"][b] != 255)
