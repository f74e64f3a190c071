"""eval_ground_truth (sbayes/mcmc_setup.py:122-172): the simulated ground truth and each of its
zones alone, against the reference's own values (tests/golden/truth_*.npz, captured by
tests/golden/make_golden_truth.py from the reference's MCMC.eval_ground_truth).

CPU: the oracle's likelihood and the host's prior on the fixture inputs pin the fixtures.
GPU: contact_zones_amd.postprocessing.eval_ground_truth through the C-ABI, within the north_star
tolerance (1e-9 relative) for likelihoods; priors are host arithmetic (1e-12).
"""
import random
import types

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import load_golden

CASES = ["truth_sim", "truth_synth"]
REL = 1e-9


def _truth(fx):
    inh = bool(fx["inheritance"])
    return types.SimpleNamespace(
        areas=fx["areas"], weights=fx["data_weights"], p_universal=fx["p_universal"],
        p_contact=fx["p_contact"], p_inheritance=fx["p_inheritance"] if inh else None,
        families=fx["families"] if inh else None)


def _prior_spec(fx):
    from contact_zones_amd.priors import PriorSpec
    return PriorSpec(size_prior=str(fx["size_prior"]))


@pytest.mark.parametrize("case", CASES)
def test_fixture_pinned_by_oracle(case):
    from oracle import lik_numpy
    from contact_zones_amd import packing
    fx = load_golden(case)
    inh = bool(fx["inheritance"])
    t = _truth(fx)
    N = fx["obs"].shape[0]
    w = fx["true_weights"]
    np.testing.assert_array_equal(
        w, fx["data_weights"] if inh else fx["data_weights"][:, :2] / fx["data_weights"][:, :2].sum(-1, keepdims=True))
    pf = t.p_inheritance if inh else None
    zos = packing.zones_to_zone_of_site(t.areas, N)
    ll = lik_numpy.loglik(fx["obs"], fx["fam_of_site"], zos, w, t.p_universal, t.p_contact, pf,
                          inheritance=inh)
    assert ll == pytest.approx(float(fx["true_ll"]), rel=REL)
    spec = _prior_spec(fx)
    pr = spec.log_prior(zos[None], t.p_universal[None], None if pf is None else pf[None],
                        fx["states"], t.areas.shape[0], inh)[0]
    assert pr == pytest.approx(float(fx["true_prior"]), rel=1e-12, abs=1e-12)
    for z in range(t.areas.shape[0]):
        zz = np.where(t.areas[z], 0, 255).astype(np.uint8)
        lz = lik_numpy.loglik(fx["obs"], fx["fam_of_site"], zz, w, t.p_universal, t.p_contact[z:z + 1], pf,
                              inheritance=inh)
        assert lz == pytest.approx(float(fx["true_lh_single_zones"][z]), rel=REL)
        pz = spec.log_prior(zz[None], t.p_universal[None], None if pf is None else pf[None],
                            fx["states"], 1, inh)[0]
        assert pz == pytest.approx(float(fx["true_prior_single_zones"][z]), rel=1e-12, abs=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("model_zones", ["truth", "other"])
def test_eval_ground_truth_gpu(case, model_zones, gpu_available):
    """The drop-in on the GPU: the sampler's model has the truth's number of zones (its own
    context) or another one (a context for the truth)."""
    from contact_zones_amd import packing
    from contact_zones_amd.mcmc import BatchedZoneMCMC
    from contact_zones_amd.postprocessing import eval_ground_truth
    fx = load_golden(case)
    inh = bool(fx["inheritance"])
    N, S = fx["obs"].shape[0], fx["states"].shape[1]
    Zt = fx["areas"].shape[0]
    adj = sp.csr_matrix((np.ones(fx["adj_indices"].size), fx["adj_indices"], fx["adj_indptr"]), shape=(N, N))
    data = types.SimpleNamespace(features=packing.obs_to_features(fx["obs"], S), states=fx["states"],
                                 network={"adj_mat": adj}, families=fx["families"] if inh else None)
    model = types.SimpleNamespace(n_zones=Zt if model_zones == "truth" else Zt + 1, min_size=3, max_size=50,
                                  inheritance=inh, sample_source=False)
    ops = {"shrink_zone": 0.4, "grow_zone": 0.4, "swap_zone": 0.2, "alter_weights": 0.0,
           "alter_p_global": 0.0, "alter_p_zones": 0.0}
    smp = BatchedZoneMCMC(model=model, data=data, operators=ops, n_chains=1,
                          var_proposal={"weights": 15, "universal": 40, "contact": 20,
                                        "inheritance": 20 if inh else None},
                          p_grow_connected=0.85, initial_size=5, priors=_prior_spec(fx), rng=random.Random(1))
    out = eval_ground_truth(smp, _truth(fx), inh, {})
    assert out["true_ll"] == pytest.approx(float(fx["true_ll"]), rel=REL)
    assert out["true_prior"] == pytest.approx(float(fx["true_prior"]), rel=1e-12, abs=1e-12)
    np.testing.assert_allclose(out["true_lh_single_zones"], fx["true_lh_single_zones"], rtol=REL)
    np.testing.assert_allclose(out["true_prior_single_zones"], fx["true_prior_single_zones"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(out["true_posterior_single_zones"], fx["true_posterior_single_zones"], rtol=REL)
    np.testing.assert_array_equal(out["true_weights"], fx["true_weights"])
