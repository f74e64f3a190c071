"""The batched drop-in end to end on the GPU: generate_samples / statistics / warm-up best chain
against the reference's own outputs (tests/golden/mh_*.npz, make_golden_mh.py)."""
import numpy as np
import pytest

from conftest import golden_cases, load_golden, mh_cases
from test_mcmc_host import make_sampler

from contact_zones_amd import packing
from contact_zones_amd.sampler import OPS

pytestmark = pytest.mark.gpu

MH_CASES = mh_cases(source=False)
SRC_CASES = mh_cases(source=True)  # SAMPLE_SOURCE = true (sbz_mh_src.hip)
MAIN = [c for c in MH_CASES + SRC_CASES if "warmup" not in c]
WARM = [c for c in MH_CASES + SRC_CASES if "warmup" in c]
RTOL = 1e-9  # log-likelihood tolerance (north_star: 1e-9 relative)


@pytest.mark.parametrize("case", MAIN)
def test_generate_samples_statistics_match_reference(case, gpu_available):
    """ZoneMCMC.generate_samples replayed on the GPU (decision tape): the statistics dict equals
    the reference's — sample ids, zones and parameters of chain 0 bit-exact, log-likelihoods
    within 1e-9, per-operator accept / reject counts summed over chains, last sample."""
    fx = load_golden(case)
    smp = make_sampler(fx)
    smp._tape = (fx["tape"], fx["tape_len"])
    n_steps = fx["step_op"].shape[1]
    np.random.seed(int(fx["seed"]))  # the initial sources' draws (np.random, as the reference)
    smp.generate_samples(n_steps, int(fx["stat_n_samples"]))
    st = smp.statistics
    assert st["sample_id"] == fx["stat_sample_id"].tolist()
    np.testing.assert_allclose(st["sample_likelihood"], fx["stat_sample_likelihood"], rtol=RTOL)
    assert st["sample_prior"] == fx["stat_sample_prior"].tolist()  # bit-exact (host Prior)
    np.testing.assert_array_equal(np.array(st["sample_zones"]), fx["stat_sample_zones"])
    np.testing.assert_array_equal(np.array(st["sample_weights"]), fx["stat_sample_weights"])
    np.testing.assert_array_equal(np.array(st["sample_p_global"]), fx["stat_sample_p_global"])
    np.testing.assert_array_equal(np.array(st["sample_p_zones"]), fx["stat_sample_p_zones"])
    if "stat_sample_p_families" in fx:
        np.testing.assert_array_equal(np.array(st["sample_p_families"]), fx["stat_sample_p_families"])
    assert st["accepted_steps"] == int(fx["stat_accepted_steps"])
    assert st["acceptance_ratio"] == float(fx["stat_acceptance_ratio"])
    for i, name in enumerate(OPS):
        assert st["accept_operator"].get(name, 0) == fx["stat_accept_operator"][i], name
        assert st["reject_operator"].get(name, 0) == fx["stat_reject_operator"][i], name
    np.testing.assert_array_equal(st["last_sample"].zones, fx["stat_last_zones"])
    np.testing.assert_array_equal(st["last_sample"].weights, fx["stat_last_weights"])
    assert st["sampling_time"] > 0 and st["swap_ratio"] == 0


@pytest.mark.parametrize("case", WARM)
def test_warmup_best_sample_matches_reference(case, gpu_available):
    """ZoneMCMCWarmup.generate_samples(warm_up=True): the best chain's final Sample."""
    fx = load_golden(case)
    smp = make_sampler(fx)
    smp._tape = (fx["tape"], fx["tape_len"])
    np.random.seed(int(fx["seed"]))
    best = smp.generate_samples(0, 0, warm_up=True, warm_up_steps=fx["step_op"].shape[1])
    N = fx["obs"].shape[0]
    np.testing.assert_array_equal(packing.zones_to_zone_of_site(best.zones, N), fx["best_zone_of_site"])
    np.testing.assert_array_equal(best.weights, fx["best_w"])
    np.testing.assert_array_equal(best.p_global[0], fx["best_p_global"])
    np.testing.assert_array_equal(best.p_zones, fx["best_p_zones"])
    if "best_p_fam" in fx:
        np.testing.assert_array_equal(best.p_families, fx["best_p_fam"])


def test_philox_run_is_self_consistent(gpu_available):
    """Production mode (Philox draws): logged log-likelihoods are full evaluations of the logged
    samples, the statistics have the reference's shape, the run is reproducible from its seed,
    and a warm-up winner can seed the main run (the MCMC.warm_up -> MCMC.sample hand-off)."""
    fx = load_golden("mh_cfg1_sim_inh_z2")

    def run(seed):
        smp = make_sampler(fx, seed=seed)
        smp.generate_samples(500, 50)
        return smp

    a, b = run(11), run(11)
    st = a.statistics
    assert len(st["sample_id"]) == 50 and st["sample_id"] == list(range(50))
    assert np.isfinite(st["sample_likelihood"]).all()
    assert st["sample_likelihood"] == b.statistics["sample_likelihood"]
    for i in (0, 17, 49):
        sample = type(st["last_sample"])(st["sample_zones"][i], st["sample_weights"][i],
                                         st["sample_p_global"][i], st["sample_p_zones"][i],
                                         st["sample_p_families"][i])
        np.testing.assert_allclose(a.likelihood(sample, 0), st["sample_likelihood"][i], rtol=1e-12)
    tot = sum(st["accept_operator"].values()) + sum(st["reject_operator"].values())
    assert tot == 500 * a.n_chains
    assert 0 < st["acceptance_ratio"] <= a.n_chains
    # warm-up -> main run hand-off
    from contact_zones_amd.mcmc import BatchedZoneMCMC, BatchedZoneMCMCWarmup
    from test_mcmc_host import objects_from_fixture
    import random
    kw = objects_from_fixture(fx)
    kw["n_chains"] = 8
    w = BatchedZoneMCMCWarmup(rng=random.Random(3), seed=5, **kw)
    best = w.generate_samples(0, 0, warm_up=True, warm_up_steps=300)
    assert best.zones.shape == (int(fx["n_zones"]), fx["obs"].shape[0])
    m = BatchedZoneMCMC(rng=random.Random(4), seed=6, initial_sample=best, **dict(kw, n_chains=2))
    s0 = m.generate_initial_sample(0)
    np.testing.assert_array_equal(s0.zones, best.zones)
    m.generate_samples(100, 10)
    assert len(m.statistics["sample_id"]) == 10


@pytest.mark.parametrize("case", [c for c in MAIN if c in MH_CASES])
def test_contribution_per_area_matches_reference(case, gpu_available):
    """postprocessing.contribution_per_area on the reference's logged samples: per-zone
    log-likelihoods within 1e-9, priors bit-exact (one batched likelihood launch)."""
    from contact_zones_amd.postprocessing import contribution_per_area
    fx = load_golden(case)
    smp = make_sampler(fx)
    st = smp.statistics
    st["sample_zones"] = list(fx["stat_sample_zones"])
    st["sample_weights"] = list(fx["stat_sample_weights"])
    st["sample_p_global"] = list(fx["stat_sample_p_global"])
    st["sample_p_zones"] = list(fx["stat_sample_p_zones"])
    st["sample_p_families"] = (list(fx["stat_sample_p_families"]) if "stat_sample_p_families" in fx
                               else [None] * len(st["sample_zones"]))
    contribution_per_area(smp, batch=16)  # several chunks
    np.testing.assert_allclose(np.array(st["sample_lh_single_zones"]), fx["stat_lh_single_zones"],
                               rtol=RTOL)
    np.testing.assert_array_equal(np.array(st["sample_prior_single_zones"]), fx["stat_prior_single_zones"])
    np.testing.assert_allclose(np.array(st["sample_posterior_single_zones"]),
                               fx["stat_lh_single_zones"] + fx["stat_prior_single_zones"], rtol=RTOL)
