"""The CPU MH restatement (oracle/mh_numpy.py) replays the reference's captured trajectories
bit for bit (tests/golden/make_golden_mh.py: seeded ZoneMCMC / ZoneMCMCWarmup runs)."""
import numpy as np
import pytest

from conftest import golden_cases, load_golden

MH_CASES = golden_cases(prefix="mh_", exclude=())


@pytest.mark.parametrize("case", MH_CASES)
def test_oracle_replays_reference_trajectory(case):
    from oracle import mh_numpy
    fx = load_golden(case)
    lls = []
    for c in range(fx["tape"].shape[0]):
        r = mh_numpy.replay(fx, c)
        np.testing.assert_array_equal(r["op"], fx["step_op"][c])
        np.testing.assert_array_equal(r["accept"], fx["step_accept"][c])
        np.testing.assert_array_equal(r["zos"], fx["step_zone_of_site"][c])
        np.testing.assert_array_equal(r["ll"], fx["step_ll"][c])
        # log prior (Prior.__call__): bit-exact at the start and after every step
        assert r["init_prior"] == fx["init_prior"][c]
        np.testing.assert_array_equal(r["prior"], fx["step_prior"][c])
        assert r["tape_used"] == int(fx["tape_len"][c])
        if bool(fx["sample_source"]):  # source assignments after every step
            np.testing.assert_array_equal(r["src"], fx["step_source"][c])
        # final parameters
        np.testing.assert_array_equal(r["state"]["w"], fx["final_w"][c])
        np.testing.assert_array_equal(r["state"]["pg"], fx["final_p_global"][c])
        np.testing.assert_array_equal(r["state"]["pz"], fx["final_p_zones"][c])
        if bool(fx["inheritance"]):
            np.testing.assert_array_equal(r["state"]["pf"], fx["final_p_fam"][c])
        lls.append(r["ll"][-1] + r["prior"][-1])
    if bool(fx["warmup"]):
        # best chain = argmax(ll + prior) after the warm-up (mcmc_generative.py:195-200)
        best = int(np.argmax(lls))
        np.testing.assert_array_equal(fx["step_zone_of_site"][best, -1], fx["best_zone_of_site"])


def test_fixtures_cover_every_operator_and_rejection_kind():
    ops = np.zeros(13, int)
    rejected_zone_moves = 0
    for case in MH_CASES:
        fx = load_golden(case)
        ops += np.bincount(fx["step_op"].ravel(), minlength=13)[:13]
        zone = fx["step_op"] <= 2
        rejected_zone_moves += int(np.sum(zone & ~fx["step_accept"]))
    assert np.all(ops[:7] > 50), ops
    assert rejected_zone_moves > 50


def test_fixtures_cover_the_source_mode_operators():
    """SAMPLE_SOURCE = true: every Gibbs operator and source-resampling zone moves."""
    ops = np.zeros(13, int)
    for case in MH_CASES:
        fx = load_golden(case)
        if bool(fx["sample_source"]):
            ops += np.bincount(fx["step_op"].ravel(), minlength=13)
    assert np.all(ops[[0, 1, 2, 8, 9, 10, 11, 12]] > 20), ops


def test_fixtures_cover_the_prior_types():
    """'counts' priors on p_global / p_families, and both non-trivial zone-size priors."""
    sizes, counts_g, counts_f = set(), 0, 0
    for case in MH_CASES:
        fx = load_golden(case)
        sizes.add(int(fx["prior_size"]))
        counts_g += "prior_alpha_global" in fx
        counts_f += "prior_alpha_fam" in fx
    assert sizes == {0, 1, 2} and counts_g >= 2 and counts_f >= 2


def test_fixtures_cover_gibbsish_sample_zones():
    """gibbsish_sample_zones (zone_sampling.py:619-702; weight 0 in the reference's own operator
    table, so captured with a non-zero weight): accepted and rejected moves in mixture and source
    mode, ZoneMCMC and ZoneMCMCWarmup, and networks with more than 100 available sites."""
    kinds = {}
    for case in MH_CASES:
        fx = load_golden(case)
        g = fx["step_op"] == 7
        if not g.any():
            continue
        key = (bool(fx["sample_source"]), bool(fx["warmup"]), fx["obs"].shape[0] > 100)
        acc, n = kinds.get(key, (0, 0))
        kinds[key] = (acc + int(np.sum(g & fx["step_accept"])), n + int(np.sum(g)))
    for key in [(False, False, False), (False, True, False), (False, False, True),
                (True, False, False), (True, True, False), (True, False, True)]:
        assert key in kinds and kinds[key][0] > 5, (key, kinds)
    assert any(acc < n for acc, n in kinds.values())
