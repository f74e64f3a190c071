"""Host prior terms (contact_zones_amd/priors.py): the full log prior equals the reference's
Prior.__call__ values captured in tests/golden/mh_*.npz, and reference Prior objects map to the
kernel's parameters (or are rejected when unsupported)."""
import types
from enum import Enum

import numpy as np
import pytest

from conftest import prior_spec, golden_cases, load_golden
from contact_zones_amd.priors import PriorSpec

MH_CASES = golden_cases("mh_", exclude=())


def spec_from_fixture(fx):
    return prior_spec(fx)


@pytest.mark.parametrize("case", MH_CASES)
def test_log_prior_matches_reference(case):
    fx = load_golden(case)
    inh = bool(fx["inheritance"])
    lp = spec_from_fixture(fx).log_prior(fx["init_zone_of_site"], fx["init_p_global"],
                                         fx["init_p_fam"] if inh else None, fx["states"],
                                         int(fx["n_zones"]), inh)
    np.testing.assert_array_equal(lp, fx["init_prior"])  # bit-exact


class T(Enum):
    UNIFORM = "uniform"
    COUNTS = "counts"
    UNIVERSAL = "universal"
    NONE = "none"
    QUADRATIC = "quadratic"
    COST = "cost_based"
    GAUSS = "gaussian"


def fake_prior(pg="uniform", pf="uniform", size="none", geo="uniform", F=3, S=4, n_fam=2):
    rng = np.random.default_rng(0)
    states = np.ones((F, S), bool)
    states[1, 3] = False
    ns = lambda t, **kw: types.SimpleNamespace(prior_type=T(t), **kw)  # noqa: E731
    dg = [rng.random(states[f].sum()) + 1 for f in range(F)]
    df = [[rng.random(states[f].sum()) + 1 for f in range(F)] for _ in range(n_fam)]
    prior = types.SimpleNamespace(size_prior=ns(size), geo_prior=ns(geo), prior_weights=ns("uniform"),
                                  prior_p_global=ns(pg, dirichlet=dg), prior_p_zones=ns("uniform"),
                                  prior_p_families=ns(pf, dirichlet=df))
    return types.SimpleNamespace(prior=prior, inheritance=True), states, dg, df


def test_spec_from_reference_prior_objects():
    model, states, dg, df = fake_prior(pg="counts", pf="counts", size="quadratic")
    s = PriorSpec.from_model(model, states)
    assert s.size_prior == 2 and not s.is_zero
    np.testing.assert_array_equal(s.alpha_global[1, states[1]], dg[1])
    assert s.alpha_global[1, 3] == 0.0
    np.testing.assert_array_equal(s.alpha_fam[1, 2, states[2]], df[1][2])
    assert PriorSpec.from_model(fake_prior()[0], states).is_zero
    assert PriorSpec.from_model(types.SimpleNamespace(inheritance=False), states).is_zero


@pytest.mark.parametrize("kw", [dict(pg="universal"), dict(pf="universal"), dict(geo="gaussian")])
def test_unsupported_prior_types_raise(kw):
    model, states, _, _ = fake_prior(**kw)
    with pytest.raises(NotImplementedError):
        PriorSpec.from_model(model, states)


def test_size_prior_values():
    """-sum log C(N, size) and -sum log size^2 on a hand-checked case."""
    from math import comb, log
    zos = np.array([[0, 0, 1, 255, 1, 1]], np.uint8)
    st = np.ones((1, 2), bool)
    pg = np.full((1, 1, 2), 0.5)
    u = PriorSpec(size_prior="uniform").log_prior(zos, pg, None, st, 2, False)[0]
    q = PriorSpec(size_prior="quadratic").log_prior(zos, pg, None, st, 2, False)[0]
    assert np.isclose(u, -(log(comb(6, 2)) + log(comb(6, 3))), rtol=1e-13)
    assert np.isclose(q, -(log(4) + log(9)), rtol=1e-13)
    with pytest.raises(NotImplementedError):
        PriorSpec(size_prior="exponential")


def test_geo_prior_from_reference_object():
    """'cost_based' geo priors carry the reference GeoPrior's cost matrix and scale."""
    model, states, _, _ = fake_prior(geo="cost_based")
    cost = np.arange(16.0).reshape(4, 4)
    model.prior.geo_prior.cost_matrix, model.prior.geo_prior.scale = cost, 7.0
    s = PriorSpec.from_model(model, states)
    assert s.geo_scale == 7.0 and not s.is_zero
    np.testing.assert_array_equal(s.geo_cost, cost)
