"""Pin the oracle (CPU restatements) to golden vectors captured from the reference.

The expected values were produced by sbayes.model.Likelihood(..., caching=False)
itself (tests/golden/make_golden_lik.py).  The numpy restatement must be
bit-identical; the C restatement follows numpy's pairwise summation and differs
only through libm's log vs numpy's SIMD log (<= a few 1e-16 relative).
"""
import numpy as np
import pytest

from conftest import golden_cases, load_golden
from oracle import lik_numpy, oracle_c

CASES = golden_cases()


def _args(d):
    return (d["obs"], d["fam_of_site"], d["zone_of_site"], d["w"], d["p_global"], d["p_zones"],
            d.get("p_fam"))


def _rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    same_inf = (a == b) | (np.isnan(a) & np.isnan(b))
    with np.errstate(invalid="ignore", divide="ignore"):
        r = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
    return float(np.max(np.where(same_inf, 0.0, r)))


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("mode", ["mixture", "source"])
def test_numpy_oracle_bit_exact(case, mode):
    d = load_golden(case)
    src = d["source"] if mode == "source" else None
    got = lik_numpy.loglik_batch(*_args(d), source=src, inheritance=bool(d["inheritance"]))
    np.testing.assert_array_equal(got, d["ll_" + mode])


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("mode", ["mixture", "source"])
def test_c_oracle_matches_reference(case, mode):
    d = load_golden(case)
    src = d["source"] if mode == "source" else None
    got = oracle_c.loglik_batch(*_args(d), source=src, inheritance=bool(d["inheritance"]))
    assert _rel(got, d["ll_" + mode]) <= 1e-15


def test_known_answer_test_model():
    """test/test_model.py:52-92: inheritance with [.4,.3,.3] == no inheritance [.4,.6] == direct."""
    d = load_golden("lik_kat")
    args = (d["obs"], d["fam_of_site"], d["zone_of_site"][0])
    lf = lik_numpy.loglik(*args, d["w3"][0], d["p_global"][0], d["p_zones"][0], d["p_fam"][0],
                          inheritance=True)
    ln = lik_numpy.loglik(*args, d["w2"][0], d["p_global"][0], d["p_zones"][0], None,
                          inheritance=False)
    assert lf == d["lh_with_family"]
    assert ln == d["lh_without_family"]
    assert lf == pytest.approx(float(d["lh_direct"]), rel=1e-12)
    assert ln == pytest.approx(lf, rel=1e-12)


def test_source_minus_inf_on_zero_weight():
    d = load_golden("lik_edge_zero")
    assert d["ll_source"][0] == -np.inf
    got = oracle_c.loglik_batch(*_args(d), source=d["source"], inheritance=True)
    assert got[0] == -np.inf
