"""ESS estimator (host side): known cases and agreement with a direct O(n * lag) restatement."""
import numpy as np

from contact_zones_amd.diagnostics import autocovariance, ess


def direct_ess(x, max_lag=2000):
    """The Tracer loop written out directly (BEAST TraceCorrelation, continuous traces)."""
    n = len(x)
    m = x.mean()
    lag_cap = min(n - 1, max_lag)
    g = np.zeros(lag_cap)
    var = 0.0
    for lag in range(lag_cap):
        g[lag] = np.dot(x[:n - lag] - m, x[lag:] - m) / (n - lag)
        if lag == 0:
            var = g[0]
        elif lag % 2 == 0:
            if g[lag - 1] + g[lag] > 0:
                var += 2.0 * (g[lag - 1] + g[lag])
            else:
                break
    return n * g[0] / var


def test_autocovariance_matches_direct():
    x = np.random.default_rng(0).normal(size=300)
    g = autocovariance(x)
    m = x.mean()
    for lag in (0, 1, 7, 299):
        assert np.isclose(g[lag], np.dot(x[:300 - lag] - m, x[lag:] - m) / (300 - lag))


def test_ess_iid_and_ar1():
    rng = np.random.default_rng(1)
    iid = rng.normal(size=20000)
    assert 0.8 * 20000 < ess(iid) < 1.25 * 20000
    phi = 0.9
    ar = np.zeros(20000)
    for t in range(1, 20000):
        ar[t] = phi * ar[t - 1] + rng.normal()
    expected = 20000 * (1 - phi) / (1 + phi)  # AR(1): ESS = n (1 - phi) / (1 + phi)
    assert 0.7 * expected < ess(ar) < 1.4 * expected
    for x in (iid[:500], ar[:3000]):
        assert np.isclose(ess(x), direct_ess(x), rtol=1e-9)


def test_ess_batched_and_degenerate():
    rng = np.random.default_rng(2)
    x = rng.normal(size=(3, 4, 100))
    e = ess(x)
    assert e.shape == (3, 4)
    assert np.isclose(e[1, 2], ess(x[1, 2]))
    assert ess(np.ones(50)) == 0.0
    assert ess(np.array([1.0])) == 0.0


def test_ess_capped_flag():
    """A trace whose pair sums stay positive up to the lag window is flagged (its ESS is then an
    upper bound), whether the window is max_lag or the trace length; a white-noise trace is not."""
    rng = np.random.default_rng(3)
    iid = rng.normal(size=400)
    walk = np.cumsum(rng.normal(size=400))  # unmixed: positive autocovariance over short lags
    e, capped = ess(np.stack([iid, walk]), max_lag=50, return_capped=True)
    assert capped.tolist() == [False, True]
    # window = the trace length: a short, strongly correlated trace reaches it
    _, capped = ess(np.array([0.0, 1.0, 2.0, 2.5, 2.0, 1.0]), max_lag=None, return_capped=True)
    assert not bool(capped)  # the mean-centred pair sums turn negative before the end
