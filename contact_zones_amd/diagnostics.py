"""Effective sample size of MCMC traces (host-side, not on the hot path).

The reference delegates ESS to Tracer, so the estimator is ours.  It follows
the BEAST / Tracer autocorrelation method: autocovariances gamma[lag] (normalised by n - lag) are
summed in adjacent pairs until the first pair whose sum is not positive (Geyer's initial positive
sequence), capped at max_lag; ACT = (gamma[0] + 2 * sum of the accepted pairs) / gamma[0] and
ESS = n / ACT.
"""
import numpy as np


def autocovariance(x):
    """gamma[lag] = sum_j (x_j - m)(x_{j+lag} - m) / (n - lag) for every lag, via FFT."""
    x = np.asarray(x, np.float64)
    n = x.shape[-1]
    d = x - x.mean(axis=-1, keepdims=True)
    m = 1 << int(np.ceil(np.log2(max(2 * n - 1, 1))))
    f = np.fft.rfft(d, n=m, axis=-1)
    acov = np.fft.irfft(f * np.conj(f), n=m, axis=-1)[..., :n]
    return acov / (n - np.arange(n))


def ess(x, max_lag=2000):
    """ESS of each trace in x (shape [..., n]); 0 for a constant trace."""
    x = np.asarray(x, np.float64)
    flat = x.reshape(-1, x.shape[-1])
    n = flat.shape[1]
    out = np.zeros(flat.shape[0])
    if n < 2:
        return out.reshape(x.shape[:-1])
    g = autocovariance(flat)
    lag_cap = min(n - 1, max_lag)
    for i in range(flat.shape[0]):
        gi = g[i]
        if not gi[0] > 0:
            continue
        var = gi[0]
        lag = 2
        while lag < lag_cap:
            pair = gi[lag - 1] + gi[lag]
            if not pair > 0:
                break
            var += 2.0 * pair
            lag += 2
        out[i] = n * gi[0] / var
    return out.reshape(x.shape[:-1])
