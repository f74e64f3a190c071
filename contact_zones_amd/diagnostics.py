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


def ess(x, max_lag=2000, return_capped=False):
    """ESS of each trace in x (shape [..., n]); 0 for a constant trace.  max_lag=None: no cap
    beyond the trace length.  return_capped: also a bool array, True where the pair sum was still
    positive at the cap (the ESS is then an upper bound, not a mixing measurement)."""
    x = np.asarray(x, np.float64)
    flat = x.reshape(-1, x.shape[-1])
    n = flat.shape[1]
    out = np.zeros(flat.shape[0])
    capped = np.zeros(flat.shape[0], bool)
    if n < 2:
        return (out.reshape(x.shape[:-1]), capped.reshape(x.shape[:-1])) if return_capped \
            else out.reshape(x.shape[:-1])
    g = autocovariance(flat)
    lag_cap = n - 1 if max_lag is None else min(n - 1, max_lag)
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
        # the pair sums stayed positive up to the cap, whether the cap was max_lag or the trace
        # length: the estimate is then limited by the window, an upper bound on the ESS
        capped[i] = lag >= lag_cap
        out[i] = n * gi[0] / var
    if return_capped:
        return out.reshape(x.shape[:-1]), capped.reshape(x.shape[:-1])
    return out.reshape(x.shape[:-1])


def logged_trace(trace, n_samples=1000):
    """The samples the reference logs from a per-step trace [..., n_steps]: after every step i
    with i % ceil(n_steps / n_samples) == 0 (MCMCGenerative.generate_samples,
    sbayes/sampling/mcmc_generative.py:205-218; N_SAMPLES 1000 in config/default_config.json)."""
    trace = np.asarray(trace)
    sps = int(np.ceil(trace.shape[-1] / n_samples))
    return trace[..., ::sps], sps


def logged_ess(trace, n_samples=1000, max_lag=2000):
    """Tracer's ESS (its lag cap, 2000 samples) of the log-likelihood samples the reference would
    log from this per-step trace, in units of logged samples, plus the thinning step and the
    chains whose estimate hit the cap."""
    logged, sps = logged_trace(trace, n_samples)
    e, capped = ess(logged, max_lag, return_capped=True)
    return e, sps, capped
