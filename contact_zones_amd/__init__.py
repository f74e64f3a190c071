"""contact_zones_amd — MI355X-native sBayes likelihood + sampler core.

The hot path of sBayes (derpetermann/contact_zones) — the per-step mixture
likelihood (sbayes/model.py:69-452) and the zone-proposal accept/reject loop
(sbayes/sampling/zone_sampling.py, mcmc_generative.py:282-351) — as hand-written
HIP kernels for gfx950 behind a C-ABI (include/sbz.h, libsbz.so), with a thin
Python host that keeps the reference's operator surface.
"""
from . import packing  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # Lazy: importing the package must not require the GPU library (CPU tests, packing).
    if name in ("LikelihoodEngine", "GpuLikelihood", "pack_sample"):
        from . import likelihood
        return getattr(likelihood, name)
    raise AttributeError(name)
