import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def golden_cases(prefix="lik_", exclude=("lik_kat",)):
    names = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith(prefix) and f.endswith(".npz"))
    return [n for n in names if n not in exclude]


def mh_cases(source=None):
    """MH golden cases; source=False / True selects SAMPLE_SOURCE = false / true runs."""
    out = []
    for c in golden_cases("mh_", exclude=()):
        src = c.startswith("mh_src")
        if source is None or src == source:
            out.append(c)
    return out


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz")) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def gpu_available():
    from contact_zones_amd._lib import lib
    n = lib().sbz_device_count()
    if n < 1:
        pytest.fail("gpu test selected but no HIP device is visible")
    return n


def prior_spec(fx):
    """The PriorSpec of a captured MH case (tests/golden/make_golden_mh.py): 'counts'
    concentrations, zone-size prior and the 'cost_based' geo prior's cost matrix and scale."""
    from contact_zones_amd.priors import PriorSpec
    return PriorSpec(fx.get("prior_alpha_global"), fx.get("prior_alpha_fam"), int(fx["prior_size"]),
                     fx.get("prior_geo_cost"),
                     float(fx["prior_geo_scale"]) if "prior_geo_scale" in fx else None)
