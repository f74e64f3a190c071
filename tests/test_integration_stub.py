"""The reference-side ctypes stub of INTEGRATION.md §2, run verbatim.

The stub is what a maintainer pastes into the reference (`sbayes/gpu.py`): plain ctypes on
libsbz.so, no import of this repository's package.  These tests take the code block out of
INTEGRATION.md as it stands, point its library path at the in-tree build and exec it, so the
document cannot drift from the ABI.  The GPU test feeds it reference-form objects (one-hot
features, (Z, N) zone masks, (N, F, C) one-hot sources; util.py:289-336, model.py:145-171) built
from the golden `lik_cfg3_balkan` (Balkan data, captured from the reference's own
Likelihood.__call__) and checks the values the reference computed, in both branches."""
import os
import re
import types

import numpy as np
import pytest

from conftest import ROOT, load_golden
from contact_zones_amd import _lib

DOC = os.path.join(ROOT, "INTEGRATION.md")


def load_stub():
    text = open(DOC).read()
    sec = text[text.index("## 2. The ctypes stub"):]
    code = re.search(r"```python\n(.*?)```", sec, flags=re.S).group(1)
    assert '"/path/to/contact_zones_amd/libsbz.so"' in code
    code = code.replace('"/path/to/contact_zones_amd/libsbz.so"', repr(_lib.LIB_PATH))
    ns = {"__name__": "sbayes_gpu_stub"}
    exec(compile(code, "INTEGRATION.md#stub", "exec"), ns)
    return ns


def reference_objects(g, b, source):
    """Reference-form Data / Model / Sample of chain b of a likelihood golden."""
    obs, fam = g["obs"], g["fam_of_site"]
    N, F = obs.shape
    S = g["p_global"].shape[-1]
    feats = np.zeros((N, F, S), bool)
    n_i, f_i = np.nonzero(obs >= 0)
    feats[n_i, f_i, obs[n_i, f_i]] = True
    Fam = g["p_fam"].shape[1]
    families = np.stack([fam == i for i in range(Fam)])
    Z = g["p_zones"].shape[1]
    zones = np.stack([g["zone_of_site"][b] == z for z in range(Z)])
    src = None
    if source:
        src = np.zeros((N, F, 3), bool)
        n_i, f_i = np.indices((N, F))
        src[n_i, f_i, g["source"][b]] = True
    data = types.SimpleNamespace(features=feats, families=families)
    model = types.SimpleNamespace(inheritance=True, n_zones=Z)
    sample = types.SimpleNamespace(zones=zones, weights=g["w"][b], p_global=g["p_global"][b][None],
                                   p_zones=g["p_zones"][b], p_families=g["p_fam"][b], source=src)
    return data, model, sample


def test_stub_binds_every_entry_it_uses():
    ns = load_stub()
    lib = ns["_lib"]
    for name in ("sbz_open", "sbz_loglik_batch", "sbz_last_error", "sbz_close"):
        assert getattr(lib, name).argtypes is not None or name == "sbz_close"
    assert ns["SBZ_INHERITANCE"] == _lib.SBZ_INHERITANCE
    assert [f[0] for f in ns["sbz_dims"]._fields_] == [f[0] for f in _lib.sbz_dims._fields_]


def test_stub_reports_a_failed_open_without_gpu():
    ns = load_stub()
    if ns["_lib"].sbz_device_count() > 0:
        pytest.skip("a HIP device is visible: the GPU test covers the stub")
    g = load_golden("lik_cfg3_balkan")
    data, model, _ = reference_objects(g, 0, False)
    with pytest.raises(RuntimeError, match="sbz_open failed"):
        ns["GpuLikelihoodStub"](data, model)


@pytest.mark.gpu
@pytest.mark.parametrize("source", [False, True])
def test_stub_matches_reference_on_balkan(gpu_available, source):
    ns = load_stub()
    g = load_golden("lik_cfg3_balkan")
    want = g["ll_source" if source else "ll_mixture"]
    for b in range(len(want)):
        data, model, sample = reference_objects(g, b, source)
        lik = ns["GpuLikelihoodStub"](data, model)
        try:
            got = lik(sample, caching=False)
        finally:
            ns["_lib"].sbz_close(lik.ctx)
        assert got == pytest.approx(want[b], rel=1e-9), (b, got, want[b])
