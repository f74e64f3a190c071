"""GPU parity: the HIP likelihood vs the reference's golden values and the oracle.

Tolerance (north_star): log-likelihoods within 1e-9 relative of the reference CPU
path.  Each table entry is computed in the reference's operation order with fused
multiply-adds (an entry within an ulp of the reference's cell), and the reduction differs
(product accumulation + one log per lane + fp64 tree sum); in practice the error is
~1e-15 relative.
"""
import numpy as np
import pytest

from conftest import golden_cases, load_golden

pytestmark = pytest.mark.gpu

REL_TOL = 1e-9
CASES = golden_cases()


def _engine(d, device=0, options=None):
    from contact_zones_amd.likelihood import LikelihoodEngine
    inh = bool(d["inheritance"])
    Fam = d["p_fam"].shape[1] if inh else 0
    return LikelihoodEngine(d["obs"], d["fam_of_site"], d["p_global"].shape[2],
                            d["p_zones"].shape[1], Fam, inh, device, options=options)


def _loglik(eng, kernel, zos, w, pg, pz, pf, src):
    """Host entry (sbz_loglik_batch, sources by site), for kernel 'hpm' the host entry with the
    sources by position (sbz_loglik_batch_pm: no transpose), or for kernel 'pm' the device entry with
    the sources by position (sbz_loglik_batch_device_pm: the layout the sampler keeps, read in place)."""
    if kernel == "hpm" and src is not None:
        out = eng.loglik(zos, w, pg, pz, pf, eng.sources_to_positions(src), source_pm=True)
        assert eng.last_kernels() in ("lik_source_rc_kernel", "lik_source_generic_kernel")
        return out
    if kernel != "pm" or src is None:
        return eng.loglik(zos, w, pg, pz, pf, src)
    import torch
    dev = torch.device("cuda:0")
    B = zos.shape[0]
    t = [torch.from_numpy(np.ascontiguousarray(v)).to(dev) if v is not None else None
         for v in (zos, w, pg, pz, pf, eng.sources_to_positions(src))]
    out = torch.empty(B, dtype=torch.float64, device=dev)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.loglik_device(B, *[x.data_ptr() if x is not None else 0 for x in t], out.data_ptr(),
                      source_pm=True)
    torch.cuda.synchronize()
    assert eng.last_kernels() in ("lik_source_rc_kernel", "lik_source_generic_kernel")
    return out.cpu().numpy()


def _assert_close(got, ref, tol=REL_TOL):
    got, ref = np.asarray(got), np.asarray(ref)
    inf = ~np.isfinite(ref)
    np.testing.assert_array_equal(got[inf], ref[inf])
    fin = ~inf
    rel = np.abs(got[fin] - ref[fin]) / np.abs(ref[fin])
    assert rel.size == 0 or rel.max() <= tol, f"max rel err {rel.max():.3e}"
    return 0.0 if rel.size == 0 else float(rel.max())


# Kernel paths: the dense mixture kernel with its banked table layout (the default where
# S + 1 <= 16) and with the packed [class][x] layout (option lik_banked = 0, the layout of every
# larger S); the source branch on the table kernel (default) with the sources by site (transposed
# to positions first) and by position (read in place, 'pm'), and on the generic per-cell kernel
# (option src_table = 0, the path of shapes the table kernel does not take).
MODES = [("mixture", "dense"), ("mixture", "packed"), ("source", "rc"), ("source", "pm"),
         ("source", "hpm"), ("source", "generic")]


def _options(kernel):
    return {"lik_banked": 0 if kernel == "packed" else 1, "src_table": 0 if kernel == "generic" else 1}


@pytest.fixture
def lik_kernel(request):
    return request.param


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("mode,lik_kernel", MODES, indirect=["lik_kernel"])
def test_golden(gpu_available, case, mode, lik_kernel):
    d = load_golden(case)
    eng = _engine(d, options=_options(lik_kernel))
    src = d["source"] if mode == "source" else None
    got = _loglik(eng, lik_kernel, d["zone_of_site"], d["w"], d["p_global"], d["p_zones"], d.get("p_fam"), src)
    _assert_close(got, d["ll_" + mode])


def test_known_answer(gpu_available):
    from contact_zones_amd.likelihood import LikelihoodEngine
    d = load_golden("lik_kat")
    S = d["p_global"].shape[2]
    e3 = LikelihoodEngine(d["obs"], d["fam_of_site"], S, 1, 1, True)
    e2 = LikelihoodEngine(d["obs"], d["fam_of_site"], S, 1, 0, False)
    lf = e3.loglik(d["zone_of_site"], d["w3"], d["p_global"], d["p_zones"], d["p_fam"])[0]
    ln = e2.loglik(d["zone_of_site"], d["w2"], d["p_global"], d["p_zones"])[0]
    assert lf == pytest.approx(float(d["lh_with_family"]), rel=1e-13)
    assert ln == pytest.approx(float(d["lh_without_family"]), rel=1e-13)
    assert lf == pytest.approx(float(d["lh_direct"]), rel=1e-12)


def _random_batch(rng, N, F, S, Z, Fam, B, inheritance, zone_size, na=0.02, nofam=0.2):
    obs = rng.integers(0, S, size=(N, F)).astype(np.int8)
    obs[rng.random((N, F)) < na] = -1
    fam = rng.integers(0, max(Fam, 1), size=N).astype(np.uint8)
    fam[rng.random(N) < nofam] = 255
    if Fam == 0:
        fam[:] = 255
    zos = np.full((B, N), 255, np.uint8)
    for b in range(B):
        perm = rng.permutation(N)
        for z in range(Z):
            zos[b, perm[z * zone_size:(z + 1) * zone_size]] = z
    C = 3 if inheritance else 2
    w = rng.dirichlet(np.ones(C), size=(B, F))
    pg = rng.dirichlet(np.ones(S), size=(B, F))
    pz = rng.dirichlet(np.ones(S), size=(B, Z, F))
    pf = rng.dirichlet(np.ones(S), size=(B, Fam, F)) if inheritance else None
    src = rng.integers(0, 1, size=(B, N, F)).astype(np.uint8)
    src[(zos[:, :, None] != 255) & (rng.random((B, N, F)) < 0.5)] = 1
    if inheritance:
        src[(fam[None, :, None] != 255) & (rng.random((B, N, F)) < 0.25)] = 2
    return obs, fam, zos, w, pg, pz, pf, src


@pytest.mark.parametrize("shape", [
    (200, 100, 5, 2, 0, 64, False, 25),      # cfg2, 64 chains
    (28, 47, 3, 3, 5, 256, True, 4),         # cfg3 shape, 256 chains
    (100, 36, 5, 6, 6, 128, True, 6),        # cfg4 shape, 128 chains per GPU
    (2000, 500, 10, 8, 4, 4, True, 62),      # cfg5 shape (few chains vs the C oracle)
    (1000, 33, 7, 3, 2, 5, True, 100),       # ragged feature tile, odd S
])
@pytest.mark.parametrize("mode,lik_kernel", MODES, indirect=["lik_kernel"])
def test_random_vs_c_oracle(gpu_available, shape, mode, lik_kernel):
    from contact_zones_amd.likelihood import LikelihoodEngine
    from oracle import oracle_c
    N, F, S, Z, Fam, B, inh, zs = shape
    rng = np.random.default_rng(hash(shape) % 2**32)
    obs, fam, zos, w, pg, pz, pf, src = _random_batch(rng, N, F, S, Z, Fam, B, inh, zs)
    eng = LikelihoodEngine(obs, fam, S, Z, Fam, inh, options=_options(lik_kernel))
    s = src if mode == "source" else None
    got = _loglik(eng, lik_kernel, zos, w, pg, pz, pf, s)
    ref = oracle_c.loglik_batch(obs, fam, zos, w, pg, pz, pf, source=s, inheritance=inh)
    _assert_close(got, ref, tol=1e-12)


def test_deterministic_and_chain_independent(gpu_available):
    """Bit-identical re-runs; a chain's value does not depend on its batch neighbours."""
    from contact_zones_amd.likelihood import LikelihoodEngine
    rng = np.random.default_rng(7)
    obs, fam, zos, w, pg, pz, pf, src = _random_batch(rng, 300, 70, 6, 3, 2, 16, True, 20)
    eng = LikelihoodEngine(obs, fam, 6, 3, 2, True)
    a = eng.loglik(zos, w, pg, pz, pf)
    b = eng.loglik(zos, w, pg, pz, pf)
    np.testing.assert_array_equal(a, b)
    perm = rng.permutation(16)
    c = eng.loglik(zos[perm], w[perm], pg[perm], pz[perm], pf[perm])
    np.testing.assert_array_equal(c, a[perm])
    one = eng.loglik(zos[3:4], w[3:4], pg[3:4], pz[3:4], pf[3:4])
    np.testing.assert_array_equal(one, a[3:4])


def test_device_pointer_path_matches_host_path(gpu_available):
    import torch
    from contact_zones_amd.likelihood import LikelihoodEngine
    rng = np.random.default_rng(8)
    obs, fam, zos, w, pg, pz, pf, src = _random_batch(rng, 500, 64, 8, 4, 3, 32, True, 30)
    eng = LikelihoodEngine(obs, fam, 8, 4, 3, True)
    host = eng.loglik(zos, w, pg, pz, pf, src)
    dev = torch.device("cuda:0")
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
         for k, v in dict(zos=zos, w=w, pg=pg, pz=pz, pf=pf, src=src).items()}
    out = torch.empty(32, dtype=torch.float64, device=dev)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.loglik_device(32, t["zos"].data_ptr(), t["w"].data_ptr(), t["pg"].data_ptr(),
                      t["pz"].data_ptr(), t["pf"].data_ptr(), t["src"].data_ptr(), out.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), host)


def test_drop_in_likelihood_interface(gpu_available):
    """GpuLikelihood(data, inheritance)(sample, caching=False) on reference-form inputs."""
    from collections import namedtuple
    from contact_zones_amd import packing
    from contact_zones_amd.likelihood import GpuLikelihood
    d = load_golden("lik_cfg3_balkan")
    S = d["p_global"].shape[2]
    Fam = d["p_fam"].shape[1]
    Data = namedtuple("Data", ["features", "families"])
    data = Data(features=packing.obs_to_features(d["obs"], S),
                families=packing.index_to_groups(d["fam_of_site"], Fam))

    class Sample:  # the attributes Likelihood.__call__ reads (zone_sampling.py:49-93)
        def __init__(self, b, source):
            self.zones = packing.index_to_groups(d["zone_of_site"][b], d["p_zones"].shape[1])
            self.weights = d["w"][b]
            self.p_global = d["p_global"][b][None]
            self.p_zones = d["p_zones"][b]
            self.p_families = d["p_fam"][b]
            self.source = packing.index_to_source(d["source"][b], 3) if source else None
            self.what_changed = None

    lik = GpuLikelihood(data, inheritance=True)
    for b in range(d["zone_of_site"].shape[0]):
        assert lik(Sample(b, False), caching=False) == pytest.approx(d["ll_mixture"][b], rel=1e-12)
        assert lik(Sample(b, True)) == pytest.approx(d["ll_source"][b], rel=1e-12)


@pytest.mark.parametrize("banked", ["1", "0"])
@pytest.mark.parametrize("shape", [(1500, 40, 6, 4, 3, 9), (2000, 64, 10, 8, 4, 9), (300, 21, 15, 3, 2, 9)])
def test_dense_edge_paths(gpu_available, banked, shape):
    """Dense kernel (banked and packed table layouts) on inputs that leave the fast path: zero
    cells (finite when another component covers them, -inf otherwise), tiny parameters whose
    products underflow (the task re-runs with per-factor renormalisation), parameters above 1
    and denormal parameters (per-feature renormalisation)."""
    from contact_zones_amd.likelihood import LikelihoodEngine
    from oracle import oracle_c
    N, F, S, Z, Fam, B = shape
    rng = np.random.default_rng(N + F)
    obs, fam, zos, w, pg, pz, pf, _ = _random_batch(rng, N, F, S, Z, Fam, B, True, N // (3 * Z))
    zoned34 = (zos[3] != 255) & (zos[4] != 255)
    obs[~zoned34 & (obs[:, 0] == 0), 0] = 1
    for b in (3, 4):
        pg[b, 0, 0] = 0.0
        pf[b, :, 0, 0] = 0.0
    s_out = int(np.flatnonzero(zos[4] == 255)[0])
    obs[s_out, 0] = 0
    zos[3, s_out] = 0
    pg[5, :, 1] = 1e-200                 # tiny: products underflow -> task re-run
    pz[6, :, :, 2] = 0.0                 # zero zoned cells
    pg[7, 3:9] *= 7.5                    # above 1 -> per-feature renormalisation
    pf[8, :, 5, :] = 4e-320              # denormal family parameters
    eng = LikelihoodEngine(obs, fam, S, Z, Fam, True, options={"lik_banked": int(banked)})
    got = eng.loglik(zos, w, pg, pz, pf)
    ref = oracle_c.loglik_batch(obs, fam, zos, w, pg, pz, pf, inheritance=True)
    assert np.isfinite(ref[3]) and ref[4] == -np.inf
    _assert_close(got, ref, tol=1e-12)
    assert eng.lds_bytes(False) > 0


@pytest.mark.parametrize("rc", ["rc", "pm", "generic"])
@pytest.mark.parametrize("shape", [(2000, 64, 10, 8, 4, 8), (300, 21, 15, 3, 2, 8), (120, 30, 4, 0, 3, 8)])
def test_source_edge_paths(gpu_available, rc, shape):
    """Source branch (row-code table kernel and the generic per-cell kernel): a selected component
    of weight 0 (-inf, model.py:181-182), tiny parameters (products underflow -> task re-run),
    parameters above 1, denormal family parameters, sources past the site's components."""
    from contact_zones_amd.likelihood import LikelihoodEngine
    from oracle import oracle_c
    N, F, S, Z, Fam, B = shape
    rng = np.random.default_rng(N * 3 + F)
    obs, fam, zos, w, pg, pz, pf, src = _random_batch(rng, N, F, S, Z, Fam, B, True, max(1, N // (3 * max(Z, 1))))
    w[3, 5, 1] = 0.0                    # zone weight 0 where a zoned site selects the zone
    if Z:
        s3 = int(np.flatnonzero(zos[3] != 255)[0])
        src[3, s3, 5] = 1
    else:
        # family weight 0 where a site with a family selects its family
        w[3, 5, 2] = 0.0
        src[3, int(np.flatnonzero(fam != 255)[0]), 5] = 2
    pg[4, :, 1] = 1e-200                # tiny
    pg[5, 3:9] *= 7.5                   # above 1
    pf[6, :, 2, :] = 4e-320             # denormal family parameters
    src[7, :, 0] = 0                    # every site from the global component at feature 0
    s2 = int(np.flatnonzero(fam == 255)[0])
    src[2, s2, 1] = 2                   # a site without family selects the family component
    eng = LikelihoodEngine(obs, fam, S, Z, Fam, True, options=_options(rc))
    got = _loglik(eng, rc, zos, w, pg, pz, pf, src)
    ref = oracle_c.loglik_batch(obs, fam, zos, w, pg, pz, pf, source=src, inheritance=True)
    assert ref[3] == -np.inf and ref[2] == -np.inf
    _assert_close(got, ref, tol=1e-12)


def test_chain_tickets_rearm_across_launches(gpu_available):
    """The last-task reduction re-arms each chain's ticket: back-to-back launches of different
    batch sizes (and task counts) reproduce single-chain values bit for bit."""
    from contact_zones_amd.likelihood import LikelihoodEngine
    rng = np.random.default_rng(21)
    obs, fam, zos, w, pg, pz, pf, _ = _random_batch(rng, 700, 90, 5, 3, 2, 24, True, 30)
    eng = LikelihoodEngine(obs, fam, 5, 3, 2, True)
    ref = np.concatenate([eng.loglik(zos[b:b + 1], w[b:b + 1], pg[b:b + 1], pz[b:b + 1], pf[b:b + 1])
                          for b in range(24)])
    for sl in (slice(0, 24), slice(3, 8), slice(0, 1), slice(5, 22), slice(0, 24)):
        got = eng.loglik(zos[sl], w[sl], pg[sl], pz[sl], pf[sl])
        np.testing.assert_array_equal(got, ref[sl])


def test_partials_handoff_stress(gpu_available):
    """The cross-workgroup hand-off of the task partials (finish_chain, sbz_lik.hip) under uneven
    load: 512 chains x W > 1 tasks spread over every XCD, launched back to back with varying batch
    sizes while another stream keeps the HBM busy.  A stale partial would change a chain's sum;
    every launch must reproduce a quiet launch of the same batch size bit for bit (the task split,
    W, depends on the batch size, so different sizes may differ in the last ulp), and the quiet
    launches must match the oracle."""
    import torch
    from contact_zones_amd.likelihood import LikelihoodEngine
    from oracle import oracle_c
    rng = np.random.default_rng(31)
    B = 512
    obs, fam, zos, w, pg, pz, pf, _ = _random_batch(rng, 300, 240, 6, 4, 3, B, True, 12)
    eng = LikelihoodEngine(obs, fam, 6, 4, 3, True)
    dev = torch.device("cuda:0")
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
         for k, v in dict(zos=zos, w=w, pg=pg, pz=pz, pf=pf).items()}
    main = torch.cuda.Stream()
    noise = torch.cuda.Stream()
    big = torch.empty(64 << 20, dtype=torch.float32, device=dev)
    eng.set_stream(main.cuda_stream)
    sizes = (B, 384, 100, 26, 7)
    quiet = {nb: eng.loglik(zos[:nb], w[:nb], pg[:nb], pz[:nb], pf[:nb]) for nb in sizes}
    outs = []
    for it in range(40):
        nb = sizes[it % len(sizes)] if it % 2 == 0 else sizes[int(rng.integers(0, len(sizes)))]
        out = torch.full((B,), np.nan, dtype=torch.float64, device=dev)
        with torch.cuda.stream(noise):
            big.mul_(1.0000001)  # keep HBM / other CUs busy while the chains finish
        with torch.cuda.stream(main):
            eng.loglik_device(nb, t["zos"].data_ptr(), t["w"].data_ptr(), t["pg"].data_ptr(),
                              t["pz"].data_ptr(), t["pf"].data_ptr(), 0, out.data_ptr(), validate=False)
        outs.append((nb, out))
    torch.cuda.synchronize()
    for nb, out in outs:
        np.testing.assert_array_equal(out.cpu().numpy()[:nb], quiet[nb])
    oracle = oracle_c.loglik_batch(obs, fam, zos[:8], w[:8], pg[:8], pz[:8], pf[:8], inheritance=True)
    for nb in sizes:
        _assert_close(quiet[nb][:7], oracle[:7], 1e-12)


def test_device_index_validation(gpu_available):
    """The device entry points trust their index bytes; sbz_check_indices_device (and
    LikelihoodEngine.loglik_device's default validate=True) refuse out-of-range zones / sources
    with SBZ_EINVAL instead of letting the kernels read out of bounds."""
    import torch
    from contact_zones_amd._lib import SbzError
    from contact_zones_amd.likelihood import LikelihoodEngine
    rng = np.random.default_rng(5)
    obs, fam, zos, w, pg, pz, pf, src = _random_batch(rng, 120, 30, 4, 2, 2, 6, True, 10)
    eng = LikelihoodEngine(obs, fam, 4, 2, 2, True)
    dev = torch.device("cuda:0")
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
         for k, v in dict(zos=zos, w=w, pg=pg, pz=pz, pf=pf, src=src).items()}
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.check_indices_device(6, t["zos"].data_ptr(), t["src"].data_ptr())  # valid: no error
    out = torch.empty(6, dtype=torch.float64, device=dev)
    bad_z = t["zos"].clone()
    bad_z[4, 77] = 2  # n_zones = 2: zone index 2 is out of range
    with pytest.raises(SbzError, match="zone_of_site"):
        eng.check_indices_device(6, bad_z.data_ptr(), 0)
    with pytest.raises(SbzError, match="zone_of_site"):
        eng.loglik_device(6, bad_z.data_ptr(), t["w"].data_ptr(), t["pg"].data_ptr(),
                          t["pz"].data_ptr(), t["pf"].data_ptr(), 0, out.data_ptr())
    bad_s = t["src"].clone()
    bad_s[5, 119, 29] = 3  # C = 3
    with pytest.raises(SbzError, match="source"):
        eng.check_indices_device(6, t["zos"].data_ptr(), bad_s.data_ptr())
    # after the refusals the engine still evaluates correctly
    eng.loglik_device(6, t["zos"].data_ptr(), t["w"].data_ptr(), t["pg"].data_ptr(),
                      t["pz"].data_ptr(), t["pf"].data_ptr(), 0, out.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), eng.loglik(zos, w, pg, pz, pf))


@pytest.mark.parametrize("rc", ["rc", "pm", "generic"])
@pytest.mark.parametrize("S,Z,Fam,inh", [(15, 3, 3, True), (16, 3, 3, True), (17, 4, 3, True),
                                         (20, 5, 5, True), (31, 2, 0, False), (32, 2, 0, False),
                                         (40, 2, 0, False)])
def test_source_wide_state_tables(gpu_available, rc, S, Z, Fam, inh):
    """Source branch with many states: S + 1 > 16 leaves fewer than 4 lane groups of S + 1 lanes
    in a wave, so the row-code kernel writes its 4 T0 rows (and the 4 zero rows) by a strided
    loop over the groups; every (class, state) entry must be written (a missed T0 row would read
    stale LDS).  Both source kernels against the oracle, with the T0 rows of every class h in use
    (zoned / unzoned sites with and without a family, every component selected)."""
    from contact_zones_amd.likelihood import LikelihoodEngine
    from oracle import oracle_c
    N, F, B = 300, 23, 6
    rng = np.random.default_rng(1000 * S + Z)
    obs, fam, zos, w, pg, pz, pf, src = _random_batch(rng, N, F, S, Z, Fam, B, inh, 20, nofam=0.3)
    if not inh:
        src = np.minimum(src, 1).astype(np.uint8)
    eng = LikelihoodEngine(obs, fam, S, Z, Fam, inh, options=_options(rc))
    got = _loglik(eng, rc, zos, w, pg, pz, pf, src)
    ref = oracle_c.loglik_batch(obs, fam, zos, w, pg, pz, pf, source=src, inheritance=inh)
    assert np.all(np.isfinite(ref))
    _assert_close(got, ref, tol=1e-12)


@pytest.mark.parametrize("rc", ["rc", "pm", "generic"])
def test_source_zero_weight_beside_nan(gpu_available, rc):
    """model.py:181-182: a selected weight of exactly 0 gives -inf even when other selected
    weights are NaN (0 / 0); without a zero selected weight the NaN cells give NaN.  The chains
    are split over several tasks, so the zero and the NaN cells land in different tasks."""
    from contact_zones_amd.likelihood import LikelihoodEngine
    from oracle import oracle_c
    N, F, S, Z, Fam, B = 700, 90, 5, 3, 2, 4
    rng = np.random.default_rng(99)
    obs, fam, zos, w, pg, pz, pf, src = _random_batch(rng, N, F, S, Z, Fam, B, True, 40)
    for b in range(B):
        w[b, 3] = [0.0, 1.0, 0.0]        # no-zone sites: 0 / 0 weights (NaN cells)
        src[b, zos[b] != 255, 3] = 1
    z0 = int(np.flatnonzero(zos[0] != 255)[0])
    src[0, z0, 3] = 0                    # chain 0: a zoned site selects the global weight 0
    w[2, 80] = [0.0, 0.5, 0.5]           # chain 2: also a zero weight far from the NaN feature
    s2 = int(np.flatnonzero(zos[2] == 255)[0])
    src[2, s2, 80] = 0
    w[3, 3] = [0.2, 0.5, 0.3]            # chain 3: no NaN, no zero weight -> finite
    eng = LikelihoodEngine(obs, fam, S, Z, Fam, True, options=_options(rc))
    with np.errstate(invalid="ignore", divide="ignore"):
        ref = oracle_c.loglik_batch(obs, fam, zos, w, pg, pz, pf, source=src, inheritance=True)
    assert ref[0] == -np.inf and np.isnan(ref[1]) and ref[2] == -np.inf and np.isfinite(ref[3])
    for _ in range(2):  # the per-chain flag is re-armed between launches
        got = _loglik(eng, rc, zos, w, pg, pz, pf, src)
        _assert_close(got, ref, tol=1e-12)
    one = _loglik(eng, rc, zos[1:2], w[1:2], pg[1:2], pz[1:2], pf[1:2], src[1:2])
    assert np.isnan(one[0])


@pytest.mark.parametrize("B", [256, 2048])
@pytest.mark.parametrize("mode", ["mixture", "source"])
def test_bench_launch_parity(gpu_available, B, mode):
    """The exact launch bench.py times (BASELINE configs[4]: 2000 sites x 500 features x 10
    states, 8 zones of 50 sites, 4 families, device pointers, validate=False; the source branch
    with the sources by position, read in place) at the bench's chains per GPU (256) and at 2048
    chains on one GPU: the task split W depends on B, so these are the long-task shapes (12 tasks
    of ~42 features at B = 256, 2 of 250 at B = 2048) no smaller case reaches.  First, last and 8
    sampled chains against the C oracle."""
    import argparse
    import torch
    import bench
    from contact_zones_amd.likelihood import LikelihoodEngine
    from oracle import oracle_c
    args = argparse.Namespace(sites=2000, features=500, states=10, zones=8, families=4,
                              zone_size=50, mode=mode, seed=5)
    obs, fam = bench.make_shared(args, np.random.default_rng(args.seed))
    args._fam = fam
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + B)
    eng = LikelihoodEngine(obs, fam, 10, 8, 4, True)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    c = bench.make_chains_torch(args, B, gen, dev, eng)
    out = torch.empty(B, dtype=torch.float64, device=dev)
    src = c["src_pm"]
    for _ in range(2):  # twice: the second launch runs on re-armed tickets
        eng.loglik_device(B, c["zos"].data_ptr(), c["w"].data_ptr(), c["pg"].data_ptr(),
                          c["pz"].data_ptr(), c["pf"].data_ptr(),
                          src.data_ptr() if src is not None else 0, out.data_ptr(), validate=False,
                          source_pm=True)
    torch.cuda.synchronize()
    if mode == "source":
        assert eng.last_kernels() == "lik_source_rc_kernel"
    got = out.cpu().numpy()
    assert np.all(np.isfinite(got))
    pick = sorted({0, B - 1, *np.random.default_rng(B).choice(B, 8, replace=False).tolist()})
    h = {k: (v[pick].cpu().numpy() if v is not None else None) for k, v in c.items()}
    src_rm = eng.sources_from_positions(h["src_pm"]) if h["src_pm"] is not None else None
    ref = oracle_c.loglik_batch(obs, fam, h["zos"], h["w"], h["pg"], h["pz"], h["pf"],
                                source=src_rm, inheritance=True)
    _assert_close(got[pick], ref, tol=1e-12)


def test_source_layouts(gpu_available):
    """The two source layouts (include/sbz.h): sbz_site_positions is the stable family sort,
    sbz_source_layout_device transposes [B][N][F] <-> [B][F][Np] exactly as the host restatement
    (padding columns 0) and back to the identity, and sbz_check_indices_device_pm refuses a
    component >= C at a site position but not in the padding columns."""
    import torch
    from contact_zones_amd._lib import SbzError
    from contact_zones_amd.likelihood import LikelihoodEngine
    rng = np.random.default_rng(17)
    N, F, S, Z, Fam, B = 300, 45, 4, 2, 3, 5   # F not a multiple of 4: the byte path
    obs, fam, zos, w, pg, pz, pf, src = _random_batch(rng, N, F, S, Z, Fam, B, True, 10)
    eng = LikelihoodEngine(obs, fam, S, Z, Fam, True)
    fc = np.where(fam == 255, 0, fam.astype(int) + 1)
    np.testing.assert_array_equal(eng.positions[:N], np.argsort(fc, kind="stable"))
    assert np.all(eng.positions[N:] == -1) and eng.n_positions % 256 == 0
    dev = torch.device("cuda:0")
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    t_src = torch.from_numpy(src).to(dev)
    pm = torch.full((B, F, eng.n_positions), 7, dtype=torch.uint8, device=dev)
    eng.source_layout_device(B, t_src.data_ptr(), pm.data_ptr(), True)
    back = torch.empty_like(t_src)
    eng.source_layout_device(B, pm.data_ptr(), back.data_ptr(), False)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(pm.cpu().numpy(), eng.sources_to_positions(src))
    np.testing.assert_array_equal(back.cpu().numpy(), src)
    np.testing.assert_array_equal(eng.sources_from_positions(pm.cpu().numpy()), src)
    t_zos = torch.from_numpy(zos).to(dev)
    pm[:, :, N:] = 9  # padding: never read, never checked
    eng.check_indices_device(B, t_zos.data_ptr(), pm.data_ptr(), source_pm=True)
    pm[2, 7, N - 1] = 3
    with pytest.raises(SbzError, match="source"):
        eng.check_indices_device(B, t_zos.data_ptr(), pm.data_ptr(), source_pm=True)


def test_options(gpu_available):
    """Context options (sbz_set_option) replace the environment: defaults, round trip, range
    checks, and the likelihood unchanged by the table layout / tasks-per-CU choices."""
    from contact_zones_amd._lib import SbzError
    from contact_zones_amd.likelihood import LikelihoodEngine
    rng = np.random.default_rng(23)
    obs, fam, zos, w, pg, pz, pf, _ = _random_batch(rng, 200, 100, 5, 2, 2, 64, True, 25)
    eng = LikelihoodEngine(obs, fam, 5, 2, 2, True)
    assert {k: eng.get_option(k) for k in ("lik_tasks_per_cu", "lik_banked", "src_table", "src_waves",
                                           "src_hbm", "src_stage", "mh_lookahead", "mh_group", "src_pack")} == \
        {"lik_tasks_per_cu": 0, "lik_banked": 1, "src_table": 1, "src_waves": 0, "src_hbm": 0,
         "src_stage": 1, "mh_lookahead": 24, "mh_group": 8, "src_pack": 1}
    ref = eng.loglik(zos, w, pg, pz, pf)
    for tpc in (1, 2, 4, 12):
        eng.set_option("lik_tasks_per_cu", tpc)
        _assert_close(eng.loglik(zos, w, pg, pz, pf), ref, tol=1e-14)
    for name, bad in (("lik_tasks_per_cu", -1), ("lik_banked", 2), ("src_waves", 3), ("mh_lookahead", 0),
                      ("mh_lookahead", 25), ("mh_group", 0), ("mh_group", 9), ("src_pack", 2)):
        with pytest.raises(SbzError):
            eng.set_option(name, bad)
    with pytest.raises(ValueError):
        eng.set_option("no_such_option", 1)


@pytest.mark.parametrize("shape", [
    (700, 92, 5, 3, 2, 6, True, 40),        # 16 sites per lane (planes of 4 groups)
    (1100, 64, 10, 8, 4, 6, True, 30),      # 32 sites per lane, one 2048-position chunk
    (3000, 20, 4, 2, 0, 5, False, 200),     # two chunks, no families, C = 2
    (2000, 500, 10, 8, 4, 3, True, 50),     # cfg5
    (600, 16, 3, 1, 1, 4, True, 100),       # F = 16: one feature tile, 128-B loads past the row end
])
def test_source_by_site_planes(gpu_available, shape):
    """The by-site source entry (sbz_loglik_batch, the reference's Sample.source order) where it
    reorders the sources into 2-bit planes (source_to_pk_kernel, option src_pack = 1, the default
    for N > 512 and F a multiple of 4): bit-identical to the byte reorder (src_pack = 0; the same
    table rows in the same order), within 1e-12 of the C oracle, through the host and the device
    entries, with a zero selected weight (-inf) and tiny parameters (task re-run) in the batch."""
    import torch
    from contact_zones_amd.likelihood import LikelihoodEngine
    from oracle import oracle_c
    N, F, S, Z, Fam, B, inh, zs = shape
    rng = np.random.default_rng(N + 7 * F)
    obs, fam, zos, w, pg, pz, pf, src = _random_batch(rng, N, F, S, Z, Fam, B, inh, zs)
    if not inh:
        src = np.minimum(src, 1).astype(np.uint8)
    s1 = int(np.flatnonzero(zos[1] != 255)[0])
    w[1, F - 1, 1] = 0.0                # chain 1: a zoned site selects a zone weight of 0 -> -inf
    src[1, s1, F - 1] = 1
    pg[2, :, 1] = 1e-200                # chain 2: tiny parameters, products underflow
    eng = LikelihoodEngine(obs, fam, S, Z, Fam, inh)
    planes = eng.loglik(zos, w, pg, pz, pf, src)
    assert eng.last_kernels() == "source_to_pk_kernel lik_source_rc_kernel<planes>"
    eng.set_option("src_pack", 0)
    byte = eng.loglik(zos, w, pg, pz, pf, src)
    assert eng.last_kernels() == "source_to_pm_kernel lik_source_rc_kernel"
    np.testing.assert_array_equal(planes, byte)
    ref = oracle_c.loglik_batch(obs, fam, zos, w, pg, pz, pf, source=src, inheritance=inh)
    assert ref[1] == -np.inf
    _assert_close(planes, ref, tol=1e-12)
    eng.set_option("src_pack", 1)
    dev = torch.device("cuda:0")
    t = [torch.from_numpy(np.ascontiguousarray(v)).to(dev) if v is not None else None
         for v in (zos, w, pg, pz, pf, src)]
    out = torch.empty(B, dtype=torch.float64, device=dev)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.loglik_device(B, *[x.data_ptr() if x is not None else 0 for x in t], out.data_ptr())
    torch.cuda.synchronize()
    assert eng.last_kernels() == "source_to_pk_kernel lik_source_rc_kernel<planes>"
    np.testing.assert_array_equal(out.cpu().numpy(), planes)
