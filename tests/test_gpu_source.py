"""GPU parity of the SAMPLE_SOURCE = true sampler (sbz_mh_src.hip): replaying the reference's
decision tapes (tests/golden/mh_src_*.npz, make_golden_mh.py — seeded ZoneMCMC / ZoneMCMCWarmup
with sample_source) reproduces every step's operator, accept flag, zone assignment and the
final sources bit for bit; Gibbs-drawn parameters are bit-exact too (same tape, same arithmetic),
log-likelihoods within the north_star tolerance of 1e-9 relative."""
import numpy as np
import pytest

from conftest import prior_spec, load_golden, mh_cases

pytestmark = pytest.mark.gpu

SRC_CASES = mh_cases(source=True)
REL_TOL = 1e-9


@pytest.fixture(params=["lds", "hbm", "lds-w1", "hbm-w4", "hbmcell"])
def src_home(request):
    """Context options: where the sampler keeps the sources — LDS (when they fit) or HBM (option
    src_hbm = 1, the path every N x F too large for LDS takes, walking the sources by position, on
    per-feature tables with per-chain count tables; 'hbmcell': the per-cell passes instead,
    src_pass_tables = 0, the path of shapes whose tables do not fit) — and the waves per chain
    (default 8, or src_waves = 1 / 4)."""
    home, _, waves = request.param.partition("-w")
    opts = {"src_hbm": 1 if home.startswith("hbm") else 0, "src_waves": int(waves or 0)}
    if home == "hbmcell":
        opts["src_pass_tables"] = 0
    return opts


def _setup(fx, options=None):
    from contact_zones_amd.likelihood import LikelihoodEngine
    from contact_zones_amd.priors import PriorSpec
    from contact_zones_amd.sampler import ChainState, Sampler
    inh = bool(fx["inheritance"])
    S = fx["states"].shape[1]
    Z = int(fx["n_zones"])
    Fam = fx["init_p_fam"].shape[1] if inh else 0
    eng = LikelihoodEngine(fx["obs"], fx["fam_of_site"], S, Z, Fam, inh, options=options)
    priors = prior_spec(fx)
    smp = Sampler(eng, fx["states"], fx["adj_indptr"], fx["adj_indices"], fx["op_probs"],
                  fx["precision"], int(fx["min_size"]), warmup=bool(fx["warmup"]), priors=priors,
                  sample_source=True,
                  gibbs_counts=(fx["gibbs_counts_global"], fx["gibbs_counts_fam"] if inh else None))
    st = ChainState(eng, fx["init_zone_of_site"], fx["init_w"], fx["init_p_global"],
                    fx["init_p_zones"], fx["init_p_fam"] if inh else None, prior=fx["init_prior"],
                    source=fx["init_source"])
    return eng, smp, st


def _check_final(fx, st, inh):
    s = st.to_numpy()
    np.testing.assert_array_equal(s["source"], fx["step_source"][:, -1])
    np.testing.assert_array_equal(s["w"], fx["final_w"])
    np.testing.assert_array_equal(s["p_global"], fx["final_p_global"])
    np.testing.assert_array_equal(s["p_zones"], fx["final_p_zones"])
    if inh:
        np.testing.assert_array_equal(s["p_fam"], fx["final_p_fam"])


@pytest.mark.parametrize("case", SRC_CASES)
def test_source_tape_replay_matches_reference(gpu_available, case, src_home):
    import torch
    fx = load_golden(case)
    inh = bool(fx["inheritance"])
    eng, smp, st = _setup(fx, src_home)
    n_steps = fx["step_op"].shape[1]
    out = smp.run(st, n_steps, fx["max_size"], fx["p_grow_connected"], tape=fx["tape"],
                  tape_len=fx["tape_len"], trace=True, trace_zones=True)
    torch.cuda.synchronize()
    assert out["status"].cpu().numpy().tolist() == [0] * st.B
    np.testing.assert_array_equal(out["tape_pos"].cpu().numpy(), fx["tape_len"])
    np.testing.assert_array_equal(out["op"].cpu().numpy(), fx["step_op"])
    np.testing.assert_array_equal(out["accept"].cpu().numpy().astype(bool), fx["step_accept"])
    np.testing.assert_array_equal(out["zone_of_site"].cpu().numpy(), fx["step_zone_of_site"])
    ll = out["ll"].cpu().numpy()
    rel = np.abs(ll - fx["step_ll"]) / np.abs(fx["step_ll"])
    assert rel.max() <= REL_TOL, rel.max()
    _check_final(fx, st, inh)
    np.testing.assert_allclose(st.prior.cpu().numpy(), fx["step_prior"][:, -1], rtol=1e-12, atol=1e-12)
    # the tracked source log-likelihood equals a fresh evaluation of the final state
    final = st.ll.cpu().numpy().copy()
    fresh = st.refresh_ll().cpu().numpy()
    assert np.max(np.abs(final - fresh) / np.abs(fresh)) <= REL_TOL
    acc, prop = st.accepted.cpu().numpy(), st.proposed.cpu().numpy()
    for b in range(st.B):
        ops = fx["step_op"][b]
        np.testing.assert_array_equal(prop[b, :13], np.bincount(ops, minlength=13)[:13])
        np.testing.assert_array_equal(acc[b, :13], np.bincount(ops[fx["step_accept"][b]], minlength=13)[:13])


def test_source_tape_replay_in_chunks(gpu_available):
    """Several launches (sources and cursor carried in HBM) give the same trajectory."""
    import torch
    fx = load_golden(SRC_CASES[0])
    eng, smp, st = _setup(fx)
    n = fx["step_op"].shape[1]
    pos = torch.zeros(st.B, dtype=torch.int64, device=st.ll.device)
    ops = []
    for a, b in [(0, 5), (5, 77), (77, n)]:
        out = smp.run(st, b - a, fx["max_size"], fx["p_grow_connected"], tape=fx["tape"],
                      tape_len=fx["tape_len"], tape_pos=pos, trace=True)
        ops.append(out["op"].cpu().numpy())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(np.concatenate(ops, axis=1), fx["step_op"])
    _check_final(fx, st, bool(fx["inheritance"]))


def test_source_philox_chains_are_valid(gpu_available, src_home):
    """Philox draws: every observation's source is a component it can come from (zone only inside
    a zone, inheritance only inside a family), the parameters stay normalised, the tracked ll
    equals a fresh evaluation and the carried prior the full prior; the run is reproducible."""
    import torch
    from contact_zones_amd.priors import PriorSpec
    fx = load_golden("mh_src_small")
    eng, smp, st = _setup(fx, src_home)
    out = smp.run(st, 3000, fx["max_size"], fx["p_grow_connected"], seed=77)
    torch.cuda.synchronize()
    assert out["status"].cpu().numpy().tolist() == [0] * st.B
    s = st.to_numpy()
    src = s["source"]
    assert src.max() <= 2
    in_zone = s["zone_of_site"] < 255
    assert not np.any((src == 1) & ~in_zone[:, :, None])
    in_fam = fx["fam_of_site"] < 255
    assert not np.any((src == 2) & ~in_fam[None, :, None])
    np.testing.assert_allclose(s["w"].sum(-1), 1.0, rtol=1e-12)
    np.testing.assert_allclose(s["p_global"].sum(-1), 1.0, rtol=1e-12)
    np.testing.assert_allclose(s["p_zones"].sum(-1), 1.0, rtol=1e-12)
    fresh = st.refresh_ll().cpu().numpy()
    assert np.max(np.abs(s["ll"] - fresh) / np.abs(fresh)) <= REL_TOL
    spec = prior_spec(fx)
    full = spec.log_prior(s["zone_of_site"], s["p_global"], s["p_fam"], fx["states"],
                          int(fx["n_zones"]), bool(fx["inheritance"]))
    np.testing.assert_allclose(s["prior"], full, rtol=1e-12, atol=1e-12)
    assert st.accepted.sum().item() > 100
    eng2, smp2, st2 = _setup(fx, src_home)
    smp2.run(st2, 3000, fx["max_size"], fx["p_grow_connected"], seed=77)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(st2.source.cpu().numpy(), src)
    np.testing.assert_array_equal(st2.zone_of_site.cpu().numpy(), s["zone_of_site"])


def test_source_sampler_large_sources_in_hbm(gpu_available):
    """N x F = 100k observations (200 KB of sources per chain, beyond LDS): the sampler keeps the
    sources in HBM; Philox steps keep every invariant and the tracked ll equals a fresh
    evaluation."""
    import torch
    from scipy.spatial import Delaunay

    from contact_zones_amd.likelihood import LikelihoodEngine
    from contact_zones_amd.sampler import ChainState, Sampler
    fx = load_golden("mh_src_small")
    rng = np.random.default_rng(4)
    N, F, S, Z, Fam, B = 400, 250, 4, 2, 2, 4
    obs = rng.integers(0, S, size=(N, F)).astype(np.int8)
    obs[rng.random((N, F)) < 0.02] = -1
    fam = rng.integers(0, Fam, size=N).astype(np.uint8)
    fam[rng.random(N) < 0.3] = 255
    states = np.ones((F, S), bool)
    indptr, indices = Delaunay(rng.random((N, 2))).vertex_neighbor_vertices
    eng = LikelihoodEngine(obs, fam, S, Z, Fam, True)
    assert eng.lds_bytes() >= 0
    smp = Sampler(eng, states, indptr, indices, fx["op_probs"], fx["precision"], 3, sample_source=True)
    zos = np.full((B, N), 255, np.uint8)
    for b in range(B):
        p = rng.permutation(N)
        zos[b, p[:10]], zos[b, p[10:20]] = 0, 1
    w = rng.dirichlet(np.ones(3), size=(B, F))
    pg = rng.dirichlet(np.ones(S), size=(B, F))
    pz = rng.dirichlet(np.ones(S), size=(B, Z, F))
    pf = rng.dirichlet(np.ones(S), size=(B, Fam, F))
    st = ChainState(eng, zos, w, pg, pz, pf, source=np.zeros((B, N, F), np.uint8))
    out = smp.run(st, 60, np.full(B, 50), np.full(B, 0.85), seed=5)
    torch.cuda.synchronize()
    assert out["status"].cpu().numpy().tolist() == [0] * B
    s = st.to_numpy()
    src = s["source"]
    assert not np.any((src == 1) & (s["zone_of_site"] == 255)[:, :, None])
    assert not np.any((src == 2) & (fam == 255)[None, :, None])
    assert np.any(src == 1) and np.any(src == 2)  # the Gibbs source draws ran
    np.testing.assert_allclose(s["p_global"].sum(-1), 1.0, rtol=1e-12)
    fresh = st.refresh_ll().cpu().numpy()
    assert np.all(np.isfinite(fresh))
    assert np.max(np.abs(s["ll"] - fresh) / np.abs(fresh)) <= REL_TOL


def test_source_sampler_lds_limit_fails_loudly(gpu_available):
    """A shape whose per-chain Gibbs scratch (F x S doubles of redraws, beside the counts) exceeds
    the 160 KiB of LDS even with the sources in HBM: the launch is refused with an error that names
    the LDS budget (include/sbz.h), nothing runs and no chain state changes."""
    from scipy.spatial import Delaunay

    from contact_zones_amd.likelihood import LikelihoodEngine
    from contact_zones_amd.sampler import ChainState, Sampler
    fx = load_golden("mh_src_small")
    rng = np.random.default_rng(9)
    N, F, S, Z, Fam, B = 40, 2100, 10, 1, 1, 2
    obs = rng.integers(0, S, size=(N, F)).astype(np.int8)
    fam = np.zeros(N, np.uint8)
    indptr, indices = Delaunay(rng.random((N, 2))).vertex_neighbor_vertices
    eng = LikelihoodEngine(obs, fam, S, Z, Fam, True)
    smp = Sampler(eng, np.ones((F, S), bool), indptr, indices, fx["op_probs"], fx["precision"], 3,
                  sample_source=True)
    zos = np.full((B, N), 255, np.uint8)
    zos[:, :5] = 0
    st = ChainState(eng, zos, rng.dirichlet(np.ones(3), size=(B, F)), rng.dirichlet(np.ones(S), size=(B, F)),
                    rng.dirichlet(np.ones(S), size=(B, Z, F)), rng.dirichlet(np.ones(S), size=(B, Fam, F)),
                    source=np.zeros((B, N, F), np.uint8))
    before = st.to_numpy()
    with pytest.raises(Exception, match="LDS"):
        smp.run(st, 10, np.full(B, 20), np.full(B, 0.85), seed=5)
    after = st.to_numpy()
    np.testing.assert_array_equal(after["zone_of_site"], before["zone_of_site"])
    np.testing.assert_array_equal(after["p_global"], before["p_global"])


@pytest.mark.parametrize("home", ["lds", "hbm"])
def test_source_host_form_replays_reference(gpu_available, home):
    """sbz_mh_run with SAMPLE_SOURCE: the host form takes the sources BY SITE ([B][N][F], the
    reference's order; the sampler copies them in and out of LDS, or transposes them to positions
    around an HBM run), the device form (ChainState) keeps them BY POSITION.  Both replay the
    reference's tape: operators, accepts, final sources and parameters bit for bit."""
    from contact_zones_amd.sampler import run_host
    fx = load_golden("mh_src_small")
    inh = bool(fx["inheritance"])
    eng, smp, st = _setup(fx, {"src_hbm": 1 if home == "hbm" else 0})
    n_steps = fx["step_op"].shape[1]
    host = {"zone_of_site": fx["init_zone_of_site"].copy(), "w": fx["init_w"].copy(),
            "p_global": fx["init_p_global"].copy(), "p_zones": fx["init_p_zones"].copy(),
            "p_fam": fx["init_p_fam"].copy() if inh else None, "source": fx["init_source"].copy(),
            "prior": np.broadcast_to(np.asarray(fx["init_prior"], np.float64), (st.B,)).copy()}
    tr = run_host(smp, host, n_steps, fx["max_size"], fx["p_grow_connected"], tape=fx["tape"],
                  tape_len=fx["tape_len"], trace=True)
    assert host["status"].tolist() == [0] * st.B
    np.testing.assert_array_equal(tr["op"], fx["step_op"])
    np.testing.assert_array_equal(tr["accept"].astype(bool), fx["step_accept"])
    np.testing.assert_array_equal(host["source"], fx["step_source"][:, -1])
    np.testing.assert_array_equal(host["w"], fx["final_w"])
    np.testing.assert_array_equal(host["p_zones"], fx["final_p_zones"])
    assert np.max(np.abs(tr["ll"] - fx["step_ll"]) / np.abs(fx["step_ll"])) <= REL_TOL
    smp.run(st, n_steps, fx["max_size"], fx["p_grow_connected"], tape=fx["tape"], tape_len=fx["tape_len"])
    dev = st.to_numpy()
    for k in ("zone_of_site", "w", "p_global", "p_zones", "source") + (("p_fam",) if inh else ()):
        np.testing.assert_array_equal(host[k], dev[k], err_msg=k)


@pytest.mark.parametrize("case", ["mh_src_gibbsish_small", "mh_src_gibbsish_warmup", "mh_src_geo"])
def test_source_philox_gibbsish_invariants(gpu_available, case, src_home):
    """gibbsish_sample_zones with source resampling of the available sites, Philox draws (weight
    set to the zone moves' total where the fixture has none): sources only from components the
    site has, zones within [MIN_M, max_size], tracked ll = a fresh evaluation, carried prior =
    the full prior (geo prior's last-zone MST included), reproducible."""
    import torch
    fx = dict(load_golden(case))
    probs = fx["op_probs"].copy()
    if probs[7] == 0:
        probs[7] = probs[:3].sum()
    fx["op_probs"] = probs
    finals = []
    for _ in range(2):
        eng, smp, st = _setup(fx, src_home)
        out = smp.run(st, 1200, fx["max_size"], fx["p_grow_connected"], seed=313, trace=True)
        torch.cuda.synchronize()
        assert out["status"].cpu().numpy().tolist() == [0] * st.B
        s = st.to_numpy()
        finals.append(s)
    src = s["source"]
    in_zone = s["zone_of_site"] < 255
    assert not np.any((src == 1) & ~in_zone[:, :, None])
    in_fam = fx["fam_of_site"] < 255
    assert not np.any((src == 2) & ~in_fam[None, :, None])
    Z = int(fx["n_zones"])
    for b in range(st.B):
        sizes = np.bincount(s["zone_of_site"][b][s["zone_of_site"][b] < 255], minlength=Z)
        assert np.all(sizes >= int(fx["min_size"])) and np.all(sizes <= fx["max_size"][b])
    fresh = st.refresh_ll().cpu().numpy()
    assert np.max(np.abs(s["ll"] - fresh) / np.abs(fresh)) <= REL_TOL
    full = prior_spec(fx).log_prior(s["zone_of_site"], s["p_global"], s.get("p_fam"), fx["states"],
                                    Z, bool(fx["inheritance"]))
    np.testing.assert_allclose(s["prior"], full, rtol=1e-12, atol=1e-12)
    ops = out["op"].cpu().numpy()
    assert (ops == 7).sum() > 50
    assert ((ops == 7) & (out["accept"].cpu().numpy() != 0)).sum() > 5
    for k in finals[0]:
        np.testing.assert_array_equal(finals[0][k], finals[1][k], err_msg=k)


def test_concurrent_contexts_match_sequential(gpu_available):
    """Two contexts sampling on their own HIP streams at once (the bench's concurrent K sweep)
    give exactly the states they give when run one after the other."""
    import torch
    cases = ["mh_src_sa_z1", "mh_src_sa_z6"]

    def run(concurrent):
        setups = [_setup(load_golden(c)) for c in cases]
        streams = [torch.cuda.Stream() for _ in cases] if concurrent else [torch.cuda.current_stream()] * 2
        torch.cuda.synchronize()
        for (eng, smp, st), c, s in zip(setups, cases, streams):
            fx = load_golden(c)
            with torch.cuda.stream(s):
                smp.run(st, 800, fx["max_size"], fx["p_grow_connected"], seed=21, chain_id0=5)
        torch.cuda.synchronize()
        return [st.to_numpy() for _, _, st in setups]

    seq, con = run(False), run(True)
    for a, b in zip(seq, con):
        for k in a:
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_source_sampler_cfg5_philox_invariants(gpu_available):
    """The bench shape (cfg5: 2000 sites x 500 features x 10 states, 8 zones, 4 families, 256
    chains) on the default path — sources in HBM, per-feature table passes, per-chain count tables
    (eng.last_kernels() names it) — under the default SAMPLE_SOURCE = true operator mix with Philox
    draws: every source a component its site allows, zone sizes within [MIN_M, MAX_M], parameters
    normalised, the tracked ll equal to a fresh evaluation within 1e-9, and the run reproducible
    bit for bit from its seed."""
    import torch
    from scipy.spatial import Delaunay

    from contact_zones_amd.likelihood import LikelihoodEngine
    from contact_zones_amd.sampler import ChainState, Sampler, precisions
    rng = np.random.default_rng(55)
    N, F, S, Z, Fam, B = 2000, 500, 10, 8, 4, 256
    min_m, max_m = 3, 50
    obs = rng.integers(0, S, size=(N, F)).astype(np.int8)
    obs[rng.random((N, F)) < 0.02] = -1
    fam = rng.integers(0, Fam, size=N).astype(np.uint8)
    fam[rng.random(N) < 0.2] = 255
    states = np.ones((F, S), bool)
    indptr, indices = Delaunay(rng.random((N, 2))).vertex_neighbor_vertices
    eng = LikelihoodEngine(obs, fam, S, Z, Fam, True)
    ops = {"shrink_zone": 0.016, "grow_zone": 0.016, "swap_zone": 0.008, "gibbs_sample_weights": 0.4,
           "gibbs_sample_p_global": 0.05, "gibbs_sample_p_zones": 0.4, "gibbs_sample_p_families": 0.11}
    prec = precisions({"weights": 15, "universal": 40, "contact": 20, "inheritance": 20})

    def make():
        zos = np.full((B, N), 255, np.uint8)
        r = np.random.default_rng(56)
        for b in range(B):  # 8 disjoint zones of 5 random sites each
            p = r.permutation(N)[:5 * Z]
            for z in range(Z):
                zos[b, p[5 * z:5 * z + 5]] = z
        w = np.broadcast_to(r.dirichlet(np.ones(3), size=F), (B, F, 3)).copy()
        pg = np.broadcast_to(r.dirichlet(np.ones(S), size=F), (B, F, S)).copy()
        pz = r.dirichlet(np.ones(S), size=(B, Z, F))
        pf = np.broadcast_to(r.dirichlet(np.ones(S), size=(Fam, F)), (B, Fam, F, S)).copy()
        st = ChainState(eng, zos, w, pg, pz, pf, source=np.zeros((B, N, F), np.uint8))
        Sampler(eng, states, indptr, indices, {"gibbs_sample_sources": 1.0}, prec, min_m,
                sample_source=True).run(st, 1, np.full(B, max_m), np.full(B, 0.85), seed=11)
        smp = Sampler(eng, states, indptr, indices, ops, prec, min_m, sample_source=True)
        out = smp.run(st, 600, np.full(B, max_m), np.full(B, 0.85), seed=12, trace=True)
        torch.cuda.synchronize()
        return st, out

    st, out = make()
    assert "tables" in eng.last_kernels()
    assert out["status"].cpu().numpy().tolist() == [0] * B
    s = st.to_numpy()
    src = s["source"]
    assert src.max() <= 2
    zs = s["zone_of_site"]
    assert not np.any((src == 1) & (zs == 255)[:, :, None])
    assert not np.any((src == 2) & (fam == 255)[None, :, None])
    sizes = np.stack([(zs == z).sum(1) for z in range(Z)], 1)
    assert sizes.min() >= min_m and sizes.max() <= max_m
    for name in ("w", "p_global", "p_zones", "p_fam"):
        np.testing.assert_allclose(s[name].sum(-1), 1.0, rtol=1e-12)
    fresh = st.refresh_ll().cpu().numpy()
    assert np.all(np.isfinite(fresh))
    assert np.max(np.abs(s["ll"] - fresh) / np.abs(fresh)) <= REL_TOL
    acc = out["accept"].cpu().numpy()
    op = out["op"].cpu().numpy()
    assert acc.mean() > 0.05 and len(np.unique(op)) >= 6
    ll_trace = out["ll"].cpu().numpy()
    st2, out2 = make()
    np.testing.assert_array_equal(out2["ll"].cpu().numpy(), ll_trace)
    np.testing.assert_array_equal(st2.source.cpu().numpy(), src)
    np.testing.assert_array_equal(st2.zone_of_site.cpu().numpy(), zs)


def test_source_sampler_gibbsish_scratch_at_lds_boundary(gpu_available):
    """the gibbsish_sample_zones scratch (21 N bytes) counts in the placement of
    the sources.  At the largest feature count whose sources still fit LDS without it (found by
    bisection on the kernel the context reports), a run with a non-zero gibbsish weight must not
    fail: the sampler moves the sources to HBM and keeps every invariant."""
    import torch
    from scipy.spatial import Delaunay

    from contact_zones_amd.likelihood import LikelihoodEngine
    from contact_zones_amd.sampler import ChainState, Sampler, precisions
    rng = np.random.default_rng(8)
    N, S, Z, Fam, B = 240, 3, 2, 2, 4
    indptr, indices = Delaunay(rng.random((N, 2))).vertex_neighbor_vertices
    fam = rng.integers(0, Fam, size=N).astype(np.uint8)
    fam[rng.random(N) < 0.3] = 255
    prec = precisions({"weights": 15, "universal": 40, "contact": 20, "inheritance": 20})
    base_ops = {"shrink_zone": 0.1, "grow_zone": 0.1, "swap_zone": 0.05, "gibbs_sample_weights": 0.25,
                "gibbs_sample_p_global": 0.1, "gibbs_sample_p_zones": 0.25, "gibbs_sample_p_families": 0.15}

    def run(F, gib_weight, steps=1, seed=3):
        r = np.random.default_rng(F)
        obs = r.integers(0, S, size=(N, F)).astype(np.int8)
        eng = LikelihoodEngine(obs, fam, S, Z, Fam, True)
        ops = dict(base_ops, gibbsish_sample_zones=gib_weight)
        smp = Sampler(eng, np.ones((F, S), bool), indptr, indices, ops, prec, 3, sample_source=True)
        zos = np.full((B, N), 255, np.uint8)
        for b in range(B):
            p = r.permutation(N)
            zos[b, p[:8]], zos[b, p[8:16]] = 0, 1
        st = ChainState(eng, zos, r.dirichlet(np.ones(3), size=(B, F)), r.dirichlet(np.ones(S), size=(B, F)),
                        r.dirichlet(np.ones(S), size=(B, Z, F)), r.dirichlet(np.ones(S), size=(B, Fam, F)),
                        source=np.zeros((B, N, F), np.uint8))
        out = smp.run(st, steps, np.full(B, 50), np.full(B, 0.85), seed=seed)
        torch.cuda.synchronize()
        return eng, st, out

    lo, hi = 20, 400  # sources in LDS at lo, in HBM at hi (without the gibbsish scratch)
    assert "<lds>" in run(lo, 0.0)[0].last_kernels() and "<hbm" in run(hi, 0.0)[0].last_kernels()
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if "<lds>" in run(mid, 0.0)[0].last_kernels():
            lo = mid
        else:
            hi = mid
    eng, st, out = run(lo, 0.3, steps=200)
    assert out["status"].cpu().numpy().tolist() == [0] * B
    assert "<hbm" in eng.last_kernels()
    s = st.to_numpy()
    assert not np.any((s["source"] == 1) & (s["zone_of_site"] == 255)[:, :, None])
    assert not np.any((s["source"] == 2) & (fam == 255)[None, :, None])
    fresh = st.refresh_ll().cpu().numpy()
    assert np.max(np.abs(s["ll"] - fresh) / np.abs(fresh)) <= REL_TOL
