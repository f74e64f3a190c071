"""GPU parity of the MH sampler: replaying the reference's decision tapes
(tests/golden/make_golden_mh.py, seeded ZoneMCMC / ZoneMCMCWarmup) reproduces every step's
operator, accept flag and zone assignment bit for bit; log-likelihoods (updated incrementally on
the GPU) stay within the north_star tolerance of 1e-9 relative of the reference's full values."""
import numpy as np
import pytest

from conftest import prior_spec, golden_cases, load_golden, mh_cases

pytestmark = pytest.mark.gpu

MH_CASES = mh_cases(source=False)  # source mode: test_gpu_source.py
REL_TOL = 1e-9


def _setup(fx, options=None):
    from contact_zones_amd.likelihood import LikelihoodEngine
    from contact_zones_amd.sampler import ChainState, Sampler
    inh = bool(fx["inheritance"])
    S = fx["states"].shape[1]
    Z = int(fx["n_zones"])
    Fam = fx["init_p_fam"].shape[1] if inh else 0
    eng = LikelihoodEngine(fx["obs"], fx["fam_of_site"], S, Z, Fam, inh, options=options)
    from contact_zones_amd.priors import PriorSpec
    priors = prior_spec(fx)
    smp = Sampler(eng, fx["states"], fx["adj_indptr"], fx["adj_indices"], fx["op_probs"],
                  fx["precision"], int(fx["min_size"]), warmup=bool(fx["warmup"]), priors=priors)
    st = ChainState(eng, fx["init_zone_of_site"], fx["init_w"], fx["init_p_global"],
                    fx["init_p_zones"], fx["init_p_fam"] if inh else None, prior=fx["init_prior"])
    return eng, smp, st


@pytest.mark.parametrize("case", MH_CASES)
def test_tape_replay_matches_reference(gpu_available, case):
    import torch
    fx = load_golden(case)
    eng, smp, st = _setup(fx)
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
    # the carried log prior (prior += proposal difference) ends at the reference's value
    np.testing.assert_allclose(st.prior.cpu().numpy(), fx["step_prior"][:, -1], rtol=1e-12, atol=1e-12)
    # the incrementally tracked ll equals a fresh full evaluation of the final state
    final = st.ll.cpu().numpy().copy()
    fresh = st.refresh_ll().cpu().numpy()
    assert np.max(np.abs(final - fresh) / np.abs(fresh)) <= REL_TOL
    # accept/propose statistics agree with the trace
    acc = st.accepted.cpu().numpy()
    prop = st.proposed.cpu().numpy()
    for b in range(st.B):
        ops = fx["step_op"][b]
        np.testing.assert_array_equal(prop[b, :8], np.bincount(ops, minlength=8)[:8])
        np.testing.assert_array_equal(acc[b, :8], np.bincount(ops[fx["step_accept"][b]], minlength=8)[:8])


@pytest.mark.parametrize("case", MH_CASES[:2])
def test_tape_replay_in_chunks(gpu_available, case):
    """Splitting the run into several launches (the cursor and LDS state carried in HBM) gives
    the same trajectory."""
    import torch
    fx = load_golden(case)
    eng, smp, st = _setup(fx)
    n = fx["step_op"].shape[1]
    pos = torch.zeros(st.B, dtype=torch.int64, device=st.ll.device)
    ops = []
    for a, b in [(0, 7), (7, 100), (100, n)]:
        out = smp.run(st, b - a, fx["max_size"], fx["p_grow_connected"], tape=fx["tape"],
                      tape_len=fx["tape_len"], tape_pos=pos, trace=True)
        ops.append(out["op"].cpu().numpy())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(np.concatenate(ops, axis=1), fx["step_op"])
    np.testing.assert_array_equal(st.zone_of_site.cpu().numpy(), fx["step_zone_of_site"][:, -1])


def test_philox_chains_are_valid_and_reproducible(gpu_available):
    """Philox mode: zone sizes stay within [MIN_M, max_size], zones stay disjoint, parameters
    stay normalised, ll matches a fresh evaluation, and a re-run with the same seed and chain
    ids is bit-identical (independent of batch composition)."""
    import torch
    fx = load_golden("mh_cfg1_sim_inh_z2")
    eng, smp, st = _setup(fx)
    out = smp.run(st, 2000, 20, 0.85, seed=1234, chain_id0=7)
    torch.cuda.synchronize()
    s = st.to_numpy()
    Z = int(fx["n_zones"])
    for b in range(st.B):
        sizes = np.bincount(s["zone_of_site"][b][s["zone_of_site"][b] < 255], minlength=Z)
        assert np.all(sizes >= int(fx["min_size"])) and np.all(sizes <= 20)
    np.testing.assert_allclose(s["w"].sum(-1), 1.0, rtol=1e-12)
    np.testing.assert_allclose(s["p_global"].sum(-1), 1.0, rtol=1e-12)
    np.testing.assert_allclose(s["p_zones"].sum(-1), 1.0, rtol=1e-12)
    fresh = st.refresh_ll().cpu().numpy()
    assert np.max(np.abs(s["ll"] - fresh) / np.abs(fresh)) <= REL_TOL
    assert st.accepted.sum().item() > 100
    # reproducible: the second chain alone, with its global id, gives the same state
    eng2, smp2, st2 = _setup(fx)
    st2_one = type(st2)(eng2, fx["init_zone_of_site"][1:2], fx["init_w"][1:2], fx["init_p_global"][1:2],
                        fx["init_p_zones"][1:2], fx["init_p_fam"][1:2])
    smp2.run(st2_one, 2000, 20, 0.85, seed=1234, chain_id0=8)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(st2_one.zone_of_site.cpu().numpy()[0], s["zone_of_site"][1])
    np.testing.assert_array_equal(st2_one.w.cpu().numpy()[0], s["w"][1])


def test_philox_carried_prior_matches_full_prior(gpu_available):
    """'counts' + zone-size priors under Philox draws: after 3000 steps the prior the kernel
    carries (prior += proposal difference) equals the full Prior of the final states."""
    import torch
    from contact_zones_amd.priors import PriorSpec
    fx = load_golden("mh_small_priors")
    eng, smp, st = _setup(fx)
    out = smp.run(st, 3000, fx["max_size"], fx["p_grow_connected"], seed=99)
    torch.cuda.synchronize()
    assert out["status"].cpu().numpy().tolist() == [0] * st.B
    s = st.to_numpy()
    spec = prior_spec(fx)
    full = spec.log_prior(s["zone_of_site"], s["p_global"], s["p_fam"], fx["states"],
                          int(fx["n_zones"]), True)
    np.testing.assert_allclose(s["prior"], full, rtol=1e-12)
    assert np.any(s["prior"] != fx["init_prior"])  # the prior moved


def _synthetic_chains(N, F, S, Z, Fam, inh, B, options=None):
    """A Delaunay network of random sites, random observations, reference-initialised zones
    (InitialSamples) and random parameters: sampler, chain state and likelihood engine."""
    import random
    from scipy.spatial import Delaunay
    from contact_zones_amd import packing
    from contact_zones_amd.likelihood import LikelihoodEngine
    from contact_zones_amd.mcmc import InitialSamples
    from contact_zones_amd.sampler import ChainState, Sampler
    rng = np.random.default_rng(N + F + S)
    obs = rng.integers(0, S, size=(N, F)).astype(np.int8)
    obs[rng.random((N, F)) < 0.03] = -1
    fam = rng.integers(0, max(Fam, 1), size=N).astype(np.uint8) if Fam else np.full(N, 255, np.uint8)
    if Fam:
        fam[rng.random(N) < 0.1] = 255
    indptr, indices = Delaunay(rng.random((N, 2))).vertex_neighbor_vertices
    order = [np.sort(indices[indptr[i]:indptr[i + 1]]) for i in range(N)]
    indices = np.concatenate(order).astype(np.int32)
    indptr = indptr.astype(np.int32)
    states = np.ones((F, S), bool)
    init = InitialSamples(packing.obs_to_features(obs, S), states, indptr, indices,
                          packing.index_to_groups(fam, Fam) if Fam else None, Z, 5, inh, None,
                          random.Random(11))
    zos = np.stack([packing.zones_to_zone_of_site(init.zones(), N) for _ in range(B)])
    w = rng.dirichlet(np.ones(3 if inh else 2), size=(B, F))
    pg = rng.dirichlet(np.ones(S), size=(B, F))
    pz = rng.dirichlet(np.ones(S), size=(B, Z, F))
    pf = rng.dirichlet(np.ones(S), size=(B, Fam, F)) if inh else None
    eng = LikelihoodEngine(obs, fam, S, Z, Fam, inh, options=options)
    ops = {"shrink_zone": 0.1, "grow_zone": 0.1, "swap_zone": 0.05, "alter_weights": 0.3,
           "alter_p_global": 0.15, "alter_p_zones": 0.2, "alter_p_families": 0.1 if inh and Fam else 0.0}
    smp = Sampler(eng, states, indptr, indices, ops, [15, 40, 20, 20], 3)
    st = ChainState(eng, zos, w, pg, pz, pf)
    return smp, st


@pytest.mark.parametrize("N,F,S,Z,Fam,inh,B,steps", [
    (3000, 40, 12, 3, 3, True, 6, 1500),    # two batches of observation chunks (Np = 4096)
    (700, 30, 40, 2, 2, True, 6, 1500),     # S + 1 > 32: observation bytes hold x, not x * 8
    (2000, 50, 10, 8, 4, True, 6, 1500),    # the bench shape's site count / zones / families
    (300, 20, 5, 2, 0, False, 6, 1500),     # no inheritance (C = 2)
    (2000, 500, 10, 8, 4, True, 256, 400),  # the bench's sampler leg: full cfg5 width, 256 chains
])
def test_philox_large_shapes_carried_ll(gpu_available, N, F, S, Z, Fam, inh, B, steps):
    """Philox runs on shapes the golden tapes do not reach: the incrementally carried ll equals a
    fresh full evaluation (likelihood kernel) within 1e-9 after every operator type ran, zones
    stay disjoint and within bounds, and parameters stay normalised."""
    import torch
    smp, st = _synthetic_chains(N, F, S, Z, Fam, inh, B)
    out = smp.run(st, steps, 40, 0.85, seed=5)
    torch.cuda.synchronize()
    assert out["status"].cpu().numpy().tolist() == [0] * B
    acc = st.accepted.cpu().numpy()
    assert np.all(acc[:, :7].sum(0)[[1, 3, 4, 5]] > 0)  # zone and parameter moves accepted
    assert np.all(st.proposed.cpu().numpy()[:, :7].sum(0)[[0, 1, 2]] > 0)  # every zone move ran
    s = st.to_numpy()
    fresh = st.refresh_ll().cpu().numpy()
    assert np.max(np.abs(s["ll"] - fresh) / np.abs(fresh)) <= REL_TOL
    for b in range(B):
        sizes = np.bincount(s["zone_of_site"][b][s["zone_of_site"][b] < 255], minlength=Z)
        assert np.all(sizes >= 3) and np.all(sizes <= 40)
    np.testing.assert_allclose(s["w"].sum(-1), 1.0, rtol=1e-12)
    np.testing.assert_allclose(s["p_zones"].sum(-1), 1.0, rtol=1e-12)


@pytest.mark.parametrize("case", ["mh_small_priors", "mh_cfg1_sim_inh_z2"])
def test_host_form_run_replays_reference(gpu_available, case):
    """sbz_mh_run (SURVEY.md §8b's host-form entry: numpy arrays in, numpy arrays out, no device
    buffers on the caller's side) replays the reference's decision tape exactly as the device
    entry does: operators, accepts, final zones and parameters, ll within 1e-9."""
    from contact_zones_amd.sampler import run_host
    fx = load_golden(case)
    eng, smp, st = _setup(fx)
    n_steps = fx["step_op"].shape[1]
    inh = bool(fx["inheritance"])
    host = {"zone_of_site": fx["init_zone_of_site"].copy(), "w": fx["init_w"].copy(),
            "p_global": fx["init_p_global"].copy(), "p_zones": fx["init_p_zones"].copy(),
            "p_fam": fx["init_p_fam"].copy() if inh else None,
            "prior": np.broadcast_to(np.asarray(fx["init_prior"], np.float64), (st.B,)).copy()}
    tr = run_host(smp, host, n_steps, fx["max_size"], fx["p_grow_connected"], tape=fx["tape"],
                  tape_len=fx["tape_len"], trace=True)
    assert host["status"].tolist() == [0] * st.B
    np.testing.assert_array_equal(host["tape_pos"], fx["tape_len"])
    np.testing.assert_array_equal(tr["op"], fx["step_op"])
    np.testing.assert_array_equal(tr["accept"].astype(bool), fx["step_accept"])
    np.testing.assert_array_equal(host["zone_of_site"], fx["step_zone_of_site"][:, -1])
    assert np.max(np.abs(tr["ll"] - fx["step_ll"]) / np.abs(fx["step_ll"])) <= REL_TOL
    # the device entry on the same inputs ends in the same state, bit for bit
    out = smp.run(st, n_steps, fx["max_size"], fx["p_grow_connected"], tape=fx["tape"],
                  tape_len=fx["tape_len"], trace=True)
    dev = st.to_numpy()
    for k in ("zone_of_site", "w", "p_global", "p_zones", "ll", "prior") + (("p_fam",) if inh else ()):
        np.testing.assert_array_equal(host[k], dev[k], err_msg=k)
    np.testing.assert_array_equal(tr["ll"], out["ll"].cpu().numpy())
    np.testing.assert_array_equal(host["proposed"], st.proposed.cpu().numpy())


def test_host_form_philox_matches_device_form(gpu_available):
    """Philox draws: host-form and device-form runs of the same chains, seed and chain ids are
    bit-identical, including the counters a continued run starts from."""
    from contact_zones_amd.sampler import run_host
    fx = load_golden("mh_small_priors")
    eng, smp, st = _setup(fx)
    inh = bool(fx["inheritance"])
    host = {k: v.copy() for k, v in st.to_numpy().items() if k != "ll"}
    for _ in range(2):
        run_host(smp, host, 300, fx["max_size"], fx["p_grow_connected"], seed=77, chain_id0=5)
        st.refresh_ll()  # sbz_mh_run starts every run from a full evaluation of the state
        out = smp.run(st, 300, fx["max_size"], fx["p_grow_connected"], seed=77, chain_id0=5)
    assert host["status"].tolist() == out["status"].cpu().numpy().tolist() == [0] * st.B
    dev = st.to_numpy()
    for k in ("zone_of_site", "w", "p_global", "p_zones", "ll", "prior") + (("p_fam",) if inh else ()):
        np.testing.assert_array_equal(host[k], dev[k], err_msg=k)
    np.testing.assert_array_equal(host["counter"], st.counter.cpu().numpy())


@pytest.mark.parametrize("case", ["mh_small_priors", "mh_cfg1_sim_inh_z2", "mh_small_bounds"])
def test_philox_planned_proposals_do_not_change_trajectories(gpu_available, case):
    """Philox mode plans the proposals of the next parameter moves in parallel lanes (option
    mh_lookahead steps at a time), computes the deltas of up to mh_group planned moves on different
    features at once (one per wave) and recomputes a plan that an accepted move made stale: the
    trajectory (operators, accepts, ll, final state, counters) is bit-identical to the
    one-step-at-a-time path (mh_lookahead = 1), over launches of different lengths."""
    import torch
    fx = load_golden(case)
    runs = []
    for la, grp in ((1, 4), (24, 4), (6, 4), (24, 1), (24, 2), (6, 3), (24, 8), (6, 8), (24, 7), (12, 5)):
        eng, smp, st = _setup(fx, {"mh_lookahead": la, "mh_group": grp})
        outs = [smp.run(st, n, fx["max_size"], fx["p_grow_connected"], seed=4242, chain_id0=3, trace=True)
                for n in (700, 5, 1301)]
        torch.cuda.synchronize()
        runs.append(([{k: v.cpu().numpy() for k, v in o.items() if hasattr(v, "cpu")} for o in outs], st.to_numpy(),
                     st.counter.cpu().numpy(), st.accepted.cpu().numpy()))
    base = runs[0]
    assert base[3][:, 3:7].sum() > 50  # parameter moves were accepted (plans went stale)
    for other in runs[1:]:
        for o1, o2 in zip(base[0], other[0]):
            for k in ("op", "accept", "ll", "status"):
                np.testing.assert_array_equal(o1[k], o2[k], err_msg=k)
        for k in base[1]:
            np.testing.assert_array_equal(base[1][k], other[1][k], err_msg=k)
        np.testing.assert_array_equal(base[2], other[2])
        np.testing.assert_array_equal(base[3], other[3])


def test_planned_batches_cut_by_lds(gpu_available):
    """Wide parameter columns (S = 60, Z = 6, Fam = 4: 663 doubles per planned step, 35 KB of cell
    tables per wave) leave room in the 160 KiB for fewer than 24 planned steps and fewer than 4
    table slots (2 here): the host cuts both, and the trajectory stays bit-identical to the
    one-step-at-a-time path."""
    import torch
    runs = []
    for la in (1, 24):
        smp, st = _synthetic_chains(300, 30, 60, 6, 4, True, 8, {"mh_lookahead": la})
        out = smp.run(st, 600, 40, 0.85, seed=9, trace=True)
        torch.cuda.synchronize()
        runs.append(({k: out[k].cpu().numpy() for k in ("op", "accept", "ll", "status")}, st.to_numpy()))
    assert runs[0][0]["status"].tolist() == [0] * 8
    assert runs[0][0]["accept"][:, :].sum() > 50
    for k in runs[0][0]:
        np.testing.assert_array_equal(runs[0][0][k], runs[1][0][k], err_msg=k)
    for k in runs[0][1]:
        np.testing.assert_array_equal(runs[0][1][k], runs[1][1][k], err_msg=k)


@pytest.mark.parametrize("alpha", [0.3, 1.0, 1.7, 4.0, 31.0, 250.0])
def test_gamma_generator_distribution(gpu_available, alpha):
    """The samplers' gamma generator (LaneRng::gamma: Marsaglia-Tsang, two Box-Muller candidates
    per round; the Dirichlet draws of the Philox-mode operators) against Gamma(alpha, 1):
    Kolmogorov-Smirnov on 2^17 draws, and the first two moments."""
    import ctypes
    from scipy import stats
    from contact_zones_amd.likelihood import LikelihoodEngine
    eng = LikelihoodEngine(np.zeros((4, 3), np.int8), np.full(4, 255, np.uint8), 2, 1, 0, False)
    n = 1 << 17
    a = np.full(n, alpha)
    out = np.empty(n)
    rc = eng._lib.sbz_draw_gamma(eng.ctx, n, a.ctypes.data_as(ctypes.c_void_p), 12345 + int(alpha * 10),
                                 out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    assert np.all(np.isfinite(out)) and np.all(out > 0)
    ks = stats.kstest(out, stats.gamma(alpha).cdf)
    assert ks.pvalue > 1e-4, ks
    se = np.sqrt(alpha / n)  # standard error of the mean
    assert abs(out.mean() - alpha) < 6 * se
    assert abs(out.var() / alpha - 1.0) < 0.05
    # reproducible: same seed, same draws
    out2 = np.empty(n)
    eng._lib.sbz_draw_gamma(eng.ctx, n, a.ctypes.data_as(ctypes.c_void_p), 12345 + int(alpha * 10),
                            out2.ctypes.data_as(ctypes.c_void_p))
    np.testing.assert_array_equal(out, out2)


@pytest.mark.parametrize("case", ["mh_gibbsish_small", "mh_gibbsish_sim", "mh_small_geo", "mh_small_priors"])
def test_philox_gibbsish_invariants(gpu_available, case):
    """gibbsish_sample_zones (zone_sampling.py:619-702) under Philox draws, its weight set to the
    zone moves' total, with the fixture's priors ('counts' and uniform zone size; the geo prior's
    last-zone MST): zones stay disjoint and within [MIN_M, max_size], the tracked ll equals a fresh
    evaluation, the carried prior the full prior, and the trajectory does not depend on the
    planning depth of the parameter moves around it."""
    import torch
    fx = dict(load_golden(case))
    probs = fx["op_probs"].copy()
    probs[7] = probs[:3].sum()
    fx["op_probs"] = probs
    runs = []
    for la in (1, 24):
        eng, smp, st = _setup(fx, {"mh_lookahead": la})
        out = smp.run(st, 1500, fx["max_size"], fx["p_grow_connected"], seed=515, chain_id0=2, trace=True)
        torch.cuda.synchronize()
        assert out["status"].cpu().numpy().tolist() == [0] * st.B
        s = st.to_numpy()
        runs.append((out["op"].cpu().numpy(), out["accept"].cpu().numpy(), out["ll"].cpu().numpy(), s))
        Z = int(fx["n_zones"])
        for b in range(st.B):
            sizes = np.bincount(s["zone_of_site"][b][s["zone_of_site"][b] < 255], minlength=Z)
            assert np.all(sizes >= int(fx["min_size"])) and np.all(sizes <= fx["max_size"][b])
        fresh = st.refresh_ll().cpu().numpy()
        assert np.max(np.abs(s["ll"] - fresh) / np.abs(fresh)) <= REL_TOL
        full = prior_spec(fx).log_prior(s["zone_of_site"], s["p_global"], s.get("p_fam"), fx["states"],
                                        Z, bool(fx["inheritance"]))
        np.testing.assert_allclose(s["prior"], full, rtol=1e-12, atol=1e-12)
        gib = runs[-1][0] == 7
        assert gib.sum() > 100
        if case.startswith("mh_gibbsish"):
            assert (gib & (runs[-1][1] != 0)).sum() > 10  # accepted gibbsish moves
    for a, b in zip(runs[0][:3], runs[1][:3]):
        np.testing.assert_array_equal(a, b)
