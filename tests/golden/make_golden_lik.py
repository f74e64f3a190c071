#!/usr/bin/env python3
"""Capture likelihood golden vectors from the reference sBayes — BUILD CONTAINER ONLY.

Writes tests/golden/lik_<case>.npz.  Every expected value is produced by the
reference itself: ``sbayes.model.Likelihood(data, inheritance)(Sample(...), caching=False)``
(sbayes/model.py:145-171), for the mixture branch (source=None) and the source
branch, on packed inputs that the tests feed to the oracle and the HIP path.

Cases follow BASELINE.json's configs:
  kat            test/test_model.py:52-92 known-answer setup (seeded), incl. the direct formula
  cfg1_sim       sim_exp1 simulated by the reference (sbayes/simulation.py), 951 x 35 x 4, Z=1
  cfg2           synthetic 200 x 100 x 5, Z=2, no families, 2 % NA
  cfg3_balkan    experiments/balkan real data, 28 x 47 x 3, Fam=5, Z=3
  cfg4_sa_z{1,6} experiments/south_america real data, 100 x 36 x 5, Fam=6, 92 NA cells
  cfg5_slice     synthetic 400 x 120 x 10, Z=8, Fam=4 (a reduced slice of the roofline shape)
  cfg5_full      synthetic 2000 x 500 x 10, Z=8, Fam=4 (one chain, full roofline shape)
  edge_*         Z=0, all sites zoned, all-NA feature, S=2, tiny/huge probabilities,
                 a zero selected source weight (-inf), single site,
                 a zero selected weight beside 0/0 normalised weights (-inf, not NaN)

Usage: python tests/golden/make_golden_lik.py   (from the repo root)
"""
import os
import sys
from collections import namedtuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import refenv  # noqa: E402

refenv.setup()

from sbayes.model import Likelihood  # noqa: E402
from sbayes.sampling.zone_sampling import Sample  # noqa: E402

from contact_zones_amd import packing  # noqa: E402

RefData = namedtuple("Data", ["features", "families"])


def ref_loglik(features, families, zones, w, pg, pz, pf, source, inheritance):
    data = RefData(features=features, families=families)
    lik = Likelihood(data=data, inheritance=inheritance)
    sample = Sample(zones=zones, weights=w, p_global=pg[None], p_zones=pz,
                    p_families=pf if inheritance else None, source=source)
    return lik(sample, caching=False)


def random_states_mask(rng, F, S, min_states=2):
    n = rng.integers(min_states, S + 1, size=F)
    mask = np.zeros((F, S), dtype=bool)
    for f in range(F):
        mask[f, :n[f]] = True
    return mask


def random_obs(rng, N, F, states, na_frac):
    n_states = states.sum(axis=1)
    obs = (rng.random((N, F)) * n_states[None, :]).astype(np.int8)
    obs[rng.random((N, F)) < na_frac] = -1
    return obs


def dirichlet_on_mask(rng, shape_prefix, states, alpha=1.0):
    F, S = states.shape
    out = np.zeros(shape_prefix + (F, S))
    g = rng.gamma(alpha, size=shape_prefix + (F, S)) * states
    out[...] = g / g.sum(axis=-1, keepdims=True)
    return out


def random_zones(rng, N, Z, size):
    perm = rng.permutation(N)
    zos = np.full(N, 255, dtype=np.uint8)
    for z in range(Z):
        zos[perm[z * size:(z + 1) * size]] = z
    return zos


def random_source(rng, zone_of_site, fam_of_site, F, C):
    """One allowed component per cell (global always; zone/family only where present)."""
    N = zone_of_site.shape[0]
    src = np.zeros((N, F), dtype=np.uint8)
    allow_z = (zone_of_site != 255)[:, None]
    allow_f = (fam_of_site != 255)[:, None] & (C == 3)
    r = rng.random((N, F))
    src[(r > 0.5) & allow_z] = 1
    src[(r < 0.25) & allow_f] = 2
    return src


def make_case(name, rng, obs, fam_of_site, states, Z, inheritance, B, zone_size,
              tweak=None, fixed_zones=None):
    N, F = obs.shape
    S = states.shape[1]
    Fam = int(fam_of_site[fam_of_site != 255].max()) + 1 if np.any(fam_of_site != 255) else 0
    C = 3 if inheritance else 2
    zos = np.stack([fixed_zones if fixed_zones is not None else random_zones(rng, N, Z, zone_size)
                    for _ in range(B)])
    w = rng.dirichlet(np.ones(C), size=(B, F))
    pg = dirichlet_on_mask(rng, (B,), states)
    pz = dirichlet_on_mask(rng, (B, Z), states)
    pf = dirichlet_on_mask(rng, (B, max(Fam, 1)), states)[:, :Fam] if inheritance else None
    src = np.stack([random_source(rng, zos[b], fam_of_site, F, C) for b in range(B)])
    if tweak is not None:
        tweak(locals())
    feats = packing.obs_to_features(obs, S)
    fams = packing.index_to_groups(fam_of_site, Fam) if Fam > 0 else np.zeros((0, N), bool)
    ll_mix = np.empty(B)
    ll_src = np.empty(B)
    for b in range(B):
        zones = packing.index_to_groups(zos[b], Z)
        pfb = pf[b] if inheritance else None
        ll_mix[b] = ref_loglik(feats, fams, zones, w[b].copy(), pg[b].copy(), pz[b].copy(),
                               pfb, None, inheritance)
        ll_src[b] = ref_loglik(feats, fams, zones, w[b].copy(), pg[b].copy(), pz[b].copy(),
                               pfb, packing.index_to_source(src[b], C), inheritance)
    out = dict(obs=obs, fam_of_site=fam_of_site, zone_of_site=zos, w=w, p_global=pg, p_zones=pz,
               source=src, states=states, inheritance=np.bool_(inheritance),
               ll_mixture=ll_mix, ll_source=ll_src)
    if inheritance:
        out["p_fam"] = pf
    np.savez_compressed(os.path.join(HERE, f"lik_{name}.npz"), **out)
    print(f"{name:14s} N={N} F={F} S={S} Z={Z} Fam={Fam} B={B}  ll_mix[0]={ll_mix[0]:.12g} "
          f"ll_src[0]={ll_src[0]:.12g}")


def case_kat():
    """test/test_model.py:52-92, seeded; stored in the same packed form plus lh_direct."""
    rng = np.random.default_rng(1001)
    N, F, S = 10, 5, 3
    p = rng.dirichlet(np.ones(S))
    x = rng.choice(S, size=(N, F), p=p).astype(np.int8)
    areas = np.array([[1, 1, 1, 1, 0, 0, 0, 0, 0, 0]], dtype=bool)
    feats = packing.obs_to_features(x, S)
    p_global = rng.dirichlet(np.ones(S), size=(1, F))
    p_areas = rng.dirichlet(np.ones(S), size=(1, F))
    w3 = np.repeat([[0.4, 0.3, 0.3]], F, axis=0)
    w2 = np.repeat([[0.4, 0.6]], F, axis=0)
    lh_fam = ref_loglik(feats, areas.copy(), areas, w3, p_global[0], p_areas, p_areas.copy(), None, True)
    lh_nofam = ref_loglik(feats, areas.copy(), areas, w2, p_global[0], p_areas, None, None, False)
    p_mixed = 0.4 * p_global + 0.6 * p_areas
    p_per = np.repeat(p_global, N, axis=0)
    p_per[areas[0]] = np.repeat(p_mixed, np.count_nonzero(areas), axis=0)
    lh_direct = np.sum(np.log(p_per[feats]))
    np.savez_compressed(os.path.join(HERE, "lik_kat.npz"), obs=x,
                        fam_of_site=packing.families_to_fam_of_site(areas, N),
                        zone_of_site=packing.zones_to_zone_of_site(areas, N)[None],
                        w3=w3[None], w2=w2[None], p_global=p_global, p_zones=p_areas[None],
                        p_fam=p_areas[None], lh_with_family=lh_fam, lh_without_family=lh_nofam,
                        lh_direct=lh_direct)
    print(f"kat            lh_fam={lh_fam:.15g} lh_nofam={lh_nofam:.15g} direct={lh_direct:.15g}")


def case_cfg1_sim():
    """sim_exp1 simulated by the reference with the test harness overrides (test_sbayes_experiment.py:19-36)."""
    from sbayes.experiment_setup import Experiment
    from sbayes.simulation import Simulation
    exp_dir = refenv.scratch_copy("experiments/simulation/sim_exp1")
    np.random.seed(1)
    import random
    random.seed(1)
    exp = Experiment(experiment_name="golden", config_file=os.path.join(exp_dir, "config.json"), log=False)
    exp.load_config(os.path.join(exp_dir, "config.json"), custom_settings={
        "simulation": {"I_CONTACT": 3, "E_CONTACT": 0.5, "STRENGTH": 1, "AREA": 4}})
    sim = Simulation(experiment=exp)
    sim.run_simulation()
    obs = packing.features_to_obs(sim.features)
    states = np.asarray(sim.states, dtype=bool)
    N = obs.shape[0]
    fam = np.full(N, 255, np.uint8)
    true_zone = packing.zones_to_zone_of_site(sim.areas, N)
    rng = np.random.default_rng(11)
    make_case("cfg1_sim", rng, obs, fam, states, Z=1, inheritance=False, B=3, zone_size=0,
              fixed_zones=true_zone)
    np.savez_compressed(os.path.join(HERE, "data_cfg1_sim.npz"), obs=obs, states=states,
                        true_zone=true_zone, locations=sim.network["locations"],
                        adj_indptr=sim.network["adj_mat"].indptr,
                        adj_indices=sim.network["adj_mat"].indices)


def load_real(rel_features, rel_states):
    from sbayes.util import read_features_from_csv
    out = read_features_from_csv(os.path.join(refenv.REFERENCE, rel_features),
                                 os.path.join(refenv.REFERENCE, rel_states))
    sites, _, features, _, _, states, families, _, _ = out
    N = features.shape[0]
    obs = packing.features_to_obs(features)
    fam = packing.families_to_fam_of_site(families, N)
    return obs, fam, np.asarray(states, bool), sites


def case_real():
    obs, fam, states, sites = load_real("experiments/balkan/data/features/features.csv",
                                        "experiments/balkan/data/features/feature_states.csv")
    make_case("cfg3_balkan", np.random.default_rng(3), obs, fam, states, Z=3, inheritance=True,
              B=4, zone_size=4)
    make_case("cfg3_balkan_noinh", np.random.default_rng(31), obs, fam, states, Z=3,
              inheritance=False, B=2, zone_size=4)
    np.savez_compressed(os.path.join(HERE, "data_cfg3_balkan.npz"), obs=obs, fam_of_site=fam,
                        states=states, locations=sites["locations"])
    obs, fam, states, sites = load_real("experiments/south_america/data/features/features.csv",
                                        "experiments/south_america/data/features/feature_states.csv")
    for z in (1, 6):
        make_case(f"cfg4_sa_z{z}", np.random.default_rng(40 + z), obs, fam, states, Z=z,
                  inheritance=True, B=3, zone_size=6)
    np.savez_compressed(os.path.join(HERE, "data_cfg4_sa.npz"), obs=obs, fam_of_site=fam,
                        states=states, locations=sites["locations"])


def synth_fam(rng, N, Fam, frac_in_family=0.8):
    fam = rng.integers(0, Fam, size=N).astype(np.uint8) if Fam > 0 else np.full(N, 255, np.uint8)
    if Fam > 0:
        fam[rng.random(N) > frac_in_family] = 255
    return fam


def case_synth():
    rng = np.random.default_rng(2)
    N, F, S = 200, 100, 5
    states = random_states_mask(rng, F, S)
    make_case("cfg2", rng, random_obs(rng, N, F, states, 0.02), np.full(N, 255, np.uint8), states,
              Z=2, inheritance=False, B=4, zone_size=N // 8)

    rng = np.random.default_rng(5)
    N, F, S = 400, 120, 10
    states = random_states_mask(rng, F, S)
    make_case("cfg5_slice", rng, random_obs(rng, N, F, states, 0.02), synth_fam(rng, N, 4), states,
              Z=8, inheritance=True, B=3, zone_size=N // 32)

    rng = np.random.default_rng(55)
    N, F, S = 2000, 500, 10
    states = random_states_mask(rng, F, S)
    make_case("cfg5_full", rng, random_obs(rng, N, F, states, 0.02), synth_fam(rng, N, 4), states,
              Z=8, inheritance=True, B=1, zone_size=N // 32)


def case_edges():
    # no zones at all
    rng = np.random.default_rng(70)
    N, F, S = 50, 30, 4
    states = random_states_mask(rng, F, S)
    make_case("edge_z0", rng, random_obs(rng, N, F, states, 0.05), synth_fam(rng, N, 2), states,
              Z=0, inheritance=True, B=2, zone_size=0)
    # every site in a zone
    rng = np.random.default_rng(71)
    make_case("edge_allzoned", rng, random_obs(rng, N, F, states, 0.05), synth_fam(rng, N, 3),
              states, Z=5, inheritance=True, B=2, zone_size=N // 5)
    # an all-NA feature and an all-NA site; binary states
    rng = np.random.default_rng(72)
    N, F, S = 37, 19, 2
    states = np.ones((F, S), bool)
    obs = random_obs(rng, N, F, states, 0.1)
    obs[:, 3] = -1
    obs[5, :] = -1
    make_case("edge_na", rng, obs, synth_fam(rng, N, 2), states, Z=2, inheritance=True, B=2,
              zone_size=6)
    # single site
    rng = np.random.default_rng(73)
    states = random_states_mask(rng, 7, 3)
    make_case("edge_onesite", rng, random_obs(rng, 1, 7, states, 0.0), np.zeros(1, np.uint8),
              states, Z=1, inheritance=True, B=2, zone_size=1)

    # tiny and huge magnitudes (exercise the HIP product path's guarded fallback)
    def tiny(loc):
        loc["pg"][0, :, :] = np.where(loc["states"], 1e-200, 0.0)
        loc["pz"][1, 0, 2, :] = np.where(loc["states"][2], 1e-300, 0.0)
    rng = np.random.default_rng(74)
    N, F, S = 64, 20, 3
    states = random_states_mask(rng, F, S)
    make_case("edge_tiny", rng, random_obs(rng, N, F, states, 0.0), synth_fam(rng, N, 2), states,
              Z=2, inheritance=True, B=2, zone_size=10, tweak=tiny)

    # a zero weight on a selected source component -> -inf in source mode; zero lh -> -inf mixture
    def zero_w(loc):
        loc["w"][0, 3, 1] = 0.0
        z0 = np.nonzero(loc["zos"][0] != 255)[0][0]
        loc["src"][0, z0, 3] = 1
        loc["pg"][1, 4, :] = 0.0
    rng = np.random.default_rng(75)
    make_case("edge_zero", rng, random_obs(rng, N, F, states, 0.0), synth_fam(rng, N, 2), states,
              Z=2, inheritance=True, B=2, zone_size=10, tweak=zero_w)


def case_zero_nan():
    """model.py:181-182 tests `any(observation_weights == 0)` before taking logs: a selected
    weight of exactly 0 gives -inf even when other selected weights are NaN (0 / 0 normalised
    weights at sites with none of the feature's non-zero components).  Chain 0: feature 3 has
    weights [0, 1, 0], so the no-zone sites' weights are 0 / 0 and a zoned site selecting the
    global component has weight 0 -> -inf.  Chain 1: the same NaN cells, no zero selected
    weight (every zoned site selects its zone at feature 3) -> NaN."""
    def zero_nan(loc):
        for b in (0, 1):
            loc["w"][b, 3] = [0.0, 1.0, 0.0]
            zoned = loc["zos"][b] != 255
            loc["src"][b, zoned, 3] = 1
        z0 = np.nonzero(loc["zos"][0] != 255)[0][0]
        loc["src"][0, z0, 3] = 0
    rng = np.random.default_rng(76)
    N, F, S = 64, 20, 3
    states = random_states_mask(rng, F, S)
    make_case("edge_zero_nan", rng, random_obs(rng, N, F, states, 0.0), synth_fam(rng, N, 2), states,
              Z=2, inheritance=True, B=2, zone_size=10, tweak=zero_nan)


if __name__ == "__main__":
    if sys.argv[1:] == ["zero_nan"]:
        case_zero_nan()
        sys.exit(0)
    case_kat()
    case_synth()
    case_real()
    case_edges()
    case_zero_nan()
    case_cfg1_sim()
