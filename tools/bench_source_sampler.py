"""Source-mode (SAMPLE_SOURCE = true, the reference default) sampler throughput on synthetic data:
B chains x K Philox MH steps with the default operator table, steps/s, us per step and ESS/s of
the log-likelihood traces.  Prints one JSON line.

  python tools/bench_source_sampler.py --sites 100 --features 36 --states 5 --zones 6 --families 6 --chains 128
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# config/default_config.json STEPS with SAMPLE_SOURCE = true (source 0.0: zone moves resample the
# sources themselves), mcmc_setup.py:70-95
STEPS = {"area": 0.05, "weights": 0.4, "universal": 0.05, "contact": 0.4, "inheritance": 0.1, "source": 0.0}


def operators(inh):
    a = dict(STEPS)
    if not inh:
        a["inheritance"] = 0.0
    ops = {"shrink_zone": a["area"] * 0.4, "grow_zone": a["area"] * 0.4, "swap_zone": a["area"] * 0.2,
           "gibbsish_sample_zones": 0.0, "gibbs_sample_sources": a["source"],
           "gibbs_sample_weights": a["weights"], "gibbs_sample_p_global": a["universal"],
           "gibbs_sample_p_zones": a["contact"], "gibbs_sample_p_families": a["inheritance"]}
    tot = sum(ops.values())
    return {k: v / tot for k, v in ops.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--sites", type=int, default=100)
    p.add_argument("--features", type=int, default=36)
    p.add_argument("--states", type=int, default=5)
    p.add_argument("--zones", type=int, default=6)
    p.add_argument("--families", type=int, default=6)
    p.add_argument("--chains", type=int, default=128)
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--burnin", type=int, default=2000)
    p.add_argument("--seed", type=int, default=3)
    a = p.parse_args()
    import torch
    from scipy.spatial import Delaunay

    from contact_zones_amd import packing
    from contact_zones_amd.diagnostics import ess
    from contact_zones_amd.likelihood import LikelihoodEngine
    from contact_zones_amd.mcmc import InitialSamples
    from contact_zones_amd.sampler import ChainState, Sampler, precisions
    from contact_zones_amd.sources import draw_sources, source_posterior
    N, F, S, Z, Fam, B = a.sites, a.features, a.states, a.zones, a.families, a.chains
    inh = Fam > 0
    rng = np.random.default_rng(a.seed)
    obs = rng.integers(0, S, size=(N, F)).astype(np.int8)
    obs[rng.random((N, F)) < 0.02] = -1
    fam = rng.integers(0, max(Fam, 1), size=N).astype(np.uint8)
    fam[rng.random(N) < 0.2] = 255
    if not inh:
        fam[:] = 255
    indptr, indices = Delaunay(rng.random((N, 2))).vertex_neighbor_vertices
    states = np.ones((F, S), bool)
    eng = LikelihoodEngine(obs, fam, S, Z, Fam, inh)
    init = InitialSamples(packing.obs_to_features(obs, S), states, indptr, indices,
                          packing.index_to_groups(fam, Fam) if inh else np.zeros((0, N), bool), Z, 5, inh,
                          None, random.Random(a.seed))
    pg0, w0 = init.p_global()[0], init.weights()
    pf0 = init.p_families() if inh else None
    zos = np.empty((B, N), np.uint8)
    pz = np.empty((B, Z, F, S))
    src = np.empty((B, N, F), np.uint8)
    np.random.seed(a.seed)
    for b in range(B):
        zones = init.zones()
        zos[b] = packing.zones_to_zone_of_site(zones, N)
        pz[b] = init.p_zones(zones)
        post = source_posterior(obs, fam, zos[b], w0, pg0, pz[b], pf0, inh)
        src[b] = draw_sources(post)
    rep = lambda x: np.broadcast_to(x, (B,) + x.shape).copy()  # noqa: E731
    st = ChainState(eng, zos, rep(w0), rep(pg0), pz, rep(pf0) if inh else None, source=src)
    smp = Sampler(eng, states, indptr, indices, operators(inh),
                  precisions({"weights": 15, "universal": 40, "contact": 20, "inheritance": 20}), 3,
                  sample_source=True)
    if a.burnin:
        smp.run(st, a.burnin, 50, 0.85, seed=a.seed * 7919)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = smp.run(st, a.steps, 50, 0.85, seed=a.seed * 7919, trace=True)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    status = out["status"].cpu().numpy()
    ll = out["ll"].cpu().numpy()
    e = ess(ll)
    print(json.dumps({"shape": f"{N}x{F}x{S} Z{Z} Fam{Fam}", "chains": B, "steps": a.steps,
                      "lds_or_hbm": "hbm" if os.environ.get("SBZ_SRC_HBM") == "1" or
                      2 * N * F > 150 * 1024 else "lds",
                      "mh_steps_per_sec": B * a.steps / wall, "us_per_step": wall / a.steps * 1e6,
                      "ess_per_sec": float(e.sum()) / wall, "acceptance": float(out["accept"].float().mean()),
                      "status_ok": bool(np.all(status == 0))}))


if __name__ == "__main__":
    main()
