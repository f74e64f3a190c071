"""Per-operator sampler timing at the bench's cfg5 shape: 256 chains x K steps with one operator
family at a time (Philox draws), device time per step.  Diagnostic only (not part of the bench).

Usage (GPU box): python tools/mh_optime.py [--steps K] [--chains B]
"""
import argparse
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from contact_zones_amd import packing  # noqa: E402
from contact_zones_amd.likelihood import LikelihoodEngine  # noqa: E402
from contact_zones_amd.mcmc import InitialSamples  # noqa: E402
from contact_zones_amd.sampler import ChainState, Sampler, precisions  # noqa: E402

SETS = {
    "default": bench.mh_operators(),
    "weights": {"alter_weights": 1.0},
    "p_global": {"alter_p_global": 1.0},
    "p_zones": {"alter_p_zones": 1.0},
    "p_families": {"alter_p_families": 1.0},
    "zone_moves": {"shrink_zone": 0.4, "grow_zone": 0.4, "swap_zone": 0.2},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--chains", type=int, default=256)
    ap.add_argument("--sites", type=int, default=2000)
    ap.add_argument("--features", type=int, default=500)
    ap.add_argument("--states", type=int, default=10)
    ap.add_argument("--zones", type=int, default=8)
    ap.add_argument("--families", type=int, default=4)
    ap.add_argument("--stamps", action="store_true",
                    help="library built with SBZ_MH_STAMP: report mean phase cycles per operator")
    ap.add_argument("--sets", default=",".join(SETS), help="comma-separated operator sets")
    ap.add_argument("--options", default="{}", help="JSON context options, e.g. {\"mh_group\": 1}")
    a = ap.parse_args()
    N, F, S, Z, Fam, B = a.sites, a.features, a.states, a.zones, a.families, a.chains
    rng = np.random.default_rng(5)
    obs = rng.integers(0, S, size=(N, F)).astype(np.int8)
    obs[rng.random((N, F)) < 0.02] = -1
    fam = rng.integers(0, Fam, size=N).astype(np.uint8)
    eng = LikelihoodEngine(obs, fam, S, Z, Fam, True, device=0, options=json.loads(a.options) or None)
    indptr, indices = bench.make_network(N, np.random.default_rng(22))
    states = np.ones((F, S), bool)
    init = InitialSamples(packing.obs_to_features(obs, S), states, indptr, indices,
                          packing.index_to_groups(fam, Fam), Z, bench.MH_M_INITIAL, True, None,
                          random.Random(3))
    pg0, pf0, w0 = init.p_global()[0], init.p_families(), init.weights()
    zos = np.empty((B, N), np.uint8)
    pz = np.empty((B, Z, F, S))
    for b in range(B):
        zones = init.zones()
        zos[b] = packing.zones_to_zone_of_site(zones, N)
        pz[b] = init.p_zones(zones)
    rep = lambda x: np.broadcast_to(x, (B,) + x.shape).copy()  # noqa: E731
    res = {}
    for name in a.sets.split(","):
        ops = SETS[name]
        st = ChainState(eng, zos, rep(w0), rep(pg0), pz, rep(pf0))
        smp = Sampler(eng, states, indptr, indices, ops, precisions(bench.MH_PRECISION), bench.MH_MIN_M)
        smp.run(st, 200, bench.MH_MAX_M, bench.MH_P_GROW, seed=1)  # warm
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = smp.run(st, a.steps, bench.MH_MAX_M, bench.MH_P_GROW, seed=2, trace=a.stamps)
        e1.record()
        torch.cuda.synchronize()
        if out["status"].cpu().numpy().any():
            raise SystemExit(f"{name}: status {np.unique(out['status'].cpu().numpy())}")
        us = e0.elapsed_time(e1) * 1e3 / a.steps
        ll_run = st.ll.clone()
        st.refresh_ll()
        drift = float(((st.ll - ll_run).abs() / st.ll.abs()).max())
        res[name] = {"us_per_step": round(us, 3), "drift": drift}
        if a.stamps:
            cyc, op = out["ll"].cpu().numpy(), out["op"].cpu().numpy()
            res[name]["cycles_by_op"] = {int(o): round(float(cyc[op == o].mean())) for o in np.unique(op)}
            # a group's members carry the same (split) stamp: runs of equal values = group sizes
            sizes = []
            for c in range(cyc.shape[0]):
                v = cyc[c]
                brk = np.flatnonzero(np.diff(v) != 0) + 1
                sizes.extend(np.diff(np.concatenate([[0], brk, [len(v)]])).tolist())
            h = np.bincount(np.minimum(sizes, 9))
            res[name]["run_sizes"] = {int(i): int(n) for i, n in enumerate(h) if n}
            res[name]["cycles_per_step_mean"] = round(float(cyc.mean()))
        print(name, res[name], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
