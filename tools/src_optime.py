"""Per-operator timing of the SAMPLE_SOURCE = true sampler (mh_src_kernel) on a synthetic shape:
one operator family at a time (Philox draws), µs per step.  Diagnostic only (not part of the bench).

Usage (GPU box): python tools/src_optime.py [--sites 28 --features 47 --states 3 --zones 3
                 --families 5 --chains 256 --steps 1000]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

SETS = {
    "default": None,
    "sources": {"gibbs_sample_sources": 1.0},
    "weights": {"gibbs_sample_weights": 1.0},
    "p_global": {"gibbs_sample_p_global": 1.0},
    "p_zones": {"gibbs_sample_p_zones": 1.0},
    "p_families": {"gibbs_sample_p_families": 1.0},
    "zone_moves": {"shrink_zone": 0.4, "grow_zone": 0.4, "swap_zone": 0.2},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sites", type=int, default=28)
    ap.add_argument("--features", type=int, default=47)
    ap.add_argument("--states", type=int, default=3)
    ap.add_argument("--zones", type=int, default=3)
    ap.add_argument("--families", type=int, default=5)
    ap.add_argument("--chains", type=int, default=256)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--burnin", type=int, default=200)
    ap.add_argument("--sets", default=",".join(SETS))
    ap.add_argument("--gpu-init", action="store_true",
                    help="initial sources from one GPU gibbs_sample_sources step (fast at large shapes)")
    a = ap.parse_args()
    shape = {k: getattr(a, k) for k in ("sites", "features", "states", "zones", "families")}
    default_ops = bench.src_operators
    out = {}
    for name in a.sets.split(","):
        ops = SETS[name]
        bench.src_operators = default_ops if ops is None else (lambda inh=True, o=ops: dict(o))
        r = bench.source_sampler_leg(shape, a.chains, a.steps, a.burnin, seed=3, gpu_init=a.gpu_init)
        out[name] = round(r["us_per_step"], 3)
        print(name, out[name], flush=True)
    print(json.dumps({"shape": shape, "chains": a.chains, "us_per_step": out}))


if __name__ == "__main__":
    main()
