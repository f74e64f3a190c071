"""Phase cycles of the SAMPLE_SOURCE = true sampler (SBZ_SRC_STAMP=k builds, tools/
build_src_variant.sh sst<k> -DSBZ_SRC_STAMP=<k>): mean shader cycles of phase k per step, by
operator, on the bench's real-data-sized synthetic legs.  Diagnostic only.

Usage (GPU box): SBZ_LIB_PATH=.../libsbz_sst<k>.so python tools/src_stamps.py [--sites 28 ...]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from contact_zones_amd import sampler as smod  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sites", type=int, default=28)
    ap.add_argument("--features", type=int, default=47)
    ap.add_argument("--states", type=int, default=3)
    ap.add_argument("--zones", type=int, default=3)
    ap.add_argument("--families", type=int, default=5)
    ap.add_argument("--chains", type=int, default=256)
    ap.add_argument("--steps", type=int, default=2000)
    a = ap.parse_args()
    shape = {k: getattr(a, k) for k in ("sites", "features", "states", "zones", "families")}
    cap = {}
    orig = smod.Sampler.run

    def run(self, *args, **kw):
        out = orig(self, *args, **kw)
        if kw.get("trace"):
            cap["out"] = out
        return out
    smod.Sampler.run = run
    r = bench.source_sampler_leg(shape, a.chains, a.steps, 200, seed=3)
    out = cap["out"]
    cyc, op = out["ll"].cpu().numpy(), out["op"].cpu().numpy()
    by_op = {int(o): round(float(cyc[op == o].mean())) for o in np.unique(op)}
    print(json.dumps({"shape": shape, "us_per_step": round(r["us_per_step"], 3), "cycles_by_op": by_op,
                      "mean_cycles": round(float(cyc.mean()))}))


if __name__ == "__main__":
    main()
