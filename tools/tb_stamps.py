"""Stage cycles of the source sampler's table passes (an SBZ_TB_STAMP=1 build of libsbz, selected with
SBZ_LIB_PATH): zone moves only at the cfg5 shape, the per-stage shader cycles per feature of a wave
(wave 0 and the last wave), from the first 16 ll-trace entries the stamp build writes.  Diagnostic only.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import bench  # noqa: E402

STAGES = ["column + weights", "table", "cells", "counts out"]


def main():
    shape = {"sites": 2000, "features": 500, "states": 10, "zones": 8, "families": 4}
    if os.environ.get("TB_SHAPE"):  # e.g. TB_SHAPE=28,47,3,3,5 (the Balkan shape)
        shape = dict(zip(["sites", "features", "states", "zones", "families"],
                         [int(v) for v in os.environ["TB_SHAPE"].split(",")]))
    chains = int(os.environ.get("TB_CHAINS", "256"))
    sets = {"zone_moves": {"shrink_zone": 0.4, "grow_zone": 0.4, "swap_zone": 0.2},
            "p_zones": {"gibbs_sample_p_zones": 1.0}, "p_global": {"gibbs_sample_p_global": 1.0},
            "weights": {"gibbs_sample_weights": 1.0}, "sources": {"gibbs_sample_sources": 1.0},
            "p_families": {"gibbs_sample_p_families": 1.0}}
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    name = sys.argv[2] if len(sys.argv) > 2 else "zone_moves"
    if name != "default":  # default: bench.src_operators, the reference's STEPS
        ops = sets[name]
        bench.src_operators = lambda inh=True: dict(ops)
    cap = {}
    orig = bench.logged_ess if hasattr(bench, "logged_ess") else None
    import contact_zones_amd.diagnostics as dg
    real = dg.logged_ess

    def grab(ll):
        cap["ll"] = np.array(ll)
        return real(np.nan_to_num(ll[:, 32:], nan=0.0, posinf=0.0, neginf=0.0))
    dg.logged_ess = grab
    r = bench.source_sampler_leg(shape, chains, steps, 0, seed=3, gpu_init=True)
    ll = cap["ll"]
    passes = ll[:, 4].mean()  # table passes run by the timed launch (slot 4 of the stamp build)
    feats = passes * (shape["features"] / 8)  # features per wave and pass (8 waves)
    w0 = ll[:, :4].mean(0) / feats
    w7 = ll[:, 16:20].mean(0) / feats
    gib = ll[:, 5:8].mean(0) / steps  # Gibbs p_* steps: subset + counts, redraw_rows, ll update
    rdr = ll[:, 8:12].mean(0) / steps  # inside redraw_rows: scan, alphas, gammas, rows + delta
    out = {"set": sys.argv[2] if len(sys.argv) > 2 else "zone_moves", "us_per_step": r["us_per_step"],
           "passes": float(passes), "cycles_per_feature_wave0": dict(zip(STAGES, w0.round(1).tolist())),
           "cycles_per_feature_lastwave": dict(zip(STAGES, w7.round(1).tolist())),
           "total_wave0": float(w0.sum()), "total_lastwave": float(w7.sum()),
           "p_step_cycles_per_step": dict(zip(["subset + counts", "redraw_rows", "ll update"],
                                              gib.round(0).tolist())),
           "redraw_cycles_per_step": dict(zip(["scan", "alphas", "gammas", "rows + delta"], rdr.round(0).tolist())),
           "p_step_total_cycles_per_step": float(ll[:, 12].mean() / steps),
           "p_step_head_cycles_per_step": float(ll[:, 13].mean() / steps),
           "weights_counts_gammas_cycles_per_step": float(ll[:, 14].mean() / steps),
           "weights_op_cycles_per_step": float(ll[:, 15].mean() / steps)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
