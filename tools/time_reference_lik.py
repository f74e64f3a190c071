"""Reference vs restatement CPU speed, both on this container's cores — BUILD CONTAINER ONLY
(imports /root/reference through tests/golden/refenv.py; the reference never travels to the GPU box).

bench.py's cpu_baseline times oracle/lik_numpy.py (kind 'port') on the GPU box's host cores.  This
tool documents how that restatement's speed relates to the reference's own
Likelihood.__call__(sample, caching=False) (sbayes/model.py:145-171) on the same single-chain input
of the bench workload, one process, one thread each (OMP / OpenBLAS threads = 1), and that both
return the same value.  Writes profiles/r03_cpu_reference_ratio.json.

Usage: OMP_NUM_THREADS=1 OPENBLAS_NUM_THREADS=1 python tools/time_reference_lik.py [seconds]
"""
import argparse
import json
import os
import sys
import time
from collections import namedtuple

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import refenv  # noqa: E402


def timed(fn, seconds):
    n, t0 = 0, time.perf_counter()
    while True:
        v = fn()
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return n / el, n, v


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 15.0
    refenv.setup()
    from sbayes.model import Likelihood
    from sbayes.sampling.zone_sampling import Sample

    import bench
    from contact_zones_amd import packing
    from oracle import lik_numpy
    out = {"seconds_per_leg": seconds, "threads": {k: os.environ.get(k) for k in
                                                    ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS")},
           "host_cpu_count": os.cpu_count(), "cases": {}}
    for fam_n in (4, 0):
        args = argparse.Namespace(sites=2000, features=500, states=10, zones=8, families=fam_n,
                                  zone_size=50, seed=5)
        rng = np.random.default_rng(args.seed)
        obs, fam = bench.make_shared(args, rng)  # the bench workload's data
        N, F, S, Z = 2000, 500, 10, 8
        zos = np.full(N, 255, np.uint8)
        perm = rng.permutation(N)
        for z in range(Z):
            zos[perm[z * 50:(z + 1) * 50]] = z
        inh = fam_n > 0
        w = rng.dirichlet(np.ones(3 if inh else 2), size=F)
        pg = rng.dirichlet(np.ones(S), size=F)
        pz = rng.dirichlet(np.ones(S), size=(Z, F))
        pf = rng.dirichlet(np.ones(S), size=(fam_n, F)) if inh else None
        Data = namedtuple("Data", ["features", "families"])
        data = Data(features=packing.obs_to_features(obs, S),
                    families=packing.index_to_groups(fam, fam_n) if inh else np.zeros((0, N), bool))
        lik = Likelihood(data=data, inheritance=inh)
        zones = packing.index_to_groups(zos, Z)
        # a fresh Sample per call: __call__ clears the sample's what_changed flags
        # (everything_updated, model.py:186-192), as each MH proposal is a new Sample
        ref_rate, ref_n, ref_v = timed(lambda: lik(Sample(zones=zones, weights=w, p_global=pg[None],
                                                          p_zones=pz, p_families=pf, source=None),
                                                   caching=False), seconds)
        port_rate, port_n, port_v = timed(lambda: lik_numpy.loglik(obs, fam, zos, w, pg, pz, pf,
                                                                   inheritance=inh), seconds)
        out["cases"][f"2000x500x10 Z8 Fam{fam_n}"] = {
            "reference_evals_per_s": ref_rate, "reference_evals": ref_n,
            "restatement_evals_per_s": port_rate, "restatement_evals": port_n,
            "restatement_over_reference": port_rate / ref_rate,
            "values_equal": bool(ref_v == port_v), "value": ref_v}
        print(fam_n, out["cases"][f"2000x500x10 Z8 Fam{fam_n}"], flush=True)
    with open(os.path.join(ROOT, "profiles", "r03_cpu_reference_ratio.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
