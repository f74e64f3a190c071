"""Draw-for-draw identity of two builds of the SAMPLE_SOURCE = true sampler (Philox mode): run the
same seeded runs with the library SBZ_LIB_PATH names and save every trace and final state, or
compare two such saves.  Diagnostic for kernel changes that must not change a single draw.

  SBZ_LIB_PATH=... python tools/src_identity.py run OUT.npz
  python tools/src_identity.py cmp A.npz B.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {
    # (N, F, S, Z, Fam, B, steps): cfg5's kernel (sources in HBM, table passes) and the LDS kernel
    "cfg5": (2000, 500, 10, 8, 4, 48, 300),
    "small": (100, 36, 5, 6, 6, 64, 2000),
}


def run_shape(name, prior_half):
    import torch
    from scipy.spatial import Delaunay

    from contact_zones_amd.likelihood import LikelihoodEngine
    from contact_zones_amd.sampler import ChainState, Sampler, precisions
    N, F, S, Z, Fam, B, steps = SHAPES[name]
    rng = np.random.default_rng(55)
    obs = rng.integers(0, S, size=(N, F)).astype(np.int8)
    obs[rng.random((N, F)) < 0.02] = -1
    fam = rng.integers(0, Fam, size=N).astype(np.uint8)
    fam[rng.random(N) < 0.2] = 255
    states = np.ones((F, S), bool)
    indptr, indices = Delaunay(rng.random((N, 2))).vertex_neighbor_vertices
    eng = LikelihoodEngine(obs, fam, S, Z, Fam, True)
    ops = {"shrink_zone": 0.03, "grow_zone": 0.03, "swap_zone": 0.02, "gibbs_sample_weights": 0.3,
           "gibbs_sample_p_global": 0.2, "gibbs_sample_p_zones": 0.22, "gibbs_sample_p_families": 0.2}
    prec = precisions({"weights": 15, "universal": 40, "contact": 20, "inheritance": 20})
    kw = {}
    if prior_half:  # Gibbs prior counts below 1: the alpha < 1 boost path
        kw = {"gibbs_counts": (np.full((F, S), 0.3), np.full((Fam, F, S), 0.45))}
    zos = np.full((B, N), 255, np.uint8)
    r = np.random.default_rng(56)
    for b in range(B):
        p = r.permutation(N)[:5 * Z]
        for z in range(Z):
            zos[b, p[5 * z:5 * z + 5]] = z
    w = np.broadcast_to(r.dirichlet(np.ones(3), size=F), (B, F, 3)).copy()
    pg = np.broadcast_to(r.dirichlet(np.ones(S), size=F), (B, F, S)).copy()
    pz = r.dirichlet(np.ones(S), size=(B, Z, F))
    pf = np.broadcast_to(r.dirichlet(np.ones(S), size=(Fam, F)), (B, Fam, F, S)).copy()
    st = ChainState(eng, zos, w, pg, pz, pf, source=np.zeros((B, N, F), np.uint8))
    Sampler(eng, states, indptr, indices, {"gibbs_sample_sources": 1.0}, prec, 3,
            sample_source=True).run(st, 1, np.full(B, 50), np.full(B, 0.85), seed=11)
    smp = Sampler(eng, states, indptr, indices, ops, prec, 3, sample_source=True, **kw)
    out = smp.run(st, steps, np.full(B, 50), np.full(B, 0.85), seed=12, trace=True)
    torch.cuda.synchronize()
    s = st.to_numpy()
    import hashlib
    # (large arrays by their SHA-256, so the saves stay small)
    res = {f"{name}_{'h' if prior_half else 'd'}_{k}": (v if v.nbytes < (1 << 20) else
           np.frombuffer(hashlib.sha256(np.ascontiguousarray(v).tobytes()).digest(), np.uint8))
           for k, v in s.items()}
    for k in ("ll", "op", "accept"):
        res[f"{name}_{'h' if prior_half else 'd'}_trace_{k}"] = out[k].cpu().numpy()
    res[f"{name}_{'h' if prior_half else 'd'}_kernels"] = np.array(str(eng.last_kernels()))
    eng.close()
    return res


def main():
    if sys.argv[1] == "run":
        res = {}
        for name in SHAPES:
            for ph in (False, True):
                res.update(run_shape(name, ph))
                print(name, ph, "done", flush=True)
        np.savez(sys.argv[2], **res)
    else:
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        bad = 0
        for k in sorted(a.files):
            same = k in b.files and a[k].shape == b[k].shape and np.array_equal(a[k], b[k], equal_nan=a[k].dtype.kind == "f")
            if not same:
                bad += 1
            print(("SAME " if same else "DIFF ") + k)
        print("IDENTICAL" if bad == 0 and set(a.files) == set(b.files) else f"DIFFERENT ({bad})")
        sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
