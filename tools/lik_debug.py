"""Compare the default likelihood kernel with the C oracle on small shapes and print the error
per shape (GPU debugging aid: python tools/lik_debug.py [tasks_per_cu])."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from contact_zones_amd.likelihood import LikelihoodEngine  # noqa: E402
from oracle import oracle_c  # noqa: E402
from test_gpu_likelihood import _random_batch  # noqa: E402

SHAPES = [(60, 16, 4, 1, 0, 3, False, 5), (60, 16, 4, 1, 2, 3, True, 5),
          (200, 32, 5, 2, 0, 4, False, 20), (300, 48, 10, 8, 4, 4, True, 20),
          (100, 36, 5, 6, 6, 4, True, 6), (2000, 64, 10, 8, 4, 3, True, 50)]
OPTIONS = {}
if len(sys.argv) > 1:  # few tasks per CU: long tasks (several 16-feature blocks, weight batches)
    OPTIONS["lik_tasks_per_cu"] = int(sys.argv[1])  # the context option (sbz_set_option)
    SHAPES = [(300, 200, 6, 4, 3, 64, True, 20), (2000, 500, 10, 8, 4, 64, True, 50)]
for (N, F, S, Z, Fam, B, inh, zs) in SHAPES:
    rng = np.random.default_rng(1)
    obs, fam, zos, w, pg, pz, pf, _ = _random_batch(rng, N, F, S, Z, Fam, B, inh, zs)
    eng = LikelihoodEngine(obs, fam, S, Z, Fam, inh, options=OPTIONS)
    got = eng.loglik(zos, w, pg, pz, pf)
    nb = min(B, 4)
    ref = oracle_c.loglik_batch(obs, fam, zos[:nb], w[:nb], pg[:nb], pz[:nb], pf[:nb] if inh else None,
                                inheritance=inh)
    print((N, F, S, Z, Fam, B, inh), "max rel", np.max(np.abs(got[:nb] - ref) / np.abs(ref)), got[:2], ref[:2],
          flush=True)
    eng.close()
