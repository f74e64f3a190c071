"""Replay one MH fixture on the GPU and report the first divergence per chain (debug aid)."""
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
from conftest import load_golden  # noqa: E402
import test_gpu_sampler as T  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "mh_small_bounds"
fx = load_golden(case)
eng, smp, st = T._setup(fx)
n = fx["step_op"].shape[1]
out = smp.run(st, n, fx["max_size"], fx["p_grow_connected"], tape=fx["tape"], tape_len=fx["tape_len"],
              trace=True, trace_zones=True)
torch.cuda.synchronize()
status = out["status"].cpu().numpy()
print(case, "status", status, "pos", out["tape_pos"].cpu().numpy(), "len", fx["tape_len"], flush=True)
ops = out["op"].cpu().numpy()
acc = out["accept"].cpu().numpy().astype(bool)
ll = out["ll"].cpu().numpy()
z = out["zone_of_site"].cpu().numpy()
for b in range(st.B):
    bad = np.flatnonzero((ops[b] != fx["step_op"][b]) | (acc[b] != fx["step_accept"][b]) |
                         np.any(z[b] != fx["step_zone_of_site"][b], axis=1))
    if bad.size:
        i = int(bad[0])
        print(f"chain {b}: first divergence at step {i}: op gpu={ops[b, i]} ref={fx['step_op'][b, i]} "
              f"acc gpu={acc[b, i]} ref={fx['step_accept'][b, i]} ll gpu={ll[b, i]:.6f} ref={fx['step_ll'][b, i]:.6f}")
        lo = max(0, i - 3)
        print("   prev ops", fx["step_op"][b, lo:i + 1], "acc", fx["step_accept"][b, lo:i + 1].astype(int),
              "gpu acc", acc[b, lo:i + 1].astype(int))
        print("   ll gpu", ll[b, lo:i + 1], "\n   ll ref", fx["step_ll"][b, lo:i + 1])
    else:
        print(f"chain {b}: identical")
