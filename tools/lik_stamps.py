"""Phase breakdown of the dense likelihood kernel from an SBZ_LIK_STAMP build (diagnostic only).

    tools/build_variant.sh stamp -DSBZ_LIK_STAMP=1
    SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_stamp.so python tools/lik_stamps.py

Runs the bench workload (cfg5, 256 chains) once per phase; the stamp build returns, per chain,
the s_memtime cycles its waves spent in that phase.  Prints cycles per wave-feature.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from contact_zones_amd.likelihood import LikelihoodEngine  # noqa: E402

PHASES = ["weights", "table build", "load issue", "gathers+renorm", "task set-up", "whole task"]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--chains", type=int, default=256)
    a = p.parse_args()
    sys.argv = sys.argv[:1]
    args = bench.parse()  # the bench's defaults: the cfg5 workload
    rng = np.random.default_rng(args.seed)
    obs, fam = bench.make_shared(args, rng)
    args._fam = fam
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed)
    t = bench.make_chains_torch(args, a.chains, gen, dev)
    eng = LikelihoodEngine(obs, fam, args.states, args.zones, args.families, args.families > 0, 0)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    out = torch.empty(a.chains, dtype=torch.float64, device=dev)
    res = {}
    for k, name in enumerate(PHASES):
        os.environ["SBZ_STAMP_PHASE"] = str(k)
        for _ in range(3):  # warm, then keep the last
            eng.loglik_device(a.chains, t["zos"].data_ptr(), t["w"].data_ptr(), t["pg"].data_ptr(),
                              t["pz"].data_ptr(), t["pf"].data_ptr(), 0, out.data_ptr(), validate=False)
        torch.cuda.synchronize()
        res[name] = float(out.double().mean().cpu()) / args.features  # cycles per chain-feature
    print(json.dumps({"cycles_per_wave_feature": res}))
    eng.close()


if __name__ == "__main__":
    main()
