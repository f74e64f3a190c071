"""Debug: the full likelihood (ChainState.refresh_ll, source branch / mixture) launched on several
HIP streams at once vs alone: bitwise identical?  Also the sampler with refresh_ll after every
launch, as the product's BatchedZoneMCMC._advance does."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.debug_streams import setup  # noqa: E402


def lik_probe(src_mode, B, K=6, R=50):
    runs = [setup(src_mode, 3, B) for _ in range(K)]
    ref = runs[0][2].refresh_ll().clone()
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(K)]
    outs = [[] for _ in range(K)]
    for r in range(R):
        for i, (eng, smp, st, mm, pg) in enumerate(runs):
            with torch.cuda.stream(streams[i]):
                outs[i].append(st.refresh_ll().clone())
    torch.cuda.synchronize()
    bad = sum(int(not torch.equal(o, ref)) for oo in outs for o in oo)
    print(f"lik source={src_mode} B={B}: {K} streams x {R} launches, {bad} differ from the lone launch", flush=True)


def sampler_probe(src_mode, B, K=6, L=20, steps=200):
    def go(runs, streams):
        lls = [[] for _ in runs]
        for _ in range(L):
            for i, (eng, smp, st, mm, pg) in enumerate(runs):
                with torch.cuda.stream(streams[i] if streams else torch.cuda.current_stream()):
                    o = smp.run(st, steps, mm, pg, seed=99, chain_id0=0)
                    st.refresh_ll()
                    lls[i].append(st.ll.clone())
            torch.cuda.synchronize()
        return [torch.stack(x).cpu().numpy() for x in lls]
    ref = go([setup(src_mode, 3, B)], None)[0]
    got = go([setup(src_mode, 3, B) for _ in range(K)], [torch.cuda.Stream() for _ in range(K)])
    bad = [i for i in range(K) if not np.array_equal(got[i], ref)]
    print(f"sampler+refresh source={src_mode} B={B}: differing runs {bad}", flush=True)


for src_mode in (True, False):
    for B in (1, 16):
        lik_probe(src_mode, B)
        sampler_probe(src_mode, B)
