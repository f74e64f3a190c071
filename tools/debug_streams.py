"""Debug: identical sampler runs on several HIP streams at once vs one at a time (South America
data, one chain each, as the product runner's main run): do the trajectories match?"""
import os, random, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from contact_zones_amd import experiment, packing
from contact_zones_amd.likelihood import LikelihoodEngine
from contact_zones_amd.mcmc import InitialSamples
from contact_zones_amd.sampler import ChainState, Sampler, precisions

path = os.path.join(ROOT, "tests", "golden", "io", "data", "experiments", "south_america", "config.json")


def setup(src_mode, Z, B):
    cfg, _ = experiment.load_config(path, {"model": {"N_AREAS": Z, "SAMPLE_SOURCE": src_mode}})
    data = experiment.ExperimentData(cfg)
    t = data.table
    m, mc = cfg["model"], cfg["mcmc"]
    spec, gibbs = experiment.build_priors(cfg, data)
    Fam = len(t.family_names)
    eng = LikelihoodEngine(t.obs, t.fam_of_site, t.n_states, Z, Fam, True, device=0)
    ind = data.network["adj_mat"]
    smp = Sampler(eng, t.applicable, ind.indptr, ind.indices, experiment.operators(cfg),
                  precisions(mc["PROPOSAL_PRECISION"]), int(m["MIN_M"]), priors=spec,
                  sample_source=src_mode, gibbs_counts=gibbs if src_mode else None)
    init = InitialSamples(data.features, t.applicable, ind.indptr, ind.indices, data.families, Z,
                          mc["M_INITIAL"], True, None, random.Random(5), sample_source=src_mode,
                          np_random=np.random.RandomState(7).random_sample)
    samples = [init(b) for b in range(B)]
    zos = np.stack([packing.zones_to_zone_of_site(x.zones, t.n_sites) for x in samples])
    st = ChainState(eng, zos, np.stack([x.weights for x in samples]),
                    np.stack([np.asarray(x.p_global)[0] for x in samples]), np.stack([x.p_zones for x in samples]),
                    np.stack([x.p_families for x in samples]),
                    prior=spec.log_prior(zos, np.stack([np.asarray(x.p_global)[0] for x in samples]),
                                         np.stack([x.p_families for x in samples]), t.applicable, Z, True),
                    source=np.stack([packing.source_to_index(x.source) for x in samples]) if src_mode else None)
    return eng, smp, st, int(m["MAX_M"]), float(mc["P_GROW_CONNECTED"])


def trace(runs, launches, steps, streams):
    outs = [[] for _ in runs]
    for L in range(launches):
        for i, (eng, smp, st, mm, pg) in enumerate(runs):
            ctx = torch.cuda.stream(streams[i]) if streams else torch.cuda.stream(torch.cuda.current_stream())
            with ctx:
                o = smp.run(st, steps, mm, pg, seed=99, chain_id0=0, trace=True)
                outs[i].append(o)
        if streams:
            torch.cuda.synchronize()
        else:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return [np.concatenate([o["ll"].cpu().numpy() for o in oo], axis=1) for oo in outs]


for src_mode in (True, False):
    for B in (1, 16):
        K = 6
        ref = trace([setup(src_mode, 3, B)], 20, 500, None)[0]
        runs = [setup(src_mode, 3, B) for _ in range(K)]
        got = trace(runs, 20, 500, [torch.cuda.Stream() for _ in range(K)])
        bad = [i for i in range(K) if not np.array_equal(got[i], ref)]
        first = []
        for i in bad:
            d = np.argwhere(got[i] != ref)
            first.append(tuple(d[0]))
        print(f"source={src_mode} B={B}: {K} concurrent runs vs one alone: differing {bad} first (chain, step) {first}",
              flush=True)
