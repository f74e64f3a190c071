#!/usr/bin/env python3
"""Benchmark: batched full sBayes log-likelihood evaluations on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[4], the roofline run, per GPU): synthetic 2000 sites x
500 features x 10 states, 8 zones, 4 families (inheritance, C = 3), 256 chains per GPU
(2048 over 8 GPUs), mixture likelihood = Likelihood.__call__(sample, caching=False)
(sbayes/model.py:145-171) per chain.  One step = one batched evaluation of all 256
resident chains: one lik_mixture_kernel launch (the chain's last task adds the task
partials in-kernel; there is no second launch).  Chains are
sharded by rank (weak scaling, no collective in the timed loop); the timed region is
bracketed by a barrier + device synchronize, and the max over ranks is reported.

Inputs are resident in HBM before timing.  To keep the measurement an HBM one (the
256 chains' parameters are 137 MB and would otherwise sit in the 256 MiB Infinity
Cache), each step evaluates the next of --pool disjoint chain batches (default 4,
548 MB in total), so every launch streams parameters that were evicted since their
last use.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "likelihood-evals/sec + ESS/sec, 2000 sites×500 feat, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--chains", type=int, default=256, help="chains per GPU")
    p.add_argument("--pool", type=int, default=4, help="disjoint chain batches cycled per step")
    p.add_argument("--sites", type=int, default=2000)
    p.add_argument("--features", type=int, default=500)
    p.add_argument("--states", type=int, default=10)
    p.add_argument("--zones", type=int, default=8)
    p.add_argument("--families", type=int, default=4)
    p.add_argument("--zone-size", type=int, default=50,
                   help="sites per zone (default: the reference's MAX_M, default_config.json:30)")
    p.add_argument("--mode", choices=["mixture", "source"], default="mixture")
    p.add_argument("--cpu-seconds", type=float, default=12.0,
                   help="bounded CPU-baseline sample (0 disables)")
    p.add_argument("--cpu-sampler-seconds", type=float, default=12.0,
                   help="sampler CPU baseline: seconds per worker process (0 disables)")
    p.add_argument("--cpu-src-sampler-seconds", type=float, default=12.0,
                   help="SAMPLE_SOURCE = true sampler CPU baseline: seconds per worker process (0 disables)")
    p.add_argument("--cpu-procs", type=int, default=0,
                   help="CPU baseline: worker processes, one per core (0: the cores this process "
                        "may run on, at most 16 = a one-GPU box's CPU share)")
    p.add_argument("--seed", type=int, default=5)
    p.add_argument("--launch-check", action="store_true",
                   help="only start the ranks (gloo, no GPU) and report the world size")
    p.add_argument("--mh-steps", type=int, default=50000,
                   help="sampler leg: timed MH steps per chain (0 disables the leg)")
    p.add_argument("--mh-burnin", type=int, default=200000, help="sampler leg: untimed MH steps")
    p.add_argument("--source-lik-steps", type=int, default=20,
                   help="source-branch likelihood leg: timed launches (0: off)")
    p.add_argument("--src-sampler-steps", type=int, default=2000,
                   help="cfg5 SAMPLE_SOURCE = true sampler leg (the reference default mode): timed MH "
                        "steps per chain (0 disables the leg)")
    p.add_argument("--src-sampler-burnin", type=int, default=500,
                   help="cfg5 SAMPLE_SOURCE = true sampler leg: untimed MH steps")
    p.add_argument("--src-steps", type=int, default=2000,
                   help="real-data sampler legs (the reference's Balkan / South America configs, "
                        "SAMPLE_SOURCE = true): timed MH steps (0 = skip)")
    p.add_argument("--src-burnin", type=int, default=2000, help="real-data legs: untimed MH steps")
    p.add_argument("--other-steps", type=int, default=100,
                   help="launches timed per other-config likelihood leg (0: skip)")
    p.add_argument("--src-chains", type=int, default=128,
                   help="real-data legs: chains per GPU (South America; Balkan runs twice as many)")
    p.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                   help="context option (include/sbz.h sbz_option, e.g. lik_tasks_per_cu=4) for every "
                        "engine of the run; A/B runs only, the defaults are the production choices")
    a = p.parse_args()
    OPTIONS.update({k: int(v) for k, v in (o.split("=", 1) for o in a.option)})
    return a


OPTIONS = {}  # --option NAME=VALUE


def make_shared(args, rng):
    import numpy as np
    N, F, S, Fam = args.sites, args.features, args.states, args.families
    obs = rng.integers(0, S, size=(N, F)).astype(np.int8)
    obs[rng.random((N, F)) < 0.02] = -1
    fam = rng.integers(0, max(Fam, 1), size=N).astype(np.uint8)
    fam[rng.random(N) < 0.2] = 255
    if Fam == 0:  # no families: the model without inheritance (C = 2)
        fam[:] = 255
    return obs, fam


def make_chains_torch(args, n_chains, gen, dev, eng=None):
    """Chain states on the device: disjoint zones of --zone-size sites, Dirichlet(1) parameters;
    in source mode the sources by position ([B][F][Np], `src_pm`, the layout the sampler keeps and
    the likelihood reads in place), generated by site and transposed once by the engine."""
    import torch
    N, F, S, Z, Fam = args.sites, args.features, args.states, args.zones, args.families
    C = 3 if Fam > 0 else 2

    zone_size = min(args.zone_size, N // max(Z, 1))
    perm = torch.argsort(torch.rand(n_chains, N, generator=gen, device=dev), dim=1)
    zos = torch.full((n_chains, N), 255, dtype=torch.uint8, device=dev)
    for z in range(Z):
        idx = perm[:, z * zone_size:(z + 1) * zone_size]
        zos.scatter_(1, idx, torch.full_like(idx, z, dtype=torch.uint8))
    w = -torch.log(torch.rand(n_chains, F, C, generator=gen, device=dev, dtype=torch.float64))
    w = w / w.sum(-1, keepdim=True)

    def probs(*shape):
        x = -torch.log(torch.rand(*shape, S, generator=gen, device=dev, dtype=torch.float64))
        return x / x.sum(-1, keepdim=True)

    pg = probs(n_chains, F)
    pz = probs(n_chains, Z, F)
    pf = probs(n_chains, Fam, F) if Fam > 0 else None
    src = None
    if args.mode == "source":  # allowed components only: global, zone where zoned, family where present
        r = torch.rand(n_chains, N, F, generator=gen, device=dev)
        src = torch.zeros(n_chains, N, F, dtype=torch.uint8, device=dev)
        src[(zos[:, :, None] != 255) & (r > 0.5)] = 1
        fam_t = torch.as_tensor(args._fam, device=dev)
        if C == 3:
            src[(fam_t[None, :, None] != 255) & (r < 0.25)] = 2
        del r
    src_pm = None
    if src is not None:
        src_pm = torch.zeros(n_chains, F, eng.n_positions, dtype=torch.uint8, device=dev)
        eng.source_layout_device(n_chains, src.data_ptr(), src_pm.data_ptr(), True)
        torch.cuda.synchronize()
        del src
    return dict(zos=zos.contiguous(), w=w.contiguous(), pg=pg.contiguous(), pz=pz.contiguous(),
                pf=pf.contiguous() if pf is not None else None, src_pm=src_pm)


def algorithmic_bytes(args, B, source=False):
    """bytes/eval = P + D/B; a launch of B chains moves B*P + D bytes."""
    N, F, S, Z, Fam = args.sites, args.features, args.states, args.zones, args.families
    C = 3 if Fam > 0 else 2
    P = 8 * F * S * (1 + Z + Fam) + 8 * F * C + N + (N * F if source else 0)
    D = N * F + N
    return P, D, B * P + D


def kernel_source_hash():
    """sha256 (16 hex digits) of the HIP sources and headers libsbz.so is built from: a committed
    PMC profile (profiles/r*_pmc.json, its _meta.source_hash) is used for this run's counters only
    when it was measured on the same kernel sources."""
    import glob
    import hashlib
    h = hashlib.sha256()
    for fn in sorted(glob.glob(os.path.join(ROOT, "contact_zones_amd", "csrc", "*.hip")) +
                     glob.glob(os.path.join(ROOT, "contact_zones_amd", "csrc", "*.h")) +
                     [os.path.join(ROOT, "include", "sbz.h")]):
        with open(fn, "rb") as f:
            h.update(os.path.basename(fn).encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def _pmc_profiles(args, B):
    """The committed PMC summaries of this workload, newest first, as (file, summary, current):
    current = measured on this build's kernel sources (kernel_source_hash)."""
    import glob
    here = os.path.dirname(os.path.abspath(__file__))
    cur = kernel_source_hash()
    out = []
    for fn in sorted(glob.glob(os.path.join(here, "profiles", "r*_pmc*.json")), reverse=True):
        try:
            d = json.load(open(fn))
        except (OSError, ValueError):
            continue
        if d.get("_meta", {}).get("workload_key") == workload_key(args, B):
            out.append((os.path.relpath(fn, here), d, d["_meta"].get("source_hash") == cur))
    return out


def workload_key(args, B):
    return (f"{args.sites}x{args.features}x{args.states}/Z{args.zones}x{args.zone_size}/"
            f"Fam{args.families}/B{B}/{args.mode}")


def pmc_traffic(args, B):
    """HBM bytes per launch of the dominant kernel from the newest committed PMC summary of this
    workload measured on these kernel sources (profiles/r*_pmc.json, written by tools/pmc.sh +
    tools/pmc_summary.py), or (None, None, note) when there is none."""
    profs = _pmc_profiles(args, B)
    for fn, d, cur in profs:
        if cur and "_hbm" in d:
            return d["_hbm"]["traffic_bytes"], fn, None
    stale = next((fn for fn, d, _ in profs if "_hbm" in d), None)
    return None, None, (f"no PMC profile of these kernel sources; the newest of an earlier build is {stale}"
                        if stale else None)


def pmc_kernel_traffic(args, B, prefix):
    """HBM bytes per launch of the kernel whose name starts with `prefix`, from the newest committed
    PMC summary of this workload measured on these kernel sources (tools/pmc.sh runs every leg's
    kernels), or (None, None)."""
    for fn, d, cur in _pmc_profiles(args, B):
        if not cur:
            continue
        for k, v in d.get("_per_kernel", {}).items():
            if k.startswith(prefix) and "traffic_bytes" in v:
                return v["traffic_bytes"], fn
    return None, None


def pmc_source_sampler():
    """PMC counters of the source-mode sampler kernel per chain-step, from the newest committed
    profiles/r*_pmc_src*.json (tools/pmc_src.sh: the cfg5 shape, 256 chains, default operators)
    measured on these kernel sources; a note naming the newest stale one otherwise."""
    import glob
    stale = None
    for fn in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_src*.json")), reverse=True):
        try:
            d = json.load(open(fn))
        except (OSError, ValueError):
            continue
        m = d.get("_meta", {})
        rel = os.path.relpath(fn, ROOT)
        if m.get("source_hash") != kernel_source_hash():
            stale = stale or rel
            continue
        for k, e in d.get("_per_kernel", {}).items():
            if not k.startswith("mh_src_kernel") or "traffic_bytes" not in e:
                continue
            steps, n, chains = m["src_steps_total"], e["dispatches"], m["src_chains"]
            per = n / steps  # dispatch means -> per step
            return {"source": rel, "kernel": k, "set": m.get("src_set"),
                    "hbm_bytes_per_chain_step": e["traffic_bytes"] * per / chains,
                    "valu_insts_per_wave_step": e["valu_insts_per_wave"] * per if "valu_insts_per_wave" in e else None,
                    "lds_insts_per_wave_step": e["lds_insts_per_wave"] * per if "lds_insts_per_wave" in e else None,
                    "wait_any_frac": e.get("wait_any_frac"), "active_inst_any_frac": e.get("active_inst_any_frac"),
                    "lds_bank_conflict_frac": e.get("lds_bank_conflict_frac"), "l2_hit_rate": e.get("l2_hit_rate"),
                    "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE x1; averaged over the profile's "
                                  "dispatches and divided by its steps"}
    return {"note": f"no PMC profile of these kernel sources; the newest of an earlier build is {stale}"
            if stale else "no PMC profile"}


def pmc_secondary(args, B):
    """The binding on-chip resources of the dominant kernel, from the same committed PMC summary
    as `traffic` (its average counters per launch; these kernel sources only): the LDS array's busy
    share of the CU cycles (SQ_LDS_IDX_ACTIVE counts LDS-array cycles, MI355X_MICROARCH.md) and the
    VALU issue share of the SIMD cycles (SQ_ACTIVE_INST_VALU counts quad-cycles).  The kernel's
    elapsed cycles per XCD are GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs); 256 CUs, 1024 SIMDs."""
    for fn, d, cur in _pmc_profiles(args, B):
        if not cur or "_hbm" not in d:
            continue
        s = d.get(d["_hbm"]["kernel"], {})
        cyc = s.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        if not cyc or "SQ_LDS_IDX_ACTIVE" not in s or "SQ_ACTIVE_INST_VALU" not in s:
            return None
        return {"lds_array_busy": s["SQ_LDS_IDX_ACTIVE"] / (256 * cyc),
                "lds_bank_conflict_share": s.get("SQ_LDS_BANK_CONFLICT", 0.0) / s["SQ_LDS_IDX_ACTIVE"],
                "valu_issue": 4.0 * s["SQ_ACTIVE_INST_VALU"] / (1024 * cyc),
                "source": fn,
                "formula": "lds_array_busy = SQ_LDS_IDX_ACTIVE / (256 CUs x GRBM_GUI_ACTIVE/8); "
                           "valu_issue = 4 x SQ_ACTIVE_INST_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE/8)"}
    return None


def _cpu_worker(shape, seconds, seed):
    """One CPU-baseline process: Likelihood.__call__(caching=False) restated in numpy
    (oracle/lik_numpy.py, bit-exact with the reference on the golden vectors) on one chain of
    the bench workload, repeated for `seconds`.  A child interpreter with OMP_NUM_THREADS =
    OPENBLAS_NUM_THREADS = 1, so it is one core's worth of work."""
    import argparse
    import numpy as np
    from oracle import lik_numpy
    args = argparse.Namespace(**shape)
    rng = np.random.default_rng(seed)
    obs, fam = make_shared(args, rng)
    N, F, S, Z, Fam = args.sites, args.features, args.states, args.zones, args.families
    zos = np.full(N, 255, np.uint8)
    perm = rng.permutation(N)
    zs = min(args.zone_size, N // max(Z, 1))
    for z in range(Z):
        zos[perm[z * zs:(z + 1) * zs]] = z
    inh = Fam > 0
    w = rng.dirichlet(np.ones(3 if inh else 2), size=F)
    pg = rng.dirichlet(np.ones(S), size=F)
    pz = rng.dirichlet(np.ones(S), size=(Z, F))
    pf = rng.dirichlet(np.ones(S), size=(Fam, F)) if inh else None
    n = 0
    t0 = time.perf_counter()
    while True:
        lik_numpy.loglik(obs, fam, zos, w, pg, pz, pf, inheritance=inh)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"n": n, "seconds": el}


def _cpu_sampler_worker(shape, seconds, seed):
    """One CPU-baseline sampler process: the MH step loop restated in numpy (oracle/mh_numpy.step,
    MCMCGenerative.step with the ZoneMCMC operators, every candidate's log-likelihood a full
    lik_numpy evaluation) with its decisions drawn from a numpy Generator (DrawTape), on one chain
    of the sampler leg's workload (the same synthetic data, network, initial sample, operator
    table and proposal precisions), run for `seconds`: steps and the log-likelihood trace."""
    import argparse
    import random
    import numpy as np
    from contact_zones_amd import packing
    from contact_zones_amd.mcmc import InitialSamples
    from oracle import mh_numpy
    args = argparse.Namespace(**shape)
    obs, fam = make_shared(args, np.random.default_rng(args.seed))
    N, F, S, Z, Fam = args.sites, args.features, args.states, args.zones, args.families
    indptr, indices = make_network(N, np.random.default_rng(args.seed + 17))
    states = np.ones((F, S), bool)
    init = InitialSamples(packing.obs_to_features(obs, S), states, indptr, indices,
                          packing.index_to_groups(fam, Fam), Z, MH_M_INITIAL, True, None,
                          random.Random(seed * 1000003))
    zones = init.zones()
    st = {"zos": packing.zones_to_zone_of_site(zones, N), "w": init.weights(), "pg": init.p_global()[0],
          "pz": init.p_zones(zones), "pf": init.p_families()}
    ops = mh_operators()
    prec = [MH_PRECISION[k] for k in ("weights", "universal", "contact", "inheritance")]
    fx = {"obs": obs, "fam_of_site": fam, "states": states, "inheritance": True, "warmup": False,
          "min_size": MH_MIN_M, "max_size": np.array([MH_MAX_M]), "p_grow_connected": np.array([MH_P_GROW]),
          "precision": np.array(prec, np.float64), "adj_indptr": indptr, "adj_indices": indices,
          "n_zones": Z}
    m = mh_numpy.Model(fx)
    tape = mh_numpy.DrawTape(np.random.default_rng(seed), [ops[k] for k in mh_numpy.OPS[:7]])
    ll, prior = m.loglik(st), m.log_prior(st)
    lls = []
    t0 = time.perf_counter()
    while True:
        st, ll, prior, _, _ = mh_numpy.step(m, st, ll, prior, 0, tape)
        lls.append(ll)
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"n": len(lls), "seconds": el, "ll": [float(v) for v in lls]}


def _cpu_src_sampler_worker(shape, seconds, seed):
    """One CPU-baseline process of the SAMPLE_SOURCE = true sampler: the numpy restatement of the
    MH step loop (oracle/mh_numpy.step with the zone moves' source resampling and the Gibbs
    operators, every candidate's log-likelihood a full lik_numpy evaluation of the selected
    components), decisions drawn from a numpy Generator (DrawTape: operator by probability, the
    Gibbs operators' beta / Dirichlet draws of the source counts, as the reference), on one chain of
    the source-mode leg's workload (source_sampler_leg's data, network, initial sample and initial
    sources), run for `seconds`: steps and the log-likelihood trace."""
    import random
    import numpy as np
    from scipy.spatial import Delaunay
    from contact_zones_amd import packing
    from contact_zones_amd.mcmc import InitialSamples
    from contact_zones_amd.sources import draw_sources, source_posterior
    from oracle import mh_numpy
    N, F, S, Z, Fam = (shape[k] for k in ("sites", "features", "states", "zones", "families"))
    inh = Fam > 0
    rng = np.random.default_rng(shape["seed"])  # source_sampler_leg's data and network
    obs = rng.integers(0, S, size=(N, F)).astype(np.int8)
    obs[rng.random((N, F)) < 0.02] = -1
    fam = rng.integers(0, max(Fam, 1), size=N).astype(np.uint8)
    fam[rng.random(N) < 0.2] = 255
    if not inh:
        fam[:] = 255
    indptr, indices = Delaunay(rng.random((N, 2))).vertex_neighbor_vertices
    states = np.ones((F, S), bool)
    init = InitialSamples(packing.obs_to_features(obs, S), states, indptr, indices,
                          packing.index_to_groups(fam, Fam) if inh else np.zeros((0, N), bool), Z,
                          MH_M_INITIAL, inh, None, random.Random(seed * 1000003))
    zones = init.zones()
    st = {"zos": packing.zones_to_zone_of_site(zones, N), "w": init.weights(), "pg": init.p_global()[0],
          "pz": init.p_zones(zones)}
    if inh:
        st["pf"] = init.p_families()
    st["src"] = draw_sources(source_posterior(obs, fam, st["zos"], st["w"], st["pg"], st["pz"], st.get("pf"), inh),
                             np.random.default_rng(seed + 31).random)
    ops = src_operators(inh)
    prec = [MH_PRECISION[k] for k in ("weights", "universal", "contact", "inheritance")]
    fx = {"obs": obs, "fam_of_site": fam, "states": states, "inheritance": inh, "warmup": False,
          "min_size": MH_MIN_M, "max_size": np.array([MH_MAX_M]), "p_grow_connected": np.array([MH_P_GROW]),
          "precision": np.array(prec, np.float64), "adj_indptr": indptr, "adj_indices": indices,
          "n_zones": Z, "sample_source": True, "gibbs_counts_global": np.ones((F, S)),
          "gibbs_counts_fam": np.ones((max(Fam, 1), F, S)) if inh else None}
    m = mh_numpy.Model(fx)
    probs = [ops.get(k, 0.0) for k in mh_numpy.OPS]
    tape = mh_numpy.DrawTape(np.random.default_rng(seed), probs)
    ll, prior = m.loglik(st), m.log_prior(st)
    lls = []
    t0 = time.perf_counter()
    while True:
        st, ll, prior, _, _ = mh_numpy.step(m, st, ll, prior, 0, tape)
        lls.append(ll)
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"n": len(lls), "seconds": el, "ll": [float(v) for v in lls]}


CPU_WORKERS = {"lik": _cpu_worker, "sampler": _cpu_sampler_worker, "src_sampler": _cpu_src_sampler_worker}


def _cgroup_cpus():
    """CPUs of this process's cgroup v2 quota (cpu.max 'quota period'), or None without one."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        return None


def _cpu_procs(args):
    """Worker processes of a CPU-baseline leg: one per core this process may use — the affinity
    mask, bounded by the cgroup's CPU quota (more processes than the quota only time-slice) and by
    the GPU box's CPU share of 16 (the pool's rule for one-GPU jobs)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    quota = _cgroup_cpus()
    usable = min(avail, int(quota)) if quota else avail
    procs = args.cpu_procs if args.cpu_procs > 0 else max(1, min(16, usable))
    return procs, avail, quota, usable


def _run_cpu_workers(kind, shape, seconds, seeds):
    """Run one CPU worker per seed as a child interpreter (`bench.py --cpu-worker`, single-threaded
    BLAS / OpenMP, nothing of this process's GPU state), all at once; every child has exited when
    this returns.  Returns their JSON results."""
    import subprocess
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-worker",
                            json.dumps({"kind": kind, "shape": shape, "seconds": seconds, "seed": sd})],
                           stdout=subprocess.PIPE, env=env) for sd in seeds]
    out = []
    try:
        for p in ps:
            so, _ = p.communicate(timeout=seconds * 10 + 300)
            if p.returncode != 0:
                raise SystemExit(f"CPU baseline worker ({kind}) failed with status {p.returncode}")
            out.append(json.loads(so.decode().strip().splitlines()[-1]))
    finally:
        for p in ps:
            if p.poll() is None:
                p.kill()
                p.wait()
    return out


def cpu_baseline(args, seconds):
    """SURVEY.md §8d CPU timing: one process per host core (single-threaded BLAS/OpenMP), each
    evaluating one chain of the bench workload for `seconds`; per-core and all-core evals/s
    with os.cpu_count() stated.  Kind 'port': the numpy restatement of the reference's
    Likelihood.__call__ (the reference itself never travels to the GPU box); its speed relative to
    the reference, both timed in the build container, is in profiles/r03_cpu_reference_ratio.json."""
    procs, avail, quota, usable = _cpu_procs(args)
    shape = {k: getattr(args, k) for k in ("sites", "features", "states", "zones", "families", "zone_size")}
    res = _run_cpu_workers("lik", shape, seconds, [args.seed] * procs)
    rates = [r["n"] / r["seconds"] for r in res]
    N, F, S, Z, Fam = args.sites, args.features, args.states, args.zones, args.families
    ratio = None  # restatement / reference speed, both timed in the build container
    try:
        with open(os.path.join(ROOT, "profiles", "r03_cpu_reference_ratio.json")) as f:
            case = json.load(f)["cases"].get(f"{N}x{F}x{S} Z{Z} Fam{Fam}")
        ratio = case["restatement_over_reference"] if case else None
    except (OSError, ValueError, KeyError):
        pass
    extra = {}
    if ratio:
        extra = {"restatement_over_reference": ratio,
                 "reference_equivalent_value": float(sum(rates)) / ratio,
                 "ratio_source": "profiles/r03_cpu_reference_ratio.json (tools/time_reference_lik.py)"}
    return {"value": float(sum(rates)), "unit": "likelihood-evals/s", "cores": procs, "kind": "port",
            **extra,
            "per_core": float(sum(rates) / procs), "per_core_min": float(min(rates)),
            "host_cpu_count": os.cpu_count(), "cores_available": avail, "cgroup_cpu_quota": quota,
            "per_gpu_share": {"cores": procs, "value": float(sum(rates))},
            "all_core_extrapolated": {"cores": usable, "value": float(sum(rates) / procs) * usable,
                                      "how": "measured per-core rate x the usable cores (affinity "
                                             "mask, cgroup quota); not run"},
            "sample": f"numpy restatement of Likelihood.__call__(caching=False) (oracle/lik_numpy.py), "
                      f"one chain at {N}x{F}x{S}, Z={Z}, Fam={Fam} per process, {procs} processes x "
                      f"{seconds:.0f} s, 1 thread each ({sum(r['n'] for r in res)} evals)"}


def cpu_baseline_sampler(args, seconds):
    """The sampler's CPU baseline, timed: one process per usable core, each running the numpy
    restatement of the MH step loop (oracle/mh_numpy.step, decisions drawn from numpy) on its own
    chain of the sampler leg's cfg5 workload for `seconds`: steps/s per core and all-core, ESS/s of
    the log-likelihood traces (Tracer's estimator on every step; a trace of this length is mostly
    the chain's initial transient, so the ESS is an upper bound of little weight).  The
    restatement's speed against the reference's own ZoneMCMC on the same shape, both timed in the
    build container, is in profiles/r05_cpu_reference_sampler_ratio.json."""
    import numpy as np
    from contact_zones_amd.diagnostics import ess
    procs, avail, quota, usable = _cpu_procs(args)
    shape = {k: getattr(args, k) for k in ("sites", "features", "states", "zones", "families", "zone_size",
                                           "seed")}
    res = _run_cpu_workers("sampler", shape, seconds, [args.seed * 7919 + i for i in range(procs)])
    rates = [r["n"] / r["seconds"] for r in res]
    e = [float(ess(np.asarray(r["ll"])[None, :], max_lag=None)[0]) if r["n"] > 3 else 0.0 for r in res]
    wall = max(r["seconds"] for r in res)
    out = {"value": float(sum(rates)), "unit": "MH steps/s", "cores": procs, "kind": "port",
           "per_core": float(sum(rates) / procs), "per_core_min": float(min(rates)),
           "ess_per_sec": float(sum(e) / wall), "steps_per_process": [r["n"] for r in res],
           "host_cpu_count": os.cpu_count(), "cores_available": avail, "cgroup_cpu_quota": quota,
           "sample": f"numpy restatement of MCMCGenerative.step + ZoneMCMC operators "
                     f"(oracle/mh_numpy.step, DrawTape decisions), one chain of the sampler leg's "
                     f"workload per process, {procs} processes x {seconds:.0f} s, 1 thread each"}
    try:
        with open(os.path.join(ROOT, "profiles", "r05_cpu_reference_sampler_ratio.json")) as f:
            r = json.load(f)
        out.update({"restatement_over_reference": r["restatement_over_reference"],
                    "reference_equivalent_value": out["value"] / r["restatement_over_reference"],
                    "ratio_source": "profiles/r05_cpu_reference_sampler_ratio.json "
                                    "(tools/time_reference_sampler.py cfg5)"})
    except (OSError, ValueError, KeyError):
        pass
    return out


def cpu_baseline_src_sampler(args, seconds):
    """The SAMPLE_SOURCE = true sampler's CPU baseline on the GPU box: one process per usable core,
    each running the numpy restatement of the source-mode MH step loop (_cpu_src_sampler_worker) on
    its own chain of the sampler_source_mode leg's cfg5 workload for `seconds`: steps/s per core and
    all-core, ESS/s of the log-likelihood traces.  The reference's own source-mode ZoneMCMC on the
    same shape, timed in the build container (the reference never travels to the box), gives the
    restatement / reference ratio (profiles/r05_cpu_reference_source_sampler.json)."""
    import numpy as np
    from contact_zones_amd.diagnostics import ess
    procs, avail, quota, usable = _cpu_procs(args)
    shape = {k: getattr(args, k) for k in ("sites", "features", "states", "zones", "families", "seed")}
    res = _run_cpu_workers("src_sampler", shape, seconds, [args.seed * 6151 + i for i in range(procs)])
    rates = [r["n"] / r["seconds"] for r in res]
    e = [float(ess(np.asarray(r["ll"])[None, :], max_lag=None)[0]) if r["n"] > 3 else 0.0 for r in res]
    wall = max(r["seconds"] for r in res)
    out = {"value": float(sum(rates)), "unit": "MH steps/s", "cores": procs, "kind": "port",
           "per_core": float(sum(rates) / procs), "per_core_min": float(min(rates)),
           "ess_per_sec": float(sum(e) / wall), "steps_per_process": [r["n"] for r in res],
           "host_cpu_count": os.cpu_count(), "cores_available": avail, "cgroup_cpu_quota": quota,
           "sample": f"numpy restatement of MCMCGenerative.step + ZoneMCMC operators with SAMPLE_SOURCE = "
                     f"true (oracle/mh_numpy.step: zone moves resample every source, Gibbs weights / p_* "
                     f"draws from the source counts), one chain of the source-mode leg's workload per "
                     f"process, {procs} processes x {seconds:.0f} s, 1 thread each"}
    try:
        with open(os.path.join(ROOT, "profiles", "r06_cpu_source_sampler_ratio.json")) as f:
            r = json.load(f)
        out.update({"restatement_over_reference": r["restatement_over_reference"],
                    "reference_equivalent_value": out["value"] / r["restatement_over_reference"],
                    "ratio_source": "profiles/r06_cpu_source_sampler_ratio.json (restatement and the "
                                    "reference's ZoneMCMC, SAMPLE_SOURCE = true, cfg5, both timed in the "
                                    "build container, 1 thread)"})
    except (OSError, ValueError, KeyError):
        pass
    return out


# sampler leg: the reference defaults (config/default_config.json:6-20, 29-30)
MH_STEPS_CFG = {"area": 0.05, "weights": 0.4, "universal": 0.05, "contact": 0.4, "inheritance": 0.1}
MH_PRECISION = {"weights": 15, "universal": 40, "contact": 20, "inheritance": 20}
MH_MIN_M, MH_MAX_M, MH_M_INITIAL, MH_P_GROW = 3, 50, 5, 0.85


def mh_operators():
    """MCMC.steps_per_operator (mcmc_setup.py:70-95), SAMPLE_SOURCE = false, normalised."""
    a = MH_STEPS_CFG
    ops = {"shrink_zone": a["area"] * 0.4, "grow_zone": a["area"] * 0.4, "swap_zone": a["area"] * 0.2,
           "gibbsish_sample_zones": 0.0, "alter_weights": a["weights"],
           "alter_p_global": a["universal"], "alter_p_zones": a["contact"],
           "alter_p_families": a["inheritance"]}
    tot = sum(ops.values())
    return {k: v / tot for k, v in ops.items()}


def make_network(N, rng):
    """Delaunay adjacency of random locations (the reference's compute_network) as sorted CSR."""
    import numpy as np
    from scipy.spatial import Delaunay
    import scipy.sparse as sp
    indptr, indices = Delaunay(rng.random((N, 2))).vertex_neighbor_vertices
    a = sp.csr_matrix((np.ones(indices.size), indices, indptr), shape=(N, N))
    a.sort_indices()
    return a.indptr.astype(np.int32), a.indices.astype(np.int32)


def sampler_leg(args, eng, obs, fam, dev, rank, world, stream):
    """B chains x K MH steps in one launch (ZoneMCMC.step, default operators); ESS of the
    log-likelihood traces (contact_zones_amd/diagnostics.py)."""
    import random
    import numpy as np
    import torch
    import torch.distributed as dist
    from contact_zones_amd import packing
    from contact_zones_amd.diagnostics import ess, logged_ess
    from contact_zones_amd.mcmc import InitialSamples
    from contact_zones_amd.sampler import ChainState, Sampler, precisions
    N, F, S, Z, Fam = args.sites, args.features, args.states, args.zones, args.families
    B, K = args.chains, args.mh_steps
    rng = np.random.default_rng(args.seed + 17)
    indptr, indices = make_network(N, rng)  # same network on every rank
    states = np.ones((F, S), bool)
    feats = packing.obs_to_features(obs, S)
    fams = packing.index_to_groups(fam, Fam)
    init = InitialSamples(feats, states, indptr, indices, fams, Z, MH_M_INITIAL, True, None,
                          random.Random(args.seed * 1000003 + rank))
    pg0, pf0, w0 = init.p_global()[0], init.p_families(), init.weights()
    zos = np.empty((B, N), np.uint8)
    pz = np.empty((B, Z, F, S))
    for b in range(B):  # generate_initial_sample per chain (zones + p_zones MLE; the rest shared)
        zones = init.zones()
        zos[b] = packing.zones_to_zone_of_site(zones, N)
        pz[b] = init.p_zones(zones)
    rep = lambda a: np.broadcast_to(a, (B,) + a.shape).copy()  # noqa: E731
    st = ChainState(eng, zos, rep(w0), rep(pg0), pz, rep(pf0))
    smp = Sampler(eng, states, indptr, indices, mh_operators(), precisions(MH_PRECISION), MH_MIN_M)
    seed = args.seed * 7919
    if args.mh_burnin > 0:
        smp.run(st, args.mh_burnin, MH_MAX_M, MH_P_GROW, seed=seed, chain_id0=rank * B)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    out = smp.run(st, K, MH_MAX_M, MH_P_GROW, seed=seed, chain_id0=rank * B, trace=True)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    status = out["status"].cpu().numpy()
    if np.any(status != 0):
        raise SystemExit(f"sampler leg: chain status {np.unique(status)}")
    ll_trace = out["ll"].cpu().numpy()
    ll_full = st.ll.clone()
    st.refresh_ll()  # drift of the incremental log-likelihood over burn-in + K steps
    drift = float(((st.ll - ll_full).abs() / st.ll.abs()).max())
    # ESS as Tracer computes it on the samples the reference logs (every ceil(K / 1000)-th step),
    # and of the full per-step trace with no lag cap
    e, sps, capped = logged_ess(ll_trace)
    e_full = ess(ll_trace, max_lag=None)
    acc = out["accept"].float().mean().item()
    t = torch.tensor([wall, ev0.elapsed_time(ev1) / 1e3, float(e.sum()), drift, acc,
                      float(e_full.sum()), float(capped.sum())], dtype=torch.float64, device=dev)
    if world > 1:
        red = t.clone()
        _all_reduce(red, dist.ReduceOp.MAX)
        sm = t.clone()
        _all_reduce(sm, dist.ReduceOp.SUM)
        t = torch.stack([red[0], red[1], sm[2], red[3], sm[4] / world, sm[5], sm[6]])
    wall_max, dev_s, ess_tot, drift_max, acc_mean, ess_full_tot, n_capped = (float(v) for v in t)
    return {
        "mh_steps_per_sec": B * K * world / wall_max,
        "ess_per_sec": ess_tot / wall_max,
        "ess_total": ess_tot,
        "ess_per_chain_mean": ess_tot / (B * world),
        "ess_trace": f"Tracer ESS (lag cap 2000 samples) of the log-likelihood samples the reference "
                     f"logs: every {sps}-th step of {K} (N_SAMPLES 1000, mcmc_generative.py:205-218)",
        "ess_capped_chains": int(n_capped),
        "ess_capped_note": "chains whose autocovariance pair sums stayed positive up to the lag cap "
                           "(max_lag or the logged trace's length): their ESS is an upper bound",
        "ess_full_trace_per_sec": ess_full_tot / wall_max,
        "ess_full_trace_per_chain_mean": ess_full_tot / (B * world),
        "chains": B * world,
        "steps": K,
        "burnin": args.mh_burnin,
        "wall_s": wall_max,
        "device_s": dev_s,
        "us_per_step": dev_s / K * 1e6,
        "acceptance": acc_mean,
        "ll_drift_rel_max": drift_max,
        "operators": "default_config.json STEPS (area .05 / weights .4 / universal .05 / contact .4 / "
                     "inheritance .1), PROPOSAL_PRECISION 15/40/20/20, MIN_M 3, MAX_M 50, M_INITIAL 5, "
                     "P_GROW_CONNECTED .85; Delaunay network of random locations; Philox draws",
    }


# source-mode leg: config/default_config.json STEPS with SAMPLE_SOURCE = true (source 0.0: zone
# moves resample the sources themselves), mcmc_setup.py:70-95
SRC_STEPS_CFG = dict(MH_STEPS_CFG, source=0.0)
CFG4 = {"sites": 100, "features": 36, "states": 5, "zones": 6, "families": 6}  # South America shape


def src_operators(inh=True):
    a = dict(SRC_STEPS_CFG)
    if not inh:
        a["inheritance"] = 0.0
    ops = {"shrink_zone": a["area"] * 0.4, "grow_zone": a["area"] * 0.4, "swap_zone": a["area"] * 0.2,
           "gibbsish_sample_zones": 0.0, "gibbs_sample_sources": a["source"],
           "gibbs_sample_weights": a["weights"], "gibbs_sample_p_global": a["universal"],
           "gibbs_sample_p_zones": a["contact"], "gibbs_sample_p_families": a["inheritance"]}
    tot = sum(ops.values())
    return {k: v / tot for k, v in ops.items()}


def source_sampler_leg(shape, B, K, burnin, seed, rank=0, world=1, device=0, gpu_init=False):
    """SAMPLE_SOURCE = true (the reference default) on synthetic data of `shape`: B chains per GPU
    x K Philox MH steps in one launch after `burnin` untimed steps; steps/s and ESS/s of the
    log-likelihood traces, max wall over ranks.  gpu_init: the chains' initial sources are drawn
    by one gibbs_sample_sources step on the GPU (every source on the global component first),
    instead of generate_initial_sample's host draw (0.2 s of numpy per chain at the cfg5 shape)."""
    import random
    import numpy as np
    import torch
    import torch.distributed as dist
    from scipy.spatial import Delaunay
    from contact_zones_amd import packing
    from contact_zones_amd.diagnostics import logged_ess
    from contact_zones_amd.likelihood import LikelihoodEngine
    from contact_zones_amd.mcmc import InitialSamples
    from contact_zones_amd.sampler import ChainState, Sampler, precisions
    from contact_zones_amd.sources import draw_sources, source_posterior
    N, F, S, Z, Fam = (shape[k] for k in ("sites", "features", "states", "zones", "families"))
    inh = Fam > 0
    rng = np.random.default_rng(seed)  # same data and network on every rank
    obs = rng.integers(0, S, size=(N, F)).astype(np.int8)
    obs[rng.random((N, F)) < 0.02] = -1
    fam = rng.integers(0, max(Fam, 1), size=N).astype(np.uint8)
    fam[rng.random(N) < 0.2] = 255
    if not inh:
        fam[:] = 255
    indptr, indices = Delaunay(rng.random((N, 2))).vertex_neighbor_vertices
    states = np.ones((F, S), bool)
    eng = LikelihoodEngine(obs, fam, S, Z, Fam, inh, device=device, options=OPTIONS)
    init = InitialSamples(packing.obs_to_features(obs, S), states, indptr, indices,
                          packing.index_to_groups(fam, Fam) if inh else np.zeros((0, N), bool), Z,
                          MH_M_INITIAL, inh, None, random.Random(seed * 1000003 + rank))
    pg0, w0 = init.p_global()[0], init.weights()
    pf0 = init.p_families() if inh else None
    zos = np.empty((B, N), np.uint8)
    pz = np.empty((B, Z, F, S))
    src = np.zeros((B, N, F), np.uint8)
    draws = np.random.default_rng(seed + 31 * rank)
    for b in range(B):  # generate_initial_sample per chain, with its initial source draw
        zones = init.zones()
        zos[b] = packing.zones_to_zone_of_site(zones, N)
        pz[b] = init.p_zones(zones)
        if not gpu_init:
            src[b] = draw_sources(source_posterior(obs, fam, zos[b], w0, pg0, pz[b], pf0, inh), draws.random)
    rep = lambda x: np.broadcast_to(x, (B,) + x.shape).copy()  # noqa: E731
    st = ChainState(eng, zos, rep(w0), rep(pg0), pz, rep(pf0) if inh else None, source=src)
    del src
    smp = Sampler(eng, states, indptr, indices, src_operators(inh), precisions(MH_PRECISION), MH_MIN_M,
                  sample_source=True)
    if gpu_init:  # the initial Gibbs draw of every source (generate_initial_sample's last step)
        Sampler(eng, states, indptr, indices, {"gibbs_sample_sources": 1.0}, precisions(MH_PRECISION),
                MH_MIN_M, sample_source=True).run(st, 1, MH_MAX_M, MH_P_GROW, seed=seed * 7919 + 1,
                                                  chain_id0=rank * B)
    if burnin:
        smp.run(st, burnin, MH_MAX_M, MH_P_GROW, seed=seed * 7919, chain_id0=rank * B)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    out = smp.run(st, K, MH_MAX_M, MH_P_GROW, seed=seed * 7919, chain_id0=rank * B, trace=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    status = out["status"].cpu().numpy()
    if np.any(status != 0):
        raise SystemExit(f"source-mode leg: chain status {np.unique(status)}")
    e = logged_ess(out["ll"].cpu().numpy())[0]
    acc = out["accept"].float().mean().item()
    t = torch.tensor([wall, float(e.sum()), acc], dtype=torch.float64, device=torch.device("cuda", device))
    if world > 1:
        mx, sm = t.clone(), t.clone()
        _all_reduce(mx, dist.ReduceOp.MAX)
        _all_reduce(sm, dist.ReduceOp.SUM)
        t = torch.stack([mx[0], sm[1], sm[2] / world])
    wall_max, ess_tot, acc_mean = (float(v) for v in t)
    kernel = eng.last_kernels()
    eng.close()
    return {"workload": f"{N}x{F}x{S} Z{Z} Fam{Fam}, SAMPLE_SOURCE = true, {B} chains/GPU", "kernel": kernel,
            "mh_steps_per_sec": B * K * world / wall_max, "ess_per_sec": ess_tot / wall_max,
            "ess_per_chain_mean": ess_tot / (B * world), "chains": B * world, "steps": K,
            "burnin": burnin, "wall_s": wall_max, "us_per_step": wall_max / K * 1e6,
            "acceptance": acc_mean,
            "sources": "HBM" if 2 * N * F > 150 * 1024 else "LDS",
            "operators": "default_config.json STEPS with source 0.0 (zone moves resample every "
                         "source), Gibbs parameter operators; Philox draws"}


EXPERIMENTS = os.path.join(ROOT, "tests", "golden", "io", "data", "experiments")  # the reference's data


def real_data_leg(name, n_zones_list, B, K, burnin, seed, rank=0, world=1, device=0, concurrent=False):
    """The reference's own experiment configs on their real data (experiments/<name>/config.json:
    features, counts priors, STEPS, PROPOSAL_PRECISION, MIN_M / MAX_M / M_INITIAL, SAMPLE_SOURCE
    default true), B chains per GPU from generate_initial_sample, K Philox MH steps after `burnin`,
    for each number of zones: steps/s and ESS/s of the log-likelihood traces (max wall over
    ranks, ESS summed over ranks).

    concurrent: after the per-K runs (one at a time, as the reference's cli.py:71-84 sweeps K),
    time the whole sweep once more with every K's run launched on a stream of its own, so the
    K runs' B-chain launches share the GPU's CUs (B = 128 chains leave half of the 256 CUs idle
    when run alone); reported as `sweep_concurrent` beside the sequential sum."""
    import random
    import numpy as np
    import torch
    import torch.distributed as dist
    from contact_zones_amd import experiment, packing
    from contact_zones_amd.diagnostics import logged_ess
    from contact_zones_amd.likelihood import LikelihoodEngine
    from contact_zones_amd.mcmc import InitialSamples
    from contact_zones_amd.sampler import ChainState, Sampler, precisions
    path = os.path.join(EXPERIMENTS, name, "config.json")
    cfg0, _ = experiment.load_config(path, {"model": {"N_AREAS": int(n_zones_list[0])}})
    data = experiment.ExperimentData(cfg0)
    t = data.table
    m, mc = cfg0["model"], cfg0["mcmc"]
    inh, src_mode = bool(m["INHERITANCE"]), bool(m["SAMPLE_SOURCE"])
    Fam = len(t.family_names) if inh else 0
    indptr, indices = data.network["adj_mat"].indptr, data.network["adj_mat"].indices
    dev = torch.device("cuda", device)
    out = {"data": f"{name}: {t.n_sites} sites x {t.n_features} features x {t.n_states} states, "
                   f"{Fam} families, SAMPLE_SOURCE = {src_mode}, {B} chains/GPU",
           "runs": {}}

    def setup(Z):
        cfg, _ = experiment.load_config(path, {"model": {"N_AREAS": int(Z)}})
        spec, gibbs = experiment.build_priors(cfg, data)
        eng = LikelihoodEngine(t.obs, t.fam_of_site, t.n_states, Z, Fam, inh, device=device, options=OPTIONS)
        smp = Sampler(eng, t.applicable, indptr, indices, experiment.operators(cfg),
                      precisions(mc["PROPOSAL_PRECISION"]), int(m["MIN_M"]), priors=spec,
                      sample_source=src_mode, gibbs_counts=gibbs if src_mode else None)
        init = InitialSamples(data.features, t.applicable, indptr, indices, data.families, Z,
                              mc["M_INITIAL"], inh, None, random.Random(seed * 1000003 + 7919 * rank + Z),
                              sample_source=src_mode)
        np.random.seed(seed + 31 * rank + Z)  # the initial source draws (np.random, as the reference)
        samples = [init(b) for b in range(B)]
        zos = np.stack([packing.zones_to_zone_of_site(x.zones, t.n_sites) for x in samples])
        w = np.stack([x.weights for x in samples])
        pg = np.stack([np.asarray(x.p_global)[0] for x in samples])
        pz = np.stack([x.p_zones for x in samples])
        pf = np.stack([x.p_families for x in samples]) if inh else None
        src = np.stack([packing.source_to_index(x.source) for x in samples]) if src_mode else None
        prior = spec.log_prior(zos, pg, pf, t.applicable, Z, inh)
        st = ChainState(eng, zos, w, pg, pz, pf, prior=prior, source=src)
        return {"Z": Z, "eng": eng, "smp": smp, "st": st, "max_m": int(m["MAX_M"]),
                "p_grow": float(mc["P_GROW_CONNECTED"])}

    def launch(r, n, trace):
        return r["smp"].run(r["st"], n, r["max_m"], r["p_grow"], seed=seed * 7919 + r["Z"],
                            chain_id0=rank * B, trace=trace)

    def reduce(wall, res_list):
        e = sum(float(logged_ess(res["ll"].cpu().numpy())[0].sum()) for res in res_list)
        acc = float(np.mean([res["accept"].float().mean().item() for res in res_list]))
        for res in res_list:
            status = res["status"].cpu().numpy()
            if np.any(status != 0):
                raise SystemExit(f"{name} leg: chain status {np.unique(status)}")
        tt = torch.tensor([wall, e, acc], dtype=torch.float64, device=dev)
        if world > 1:
            mx, sm = tt.clone(), tt.clone()
            _all_reduce(mx, dist.ReduceOp.MAX)
            _all_reduce(sm, dist.ReduceOp.SUM)
            tt = torch.stack([mx[0], sm[1], sm[2] / world])
        return (float(v) for v in tt)

    def sync():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()

    runs = []
    for Z in n_zones_list:
        r = setup(Z)
        runs.append(r)
        if burnin:
            launch(r, burnin, False)
        sync()
        t0 = time.perf_counter()
        res = launch(r, K, True)
        sync()
        wall_max, ess_tot, acc = reduce(time.perf_counter() - t0, [res])
        out["runs"][f"Z={Z}"] = {"chains": B * world, "steps": K, "burnin": burnin,
                                 "mh_steps_per_sec": B * K * world / wall_max,
                                 "ess_per_sec": ess_tot / wall_max, "us_per_step": wall_max / K * 1e6,
                                 "acceptance": acc, "wall_s": wall_max}
        if not concurrent:
            r["eng"].close()
    if concurrent and len(runs) > 1:
        seq_wall = sum(v["wall_s"] for v in out["runs"].values())
        streams = [torch.cuda.Stream(dev) for _ in runs]
        sync()
        t0 = time.perf_counter()
        res_list = []
        for r, s in zip(runs, streams):
            with torch.cuda.stream(s):
                res_list.append(launch(r, K, True))
        sync()
        wall_max, ess_tot, acc = reduce(time.perf_counter() - t0, res_list)
        n = len(runs)
        out["sweep_concurrent"] = {
            "zones": list(n_zones_list), "chains_per_run": B * world, "steps": K,
            "mh_steps_per_sec": n * B * K * world / wall_max, "ess_per_sec": ess_tot / wall_max,
            "wall_s": wall_max, "sequential_wall_s": seq_wall,
            "sequential_mh_steps_per_sec": n * B * K * world / seq_wall,
            "speedup_vs_sequential": seq_wall / wall_max, "acceptance": acc,
            "how": f"the {n} K runs (each continuing its chains after the per-K run) launched at once, "
                   f"one HIP stream each; sequential = the per-K runs' walls added"}
        for r in runs:
            r["eng"].close()
    return out


def _all_reduce(t, op):
    """all_reduce of a (device) tensor in place; over gloo (the CPU rehearsal backend) through a
    host copy."""
    import torch.distributed as dist
    if dist.get_backend() == "nccl":
        dist.all_reduce(t, op=op)
        return
    h = t.cpu()
    dist.all_reduce(h, op=op)
    t.copy_(h)


def source_lik_leg(args, eng, gen, dev, stream, rank, world):
    """The source branch of the likelihood (model.py:177-184) on the same
    workload: every cell's component drawn among those the site has, B chains, full evaluation
    with the sources by position as the sampler keeps them (lik_source_rc_kernel reads them in
    place; sbz_loglik_batch_device_pm), timed with HIP events on the engine's stream."""
    import copy
    import torch
    import torch.distributed as dist
    a = copy.copy(args)
    a.mode = "source"
    B, K = args.chains, args.source_lik_steps
    pool = [make_chains_torch(a, B, gen, dev, eng) for _ in range(2)]
    out = torch.empty(2, B, dtype=torch.float64, device=dev)

    def step(i):
        c = pool[i % 2]
        eng.loglik_device(B, c["zos"].data_ptr(), c["w"].data_ptr(), c["pg"].data_ptr(),
                          c["pz"].data_ptr(), c["pf"].data_ptr() if c["pf"] is not None else 0,
                          c["src_pm"].data_ptr(), out[i % 2].data_ptr(), validate=False, source_pm=True)
    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for i in range(K):
        step(i)
    ev1.record(stream)
    torch.cuda.synchronize()
    t = torch.tensor([ev0.elapsed_time(ev1) / 1e3], dtype=torch.float64, device=dev)
    if world > 1:
        _all_reduce(t, dist.ReduceOp.MAX)
    secs = float(t[0])
    P, D, per_launch = algorithmic_bytes(a, B, True)
    launch_s = secs / K
    # the by-site entry (the reference's Sample.source order, [B][N][F]): the same launches with
    # the sources by site, reordered by position on the device by the entry (source_to_pk_kernel:
    # 2-bit planes, the default; with src_pack = 0 one byte per cell, source_to_pm_kernel)
    c0 = pool[0]
    src_site = torch.empty(B, args.sites, args.features, dtype=torch.uint8, device=dev)
    eng.source_layout_device(B, c0["src_pm"].data_ptr(), src_site.data_ptr(), False)

    def step_site():
        eng.loglik_device(B, c0["zos"].data_ptr(), c0["w"].data_ptr(), c0["pg"].data_ptr(),
                          c0["pz"].data_ptr(), c0["pf"].data_ptr() if c0["pf"] is not None else 0,
                          src_site.data_ptr(), out[1].data_ptr(), validate=False, source_pm=False)
    step_site()
    torch.cuda.synchronize()
    ref = out[1].clone()
    step(0)
    torch.cuda.synchronize()
    if not torch.equal(out[0], ref):
        raise SystemExit("source branch: by-site and by-position launches disagree")

    def time_site():
        ev0.record(stream)
        for i in range(K):
            step_site()
        ev1.record(stream)
        torch.cuda.synchronize()
        t = torch.tensor([ev0.elapsed_time(ev1) / 1e3], dtype=torch.float64, device=dev)
        if world > 1:
            _all_reduce(t, dist.ReduceOp.MAX)
        return float(t[0]) / K, eng.last_kernels()
    site_launch_s, site_kernels = time_site()
    eng.set_option("src_pack", 0)
    step_site()
    torch.cuda.synchronize()
    if not torch.equal(out[1], ref):
        raise SystemExit("source branch: by-site launches with byte and 2-bit reorders disagree")
    byte_launch_s, byte_kernels = time_site()
    eng.set_option("src_pack", 1)
    del pool, src_site
    traffic, traffic_src = pmc_kernel_traffic(args, B, "lik_source_rc_kernel")
    return {"evals_per_sec": B * K * world / secs, "launch_us": launch_s * 1e6,
            "by_site": {"launch_us": site_launch_s * 1e6, "kernels": site_kernels,
                        "reorder_us_est": (site_launch_s - launch_s) * 1e6,
                        "byte_reorder": {"launch_us": byte_launch_s * 1e6, "kernels": byte_kernels,
                                         "reorder_us_est": (byte_launch_s - launch_s) * 1e6},
                        "how": "the same launches with the sources by site ([B][N][F], the reference's "
                               "order): sbz_loglik_batch_device reorders them by position first, into "
                               "2-bit planes (default) or bytes (src_pack = 0, 'byte_reorder'); "
                               "reorder_us_est = by-site launch - by-position launch; all three "
                               "launches give bit-identical values (checked)"},
            "bytes_per_eval": P + D / B, "bytes_per_launch": per_launch,
            "achieved_GBs": per_launch / launch_s / 1e9,
            "frac": per_launch / launch_s / 1e9 / HBM_PEAK_GBS, "steps": K,
            "traffic": traffic, "traffic_source": traffic_src,
            "traffic_over_algorithmic": traffic / per_launch if traffic else None,
            "kernels": eng.last_kernels()}


OTHER_CONFIGS = [
    # name, sites, features, states, zones, families, zone size, chains per GPU (BASELINE configs)
    ("cfg2_200x100x5_Z2", 200, 100, 5, 2, 0, 25, 64),
    ("cfg3_shape_28x47x3_Z3_Fam5", 28, 47, 3, 3, 5, 5, 256),
    ("cfg4_shape_100x36x5_Z6_Fam6", 100, 36, 5, 6, 6, 8, 128),
    ("cfg5_Fam0_2000x500x10_Z8", 2000, 500, 10, 8, 0, 50, 256),
]


def other_configs_leg(args, dev, stream, rank, world, local_rank):
    """Full-evaluation likelihood launches at the other BASELINE.json config shapes (synthetic data
    of those shapes; cfg5 also without families, C = 2, as SURVEY.md §8d asks).  The small shapes
    are a few microseconds of work per launch, so they measure launch latency, not HBM: those
    configs are carried by the sampler kernels, which update the log-likelihood incrementally
    inside one persistent launch (see sampler / sampler_real_data)."""
    import copy
    import numpy as np
    import torch
    import torch.distributed as dist
    from contact_zones_amd.likelihood import LikelihoodEngine
    K = args.other_steps
    res = {}
    for name, N, F, S, Z, Fam, zs, B in OTHER_CONFIGS:
        a = copy.copy(args)
        a.sites, a.features, a.states, a.zones, a.families, a.zone_size = N, F, S, Z, Fam, zs
        a.mode = "mixture"
        rng = np.random.default_rng(args.seed + 17)
        obs, fam = make_shared(a, rng)
        a._fam = fam
        eng = LikelihoodEngine(obs, fam, S, Z, Fam, Fam > 0, device=local_rank, options=OPTIONS)
        eng.set_stream(stream.cuda_stream)
        gen = torch.Generator(device=dev)
        gen.manual_seed(args.seed * 7919 + rank)
        pool = [make_chains_torch(a, B, gen, dev) for _ in range(2)]
        out = torch.empty(2, B, dtype=torch.float64, device=dev)

        def step(i):
            c = pool[i % 2]
            eng.loglik_device(B, c["zos"].data_ptr(), c["w"].data_ptr(), c["pg"].data_ptr(),
                              c["pz"].data_ptr(), c["pf"].data_ptr() if c["pf"] is not None else 0,
                              0, out[i % 2].data_ptr(), validate=False)
        for i in range(5):
            step(i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        for i in range(K):
            step(i)
        ev1.record(stream)
        torch.cuda.synchronize()
        if not torch.isfinite(out).all():
            raise SystemExit(f"non-finite log-likelihood in the {name} leg")
        t = torch.tensor([ev0.elapsed_time(ev1) / 1e3], dtype=torch.float64, device=dev)
        if world > 1:
            _all_reduce(t, dist.ReduceOp.MAX)
        secs = float(t[0])
        P, D, per_launch = algorithmic_bytes(a, B)
        launch_s = secs / K
        res[name] = {"chains_per_gpu": B, "evals_per_sec": B * K * world / secs,
                     "launch_us": launch_s * 1e6, "bytes_per_eval": P + D / B,
                     "frac": per_launch / launch_s / 1e9 / HBM_PEAK_GBS, "kernels": eng.last_kernels()}
        eng.close()
        del pool
    res["note"] = ("full-evaluation launches at these shapes are launch-latency bound (a few us of "
                   "work each); the configs themselves run on the sampler kernels (incremental ll)")
    return res


def reap_children():
    """End and reap every process this one started that is still alive (the CPU-baseline workers
    are waited for where they run; this is the check that nothing else was left behind).  Returns
    what it found: [{"pid", "name", "cmdline"}]."""
    try:
        import psutil
    except ImportError:  # pragma: no cover
        return []
    me = psutil.Process()
    kids = me.children(recursive=True)
    found = []
    for k in kids:
        try:
            found.append({"pid": k.pid, "name": k.name(), "cmdline": " ".join(k.cmdline())[:200]})
            k.terminate()
        except psutil.Error:
            pass
    _, alive = psutil.wait_procs(kids, timeout=5)
    for k in alive:
        try:
            k.kill()
        except psutil.Error:
            pass
    psutil.wait_procs(alive, timeout=5)
    return found


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def self_launch(n):
    """`bench.py --gpus N` started directly (no WORLD_SIZE): run the same command as N ranks under
    torch.distributed.run, one per GPU, as a child process (nothing here has touched the GPU), and
    exit with its status.  Rank 0 prints the JSON line."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    if len(sys.argv) == 3 and sys.argv[1] == "--cpu-worker":  # a CPU-baseline child (no GPU)
        spec = json.loads(sys.argv[2])
        print(json.dumps(CPU_WORKERS[spec["kind"]](spec["shape"], spec["seconds"], spec["seed"])), flush=True)
        return
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        raise SystemExit(self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    if args.launch_check:  # the launch path alone (CPU, gloo): ranks meet and report
        import torch
        import torch.distributed as dist
        if world > 1:
            dist.init_process_group("gloo")
        t = torch.tensor([float(rank), 1.0])
        if world > 1:
            dist.all_reduce(t)
            dist.destroy_process_group()
        if rank == 0:
            print(json.dumps({"launch_check": True, "world_size": world, "rank_sum": int(t[0]),
                              "ranks": int(t[1])}), flush=True)
        return

    import numpy as np
    import torch
    import torch.distributed as dist

    # one rank per GPU; a rehearsal with more ranks than GPUs (SBZ_DIST_BACKEND=gloo: RCCL
    # refuses two ranks on one device) shares the GPUs round-robin and is marked as such in the
    # line (n_gpus = the distinct devices, "rehearsal": true), never reported as N GPUs
    n_dev = max(1, torch.cuda.device_count())
    devices_used = min(world, n_dev)
    rehearsal = world > n_dev
    local_rank = local_rank % n_dev
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        backend = os.environ.get("SBZ_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from contact_zones_amd.likelihood import LikelihoodEngine

    rng = np.random.default_rng(args.seed)
    obs, fam = make_shared(args, rng)  # replicated on every rank (1 MB)
    args._fam = fam
    eng = LikelihoodEngine(obs, fam, args.states, args.zones, args.families, args.families > 0,
                           device=local_rank, options=OPTIONS)
    stream = torch.cuda.current_stream()
    eng.set_stream(stream.cuda_stream)

    B = args.chains
    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed * 1000003 + rank)  # chains differ per rank (global chain ids)
    pool = [make_chains_torch(args, B, gen, dev, eng) for _ in range(args.pool)]
    out = torch.empty(args.pool, B, dtype=torch.float64, device=dev)
    src_mode = args.mode == "source"

    def step(i):
        c = pool[i % args.pool]
        eng.loglik_device(B, c["zos"].data_ptr(), c["w"].data_ptr(), c["pg"].data_ptr(),
                          c["pz"].data_ptr(), c["pf"].data_ptr() if c["pf"] is not None else 0,
                          c["src_pm"].data_ptr() if src_mode else 0, out[i % args.pool].data_ptr(),
                          validate=False, source_pm=True)  # generated in range by make_chains_torch

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step(i)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ev_ms = ev0.elapsed_time(ev1)
    if not torch.isfinite(out).all() and not os.environ.get("SBZ_ALLOW_NONFINITE"):
        raise SystemExit("non-finite log-likelihood in bench")

    t = torch.tensor([wall, ev_ms / 1e3], dtype=torch.float64, device=dev)
    if world > 1:
        _all_reduce(t, dist.ReduceOp.MAX)
    wall_max, ev_max = float(t[0]), float(t[1])

    total_evals = B * args.steps * world
    value = total_evals / wall_max
    P, D, per_launch = algorithmic_bytes(args, B, src_mode)
    # roofline from the timed wall clock per step (max over ranks, = ms_per_step); the HIP-event
    # device time of the same launches is reported beside it under its own name
    step_s = wall_max / args.steps
    launch_s = ev_ms / 1e3 / args.steps  # this rank's device time per launch (HIP events)
    achieved = per_launch / step_s / 1e9

    traffic, traffic_src, traffic_note = pmc_traffic(args, B)
    secondary = pmc_secondary(args, B)
    src_leg = None
    if args.source_lik_steps > 0 and not src_mode:
        del pool
        torch.cuda.empty_cache()
        src_leg = source_lik_leg(args, eng, gen, dev, stream, rank, world)
    sampler = None
    if args.mh_steps > 0 and args.mode == "mixture" and args.families > 0:
        sampler = sampler_leg(args, eng, obs, fam, dev, rank, world, stream)
    sampler_src = None
    if args.src_sampler_steps > 0 and args.mode == "mixture" and args.families > 0:
        # the reference's default mode (SAMPLE_SOURCE = true, config/default_config.json:32) on the
        # same cfg5 shape and chains per GPU: sources in HBM, the feature-table passes
        shape = {k: getattr(args, k) for k in ("sites", "features", "states", "zones", "families")}
        sampler_src = source_sampler_leg(shape, B, args.src_sampler_steps, args.src_sampler_burnin, args.seed,
                                         rank, world, local_rank, gpu_init=True)
        if sampler_src is not None:
            sampler_src["pmc"] = pmc_source_sampler()
            try:  # the reference's own source-mode sampler, timed in the build container (it never
                # travels to the GPU box): a reported figure beside the leg, not a box measurement
                with open(os.path.join(ROOT, "profiles", "r05_cpu_reference_source_sampler.json")) as f:
                    r = json.load(f)
                sampler_src["reference_cpu_container"] = {
                    "steps_per_sec_per_core": r["reference_steps_per_sec_per_core"], "cores": 1,
                    "kind": "reference", "where": r["where"],
                    "source": "profiles/r05_cpu_reference_source_sampler.json"}
            except (OSError, ValueError, KeyError):
                pass
    other = None
    if args.other_steps > 0 and not src_mode:
        other = other_configs_leg(args, dev, stream, rank, world, local_rank)
    real = None
    if args.src_steps > 0:
        # configs[2] (Balkan, 3 zones, 256 chains) and configs[3] (South America, K = 1..6 zone
        # sweep, 128 chains per GPU = 512 over 4 GPUs) on the reference's own data
        real = {"cfg3_balkan": real_data_leg("balkan", [3], args.src_chains * 2, args.src_steps,
                                             args.src_burnin, args.seed, rank, world, local_rank),
                "cfg4_south_america": real_data_leg("south_america", [1, 2, 3, 4, 5, 6], args.src_chains,
                                                    args.src_steps, args.src_burnin, args.seed, rank,
                                                    world, local_rank, concurrent=True)}
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "likelihood-evals/s",
            "n_gpus": devices_used,
            **({"rehearsal": True, "ranks": world,
                "rehearsal_note": f"{world} ranks on {devices_used} GPU(s): a test of the N > 1 path, "
                                  f"not an N-GPU measurement"} if rehearsal else {}),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": f"cfg5 roofline run: {args.sites} sites x {args.features} features x "
                            f"{args.states} states, {args.zones} zones, {args.families} families, "
                            f"{B} chains/GPU, {args.mode} log-likelihood, full evaluation per chain",
                "chains_per_gpu": B,
                "global_chains": B * world,
                "mode": args.mode,
                "pool_batches": args.pool,
                "zone_size": args.zone_size,
                "workload_key": workload_key(args, B),
                "parallelism": (f"chains sharded over {world} ranks on {devices_used} GPU(s) (rehearsal)"
                                if rehearsal else f"chains sharded over {world} GPU(s)"),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "timing": "achieved = bytes_per_launch / ms_per_step (timed wall clock, max over ranks)",
                "traffic": traffic,
                "traffic_source": traffic_src,
                **({"traffic_note": traffic_note} if traffic_note else {}),
                "kernel_source_hash": kernel_source_hash(),
                "bytes_per_eval": P + D / B,
                "bytes_per_launch": per_launch,
                "step_us": step_s * 1e6,
                "launch_us_event": launch_s * 1e6,
                "frac_event": per_launch / launch_s / 1e9 / HBM_PEAK_GBS,
                **({"secondary": secondary} if secondary else {}),
            },
            "device_time_s": ev_max,
        }
        if src_leg is not None:
            line["likelihood_source_branch"] = src_leg
        if other is not None:
            line["likelihood_other_configs"] = other
        if sampler is not None:
            line["sampler"] = sampler
        if sampler_src is not None:
            line["sampler_source_mode"] = sampler_src
        if real is not None:
            line["sampler_real_data"] = real
        if world == 1 and args.cpu_seconds > 0:
            line["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
            line["speedup_vs_cpu"] = value / line["cpu_baseline"]["value"]
            if sampler is not None and args.cpu_sampler_seconds > 0:
                sampler["cpu_baseline"] = cpu_baseline_sampler(args, args.cpu_sampler_seconds)
                sampler["speedup_vs_cpu_steps"] = sampler["mh_steps_per_sec"] / sampler["cpu_baseline"]["value"]
            if sampler_src is not None and args.cpu_src_sampler_seconds > 0:
                sampler_src["cpu_baseline"] = cpu_baseline_src_sampler(args, args.cpu_src_sampler_seconds)
                sampler_src["speedup_vs_cpu_steps"] = (sampler_src["mh_steps_per_sec"] /
                                                       sampler_src["cpu_baseline"]["value"])
        line["processes_at_exit"] = reap_children()
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    left = reap_children()
    if left:
        print(f"bench: ended child processes at exit: {left}", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
