"""Chain sharding does not change results.

The batched samplers shard the chains contiguously over the ranks and key every chain's Philox
stream by its GLOBAL chain id, so a run's warm-up winner (the arg-max over all chains,
mcmc_generative.py:195-200), the logged chain's trajectory (chain_idx[0] on rank 0, :205-218) and
the results files must not depend on the number of ranks.  These tests run the reference's Balkan
experiment config through `python -m contact_zones_amd` as 1 rank and as 2 ranks on the one GPU of
the box (both ranks on device 0; the collectives over gloo, since RCCL refuses two ranks on one
device) with the same seed, and compare the results files byte for byte.  A second test runs the
run-level collectives over RCCL with one rank per GPU; it needs >= 2 GPUs and skips on a one-GPU box
(the driver's 8-GPU node runs it)."""
import filecmp
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(ROOT, "tests", "golden", "io", "data", "experiments", "balkan", "config.json")
CFG_SA = os.path.join(ROOT, "tests", "golden", "io", "data", "experiments", "south_america", "config.json")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                           "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra)
    return env


def _run(out, ranks, source, chains=None, extra=(), cfg=CFG, n_areas=2):
    settings = {"model": {"N_AREAS": n_areas, "SAMPLE_SOURCE": source},
                "mcmc": {"N_STEPS": 3000, "N_SAMPLES": 30, "N_CHAINS": 5,
                         "WARM_UP": {"N_WARM_UP_STEPS": 600, "N_WARM_UP_CHAINS": 7}},
                "results": {"RESULTS_PATH": str(out)}}
    args = ["-m", "contact_zones_amd", cfg, "--seed", "11", "--name", "x", "--set", json.dumps(settings)]
    if chains is not None:
        args += ["--chains", str(chains)]
    args += list(extra)
    if ranks == 1:
        cmd = [sys.executable] + args
        env = _env()
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
               str(ranks), "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
        env = _env(SBZ_DIST_BACKEND="gloo")
    import time
    t0 = time.perf_counter()
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    _run.wall = time.perf_counter() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    files = sorted(os.path.relpath(os.path.join(d, f), out) for d, _, fs in os.walk(out) for f in fs)
    assert files, r.stderr[-2000:]
    return files


@pytest.mark.parametrize("source", [False, True])
def test_two_ranks_match_one_rank(gpu_available, tmp_path, source):
    one, two = tmp_path / "r1", tmp_path / "r2"
    f1 = _run(one, 1, source)
    f2 = _run(two, 2, source)
    assert f1 == f2
    for f in f1:
        assert filecmp.cmp(one / f, two / f, shallow=False), f"{f} differs between 1 and 2 ranks"


@pytest.mark.parametrize("source", [False, True])
def test_independent_chains_gathered_to_rank0(gpu_available, tmp_path, source):
    """--chains 4 (independent main-run chains, MC3 off): every chain's samples gathered to rank 0
    in windows as the run goes (mcmc.ChainLog, parallel.gather_to_root) and written as results files
    of their own (chains 1.. without parameters, chain 2's with: --chain-params 2).  As 2
    ranks (two chains each) the files equal the 1-rank run's byte for byte, and chain 0's files
    equal a 1-chain run's (Philox streams keyed by the global chain id)."""
    one, two, single = tmp_path / "r1", tmp_path / "r2", tmp_path / "s"
    # windows of 7 of the 30 logged samples (the last one partial); chain 2 logs its parameters
    extra = ["--chain-params", "2", "--log-window", "7"]
    f1 = _run(one, 1, source, chains=4, extra=extra)
    f2 = _run(two, 2, source, chains=4, extra=extra)
    assert f1 == f2
    for c in (1, 2, 3):
        assert any(f.endswith(f"_chain{c}.txt") and "stats_" in f for f in f1), f1
        assert any(f.endswith(f"_chain{c}.txt") and "areas_" in f for f in f1), f1
    for f in f1:
        assert filecmp.cmp(one / f, two / f, shallow=False), f"{f} differs between 1 and 2 ranks"
    fs = _run(single, 1, source)
    assert fs and all(f in f1 for f in fs)
    for f in fs:
        assert filecmp.cmp(one / f, single / f, shallow=False), f"{f}: chain 0 differs from a 1-chain run"
    # the chains are independent: their samples differ
    a = (one / [f for f in f1 if f.endswith("_chain1.txt") and "stats_" in f][0]).read_text()
    b = (one / [f for f in f1 if f.endswith("_chain2.txt") and "stats_" in f][0]).read_text()
    assert a != b
    # chain 1 without parameters: sample, posterior, likelihood, prior, sizes; chain 2 with them
    h1, h2 = a.splitlines()[0].split("\t"), b.splitlines()[0].split("\t")
    assert h1 == ["Sample", "posterior", "likelihood", "prior", "size_a0", "size_a1"], h1
    assert h2[:6] == h1 and any(c.startswith("w_universal_") for c in h2) and "post_a1" in h2
    assert len(a.splitlines()) == len(b.splitlines()) == 31


@pytest.mark.parametrize("source", [True])
def test_zone_sweep_jobs_concurrent_and_sharded(gpu_available, tmp_path, source):
    """The South America config's K = 1..6 zone sweep (BASELINE configs[3]) as one product run
    (VERDICT r5 item 4): the six (run, K) jobs one after another (--jobs sequential, the
    reference's cli.py:71-84 order), all at once on six HIP streams of one process (the default),
    and sharded over 2 ranks (jobs 0, 2, 4 on rank 0, 1, 3, 5 on rank 1; gloo, both on the one
    GPU): every results file byte-identical.  Prints the walls (process start to exit)."""
    seq, con, two = tmp_path / "seq", tmp_path / "con", tmp_path / "two"
    sweep = [1, 2, 3, 4, 5, 6]
    fs = _run(seq, 1, source, extra=["--jobs", "sequential"], cfg=CFG_SA, n_areas=sweep)
    w_seq = _run.wall
    fc = _run(con, 1, source, cfg=CFG_SA, n_areas=sweep)
    w_con = _run.wall
    f2 = _run(two, 2, source, extra=["--shard", "jobs"], cfg=CFG_SA, n_areas=sweep)
    w_two = _run.wall
    assert len([f for f in fs if os.path.basename(f).startswith("stats_n")]) == 6, fs
    assert fs == fc == f2
    for f in fs:
        assert filecmp.cmp(seq / f, con / f, shallow=False), f"{f}: concurrent differs from sequential"
        assert filecmp.cmp(seq / f, two / f, shallow=False), f"{f}: 2-rank job sharding differs"
    print(f"K = 1..6 sweep walls (process): sequential {w_seq:.1f} s, concurrent {w_con:.1f} s, "
          f"2 ranks x 3 jobs {w_two:.1f} s")


def _rccl_worker():
    """Body of one RCCL rank (a script run under torch.distributed.run)."""
    return r"""
import os, torch, torch.distributed as dist, numpy as np
from contact_zones_amd.parallel import (all_reduce_sum, best_chain, broadcast_arrays,
                                        broadcast_seed, gather_to_root, shard_range)
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(int(os.environ["LOCAL_RANK"]))
dist.init_process_group("nccl", device_id=torch.device("cuda", int(os.environ["LOCAL_RANK"])))
assert dist.get_backend() == "nccl"
assert broadcast_seed(99 if rank == 0 else 5) == 99
s = all_reduce_sum(torch.full((3,), rank + 1, dtype=torch.int64, device="cuda"))
assert s.tolist() == [world * (world + 1) // 2] * 3
post = np.arange(9, dtype=np.float64) % 4
lo, hi = shard_range(9, rank, world)
assert best_chain(post[lo:hi], lo) == (3, 3.0)
got = broadcast_arrays([np.arange(6.0).reshape(2, 3)] if rank == 1 else None, 1)
assert got[0].tolist() == np.arange(6.0).reshape(2, 3).tolist()
loc = torch.arange(lo, hi, dtype=torch.float64, device="cuda")[:, None].repeat(1, 4)
g = gather_to_root(loc, 9)
assert (g.cpu()[:, 0].tolist() == list(range(9))) if rank == 0 else g is None
dist.barrier()
dist.destroy_process_group()
print("RCCL_OK", rank)
"""


def test_rccl_two_ranks_run_level_collectives(gpu_available, tmp_path):
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs >= 2 GPUs (one RCCL rank per GPU); the driver's 8-GPU node runs it")
    body = tmp_path / "rccl_worker.py"
    body.write_text("import sys; sys.path.insert(0, %r)\n" % ROOT + _rccl_worker())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(body)]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.count("RCCL_OK") == 2


def _chainlog_memory_worker():
    """Body of one rank: an independent-chains run at the cfg5 shape (2000 sites x 500 features x
    10 states, 8 zones, 4 families; mixture operators) with every chain logged (mcmc.ChainLog),
    reporting this rank's window bytes and its peak device memory while sampling."""
    return r"""
import json, os, random, sys, types
import numpy as np, scipy.sparse as sp, torch
from scipy.spatial import Delaunay
from contact_zones_amd.experiment import init_distributed
from contact_zones_amd.mcmc import BatchedZoneMCMC
rank, dev = init_distributed()
import bench
N, F, S, Z, Fam, CH, NLOG, SPS = 2000, 500, 10, 8, 4, 64, 100, 10
rng = np.random.default_rng(5)
obs = rng.integers(0, S, size=(N, F))
fam = rng.integers(0, Fam, size=N)
feats = np.zeros((N, F, S), bool)
feats[np.arange(N)[:, None], np.arange(F)[None, :], obs] = True
indptr, indices = Delaunay(rng.random((N, 2))).vertex_neighbor_vertices
adj = sp.csr_matrix((np.ones(indices.size, int), indices, indptr), shape=(N, N))
data = types.SimpleNamespace(features=feats, states=np.ones((F, S), bool), network={"adj_mat": adj},
                             families=np.stack([fam == i for i in range(Fam)]))
model = types.SimpleNamespace(n_zones=Z, min_size=3, max_size=50, inheritance=True, sample_source=False)
smp = BatchedZoneMCMC(model=model, data=data, operators=bench.mh_operators(), n_chains=CH,
                      var_proposal=bench.MH_PRECISION, p_grow_connected=0.85, initial_size=5, seed=7,
                      rng=random.Random(3), log_all_chains=True)
peak = {}
orig = smp._advance
def advance(n):
    orig(n)
    if smp._chain_log is not None and "base" not in peak:
        torch.cuda.synchronize()
        peak["base"] = torch.cuda.memory_allocated()
        peak["window"] = smp._chain_log.window_bytes()
        peak["W"] = smp._chain_log.W
        torch.cuda.reset_peak_memory_stats()
smp._advance = advance
smp.generate_samples(NLOG * SPS, NLOG)
torch.cuda.synchronize()
peak["peak"] = torch.cuda.max_memory_allocated()
peak["rank"] = rank
if rank == 0:
    cs = smp.chain_statistics
    peak["chains"] = len(cs)
    peak["samples"] = sorted({len(c["sample_zones"]) for c in cs})
    peak["params_chain1"] = "sample_weights" in cs[1]
print("CHAINLOG " + json.dumps(peak), flush=True)
import torch.distributed as dist
dist.barrier()
dist.destroy_process_group()
"""


def test_chain_log_memory_cfg5_two_ranks(gpu_available, tmp_path):
    """The run-end gather sized for the north-star run: 64 chains x 100 logged
    samples at the cfg5 shape, as 2 gloo ranks on the one GPU.  Each rank holds one window of W
    samples on the device — B (N + 16) W bytes, no parameters (chain 0's come through `statistics`)
    — and its peak device memory while sampling stays within that window above the state (the
    bound: one more window for a partial window's contiguous copy, plus 16 MB for the launches'
    own outputs), where keeping every sample on the device would take 100 x 32 x 534 KB = 1.7 GB
    per rank.  Rank 0 ends with all 64 chains x 100 samples."""
    body = tmp_path / "chainlog_worker.py"
    body.write_text("import sys; sys.path.insert(0, %r)\n" % ROOT + _chainlog_memory_worker())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(body)]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(SBZ_DIST_BACKEND="gloo"), capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    rep = {d["rank"]: d for d in (json.loads(x.split(" ", 1)[1]) for x in r.stdout.splitlines()
                                  if x.startswith("CHAINLOG "))}
    assert set(rep) == {0, 1}
    for d in rep.values():
        B, N, W = 32, 2000, d["W"]
        assert d["window"] == B * W * (N + 16)
        assert d["peak"] - d["base"] <= d["window"] + (16 << 20), d
        print(f"rank {d['rank']}: window {W} samples = {d['window'] / 2**20:.1f} MiB, "
              f"peak above base {(d['peak'] - d['base']) / 2**20:.1f} MiB")
    assert rep[0]["chains"] == 64 and rep[0]["samples"] == [100] and not rep[0]["params_chain1"]
