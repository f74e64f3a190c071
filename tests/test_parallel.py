"""Chain sharding and the sampler's collectives, world_size 2 over gloo on the CPU (the same code
runs over RCCL on the GPU box; see contact_zones_amd/parallel.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from contact_zones_amd.parallel import (all_reduce_sum, best_chain, broadcast_arrays,
                                        broadcast_seed, gather_to_root, owner_of, shard_range)


def test_shard_range_covers_every_chain_once():
    for n in (0, 1, 5, 15, 256, 2048, 2049):
        for w in (1, 2, 3, 4, 8):
            seen = []
            for r in range(w):
                lo, hi = shard_range(n, r, w)
                assert 0 <= lo <= hi <= n
                assert hi - lo in (n // w, n // w + 1)
                seen += list(range(lo, hi))
                for c in range(lo, hi):
                    assert owner_of(c, n, w) == r
            assert seen == list(range(n))
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, results):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        out = {}
        out["seed"] = broadcast_seed(1234 if rank == 0 else 999)
        out["sum"] = all_reduce_sum(torch.tensor([[rank + 1, 10], [2, 3]], dtype=torch.int64)).tolist()
        # log posterior per global chain: 7 chains, max 5.0 at chains 2 and 5 (tie -> 2)
        post = np.array([1.0, -2.0, 5.0, 0.0, 3.0, 5.0, 4.0])
        lo, hi = shard_range(7, rank, world)
        out["best"] = best_chain(post[lo:hi], lo)
        # no chain on one rank: still participates
        lo0, hi0 = (0, 3) if rank == 0 else (3, 3)
        out["best_empty"] = best_chain(np.array([0.5, 2.0, -1.0])[lo0:hi0], lo0)
        owner = owner_of(5, 7, world)
        arrs = [np.arange(12, dtype=np.float64).reshape(3, 4), np.array([[True, False]]),
                np.zeros((0, 3))] if rank == owner else None
        got = broadcast_arrays(arrs, owner)
        out["bcast"] = [(a.dtype.str, a.shape, a.tolist()) for a in got]
        local = torch.arange(lo * 10, hi * 10, dtype=torch.float64).reshape(hi - lo, 10)
        g = gather_to_root(local, 7)
        out["gather"] = g.tolist() if g is not None else None
        # explicit row counts per rank (ChainLog's parameter chains): 1 row on rank 0, none on rank 1
        g = gather_to_root(torch.full((1 - rank, 2), 7.0), 1, sizes=[1, 0])
        out["gather_sizes"] = g.tolist() if g is not None else None
        results[rank] = out
    finally:
        dist.destroy_process_group()


def test_collectives_world_size_2():
    port = _free_port()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    with mp.Manager() as m:
        results = m.dict()
        mp.spawn(_worker, args=(2, port, results), nprocs=2, join=True)
        res = dict(results)
    for r in range(2):
        o = res[r]
        assert o["seed"] == 1234
        assert o["sum"] == [[3, 20], [4, 6]]
        assert o["best"] == (2, 5.0)
        assert o["best_empty"] == (1, 2.0)
        assert o["bcast"][0] == ("<f8", (3, 4), np.arange(12.0).reshape(3, 4).tolist())
        assert o["bcast"][1] == ("|b1", (1, 2), [[True, False]])
        assert o["bcast"][2][1] == (0, 3)
    # only rank 0 receives the gathered rows
    assert res[0]["gather"] == np.arange(70, dtype=np.float64).reshape(7, 10).tolist()
    assert res[1]["gather"] is None
    assert res[0]["gather_sizes"] == [[7.0, 7.0]] and res[1]["gather_sizes"] is None


def test_bench_self_launch_two_ranks():
    """`bench.py --gpus 2` without WORLD_SIZE starts its own two ranks (torch.distributed.run as
    a child process, no exec) and prints rank 0's line; --launch-check stops after the ranks met
    over gloo, so this runs on the CPU."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line == {"launch_check": True, "world_size": 2, "rank_sum": 1, "ranks": 2}


def test_bench_cpu_baseline_processes():
    """The CPU baseline runs one spawned single-threaded process per core and reports per-core and
    all-core rates, here on a small shape."""
    import argparse
    import bench
    args = argparse.Namespace(sites=200, features=40, states=5, zones=2, families=2, zone_size=20,
                              seed=3, cpu_procs=2)
    r = bench.cpu_baseline(args, 0.5)
    assert r["cores"] == 2 and r["kind"] == "port" and r["host_cpu_count"] == os.cpu_count()
    assert r["value"] > 0 and abs(r["per_core"] * 2 - r["value"]) < 1e-9 * r["value"]


def test_bench_cpu_sampler_baseline_processes():
    """The sampler's CPU baseline runs the restated MH step loop
    (oracle/mh_numpy.step) in one child process per core, all reaped when it returns, and reports
    measured steps/s per core and all-core, and the ESS of their traces."""
    import argparse
    import bench
    args = argparse.Namespace(sites=200, features=40, states=5, zones=2, families=2, zone_size=20,
                              seed=3, cpu_procs=2)
    r = bench.cpu_baseline_sampler(args, 0.5)
    assert r["cores"] == 2 and r["kind"] == "port" and r["unit"] == "MH steps/s"
    assert r["value"] > 0 and len(r["steps_per_process"]) == 2 and min(r["steps_per_process"]) > 0


def test_bench_cpu_source_sampler_baseline_processes():
    """The SAMPLE_SOURCE = true sampler's CPU baseline: the restated step loop
    with source resampling and the Gibbs operators drawing from their beta / Dirichlet
    distributions (oracle/mh_numpy, DrawTape) in one child process per core, all reaped when it
    returns: steps/s per core and all-core, the ESS of the traces, the container ratio to the
    reference."""
    import argparse
    import bench
    args = argparse.Namespace(sites=60, features=12, states=4, zones=2, families=2, zone_size=10,
                              seed=3, cpu_procs=2)
    r = bench.cpu_baseline_src_sampler(args, 0.5)
    assert r["cores"] == 2 and r["kind"] == "port" and r["unit"] == "MH steps/s"
    assert r["value"] > 0 and len(r["steps_per_process"]) == 2 and min(r["steps_per_process"]) > 0
    assert r["restatement_over_reference"] > 0


def test_bench_reaps_children():
    """bench.reap_children ends and reports any process the bench left behind:
    a sleeping child is found, terminated and reaped; a second call finds nothing.  (Inside the whole
    suite the test process may hold other children of earlier tests, e.g. a process pool's workers,
    which the first call ends too.)"""
    import subprocess
    import sys
    import bench
    p = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(60)"])
    found = bench.reap_children()
    assert p.pid in [d["pid"] for d in found]
    assert p.poll() is not None
    assert bench.reap_children() == []


def test_bench_source_sampler_pmc_needs_the_same_kernel_sources(tmp_path, monkeypatch):
    """The source-mode leg reports PMC counters per chain-step only from a committed profile measured
    on the current kernel sources (its _meta.source_hash); an older build's profile is named, not
    used."""
    import json
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    d = {"_meta": {"source_hash": "abc", "src_steps_total": 101, "src_chains": 256, "src_set": "default"},
         "_per_kernel": {"mh_src_kernel<3, true, 8, true>": {"dispatches": 2, "traffic_bytes": 101 * 256 * 1000.0,
                                                               "valu_insts_per_wave": 101 * 500.0}}}
    (prof / "r09_pmc_src.json").write_text(json.dumps(d))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "kernel_source_hash", lambda: "abc")
    r = bench.pmc_source_sampler()
    assert r["source"] == "profiles/r09_pmc_src.json"
    assert abs(r["hbm_bytes_per_chain_step"] - 2000.0) < 1e-9 and abs(r["valu_insts_per_wave_step"] - 1000.0) < 1e-9
    monkeypatch.setattr(bench, "kernel_source_hash", lambda: "other")
    r = bench.pmc_source_sampler()
    assert "source" not in r and "r09_pmc_src.json" in r["note"]


class _FakeSampler:
    """What ChainLog reads of a BatchedZoneMCMC: shapes, shard, state (CPU tensors here)."""

    def __init__(self, rank, world, n, N=11, F=3, S=4, Z=2, Fam=2):
        import types
        from contact_zones_amd.priors import PriorSpec
        self.n_chains, self.rank, self.world_size, self._group = n, rank, world, None
        self.lo, self.hi = shard_range(n, rank, world)
        self.n_sites, self.n_features, self.n_states, self.n_zones = N, F, S, Z
        self.inheritance, self.n_families = True, Fam
        self.priors, self.applicable_states = PriorSpec(), np.ones((F, S), bool)
        self.statistics = {"chain0": True}
        B = self.hi - self.lo
        self._state = types.SimpleNamespace(
            zone_of_site=torch.zeros((B, N), dtype=torch.uint8), ll=torch.zeros(B, dtype=torch.float64),
            prior=torch.zeros(B, dtype=torch.float64), w=torch.zeros((B, F, 3), dtype=torch.float64),
            p_global=torch.zeros((B, F, S), dtype=torch.float64),
            p_zones=torch.zeros((B, Z, F, S), dtype=torch.float64),
            p_fam=torch.zeros((B, Fam, F, S), dtype=torch.float64))

    def set_step(self, t):
        """Chain c's state at logging point t: recognisable values."""
        st = self._state
        for i, c in enumerate(range(self.lo, self.hi)):
            st.zone_of_site[i] = torch.tensor([(c + t + s) % 3 if (c + t + s) % 3 < 2 else 255
                                               for s in range(self.n_sites)], dtype=torch.uint8)
            st.ll[i] = -1000.0 * c - t
            st.prior[i] = -c - 0.5 * t
            st.w[i] = 100 * c + t
            st.p_global[i] = 100 * c + t + 0.25
            st.p_zones[i] = 100 * c + t + 0.5
            st.p_fam[i] = 100 * c + t + 0.75


def _chainlog_worker(rank, world, port, results):
    from contact_zones_amd.mcmc import ChainLog
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        smp = _FakeSampler(rank, world, 5)
        log = ChainLog(smp, 7, params=[2, 4], window=3)   # windows of 3, 3, 1 samples
        for t in range(7):
            smp.set_step(t)
            log.snap(10 + t)
        out = log.finish()
        results[rank] = None if out is None else [
            {k: (np.asarray(v).tolist() if k != "chain0" else v) for k, v in d.items() if k != "last_sample"}
            for d in out]
    finally:
        dist.destroy_process_group()


def test_chain_log_windows_gathered_to_rank0():
    """mcmc.ChainLog over 2 gloo ranks: every chain's zones, ll and carried prior at 7 logging
    points in windows of 3 (the last partial), parameters of chains 2 and 4 only; everything on
    rank 0, nothing on rank 1, each value the chain's own."""
    port = _free_port()
    with mp.Manager() as m:
        results = m.dict()
        mp.spawn(_chainlog_worker, args=(2, port, results), nprocs=2, join=True)
        res = dict(results)
    assert res[1] is None
    out = res[0]
    assert len(out) == 5 and out[0] == {"chain0": True}
    for c in range(1, 5):
        d = out[c]
        assert d["chain"] == c and d["sample_id"] == list(range(10, 17))
        assert d["sample_likelihood"] == [-1000.0 * c - t for t in range(7)]
        for t in range(7):
            zos = [(c + t + s) % 3 for s in range(11)]
            want = [[z == k for z in zos] for k in range(2)]
            assert d["sample_zones"][t] == want
        if c in (2, 4):
            assert d["sample_weights"] == [np.full((3, 3), 100.0 * c + t).tolist() for t in range(7)]
            assert d["sample_p_families"][6] == np.full((2, 3, 4), 100.0 * c + 6.75).tolist()
            assert d["sample_prior"] == [0.0] * 7   # zero priors, evaluated in full on the host
        else:
            assert "sample_weights" not in d
            assert d["sample_prior"] == [-c - 0.5 * t for t in range(7)]  # the carried prior
