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


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                           "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra)
    return env


def _run(out, ranks, source, chains=None):
    settings = {"model": {"N_AREAS": 2, "SAMPLE_SOURCE": source},
                "mcmc": {"N_STEPS": 3000, "N_SAMPLES": 30, "N_CHAINS": 5,
                         "WARM_UP": {"N_WARM_UP_STEPS": 600, "N_WARM_UP_CHAINS": 7}},
                "results": {"RESULTS_PATH": str(out)}}
    args = ["-m", "contact_zones_amd", CFG, "--seed", "11", "--name", "x", "--set", json.dumps(settings)]
    if chains is not None:
        args += ["--chains", str(chains)]
    if ranks == 1:
        cmd = [sys.executable] + args
        env = _env()
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
               str(ranks), "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
        env = _env(SBZ_DIST_BACKEND="gloo")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
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
    at the end of the run (parallel.gather_rows) and written as results files of their own.  As 2
    ranks (two chains each) the files equal the 1-rank run's byte for byte, and chain 0's files
    equal a 1-chain run's (Philox streams keyed by the global chain id)."""
    one, two, single = tmp_path / "r1", tmp_path / "r2", tmp_path / "s"
    f1 = _run(one, 1, source, chains=4)
    f2 = _run(two, 2, source, chains=4)
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


def _rccl_worker():
    """Body of one RCCL rank (a script run under torch.distributed.run)."""
    return r"""
import os, torch, torch.distributed as dist, numpy as np
from contact_zones_amd.parallel import (all_reduce_sum, best_chain, broadcast_arrays,
                                        broadcast_seed, gather_rows, shard_range)
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
assert gather_rows(loc, 9).cpu()[:, 0].tolist() == list(range(9))
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
