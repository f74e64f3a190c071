"""Seed plumbing of the experiment runner (contact_zones_amd/experiment.py): every phase and
every (run, n_zones) job draws from its own stream, and all ranks agree on the experiment seed."""
import os
import socket

import torch.distributed as dist
import torch.multiprocessing as mp

from contact_zones_amd.experiment import agree_seed, derive_seeds


def test_phase_seeds_are_distinct_and_reproducible():
    seen = set()
    for run in range(3):
        for nz in (1, 2, 6):
            d = derive_seeds(7, run, nz)
            assert d == derive_seeds(7, run, nz)
            assert len(set(d.values())) == 3
            assert all(0 <= v < 2**63 for v in d.values())
            seen.update(d.values())
    assert len(seen) == 27
    assert derive_seeds(7, 0, 2) != derive_seeds(8, 0, 2)


def test_agree_seed_single_process():
    assert agree_seed(5) == 5
    a, b = agree_seed(None), agree_seed(None)
    assert a != b and 0 <= a < 2**63


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, results):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        # no --seed: rank 0 draws from OS entropy, every rank gets its value
        results[rank] = (agree_seed(None), agree_seed(100 + rank))
    finally:
        dist.destroy_process_group()


def test_agree_seed_world_size_2():
    with mp.Manager() as m:
        res = m.dict()
        mp.spawn(_worker, args=(2, _free_port(), res), nprocs=2, join=True)
        res = dict(res)
    assert res[0][0] == res[1][0]
    assert res[0][1] == res[1][1] == 100
