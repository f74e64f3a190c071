"""Chain sharding and the few collectives of the batched sampler (one process per GPU).

Chains are independent (the reference never couples them: MC3 off, mcmc_setup.py:103-114), so
the step loop has no collective.  What crosses ranks:
  * the Philox seed (rank 0's, broadcast once per run);
  * per-operator accept / proposal counters (sum, once per run);
  * the warm-up arg-max of (log posterior, chain id) (mcmc_generative.py:195-200) and the
    broadcast of the winning Sample from its owner;
  * the per-window gather of every chain's logged samples to rank 0 (gather_to_root; an
    independent-chains run, mcmc.ChainLog).
With the nccl backend (RCCL over xGMI on MI355X) tensors live on the rank's GPU; with gloo (the
CPU tests) on the host.
"""
import numpy as np


def _dist():
    try:
        import torch.distributed as dist
    except ImportError:  # pragma: no cover
        return None
    return dist if dist.is_available() and dist.is_initialized() else None


def shard_range(n, rank, world):
    """Contiguous balanced shard [lo, hi) of n chains for `rank` of `world`."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} of world {world}")
    base, rem = divmod(int(n), int(world))
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def owner_of(chain, n, world):
    """Rank that holds global chain `chain` under shard_range."""
    for r in range(world):
        lo, hi = shard_range(n, r, world)
        if lo <= chain < hi:
            return r
    raise ValueError(f"chain {chain} out of range({n})")


def _device(group=None):
    import torch
    d = _dist()
    if d is not None and d.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def broadcast_seed(seed, group=None):
    """Rank 0's seed on every rank."""
    d = _dist()
    if d is None or d.get_world_size(group) == 1:
        return int(seed)
    import torch
    t = torch.tensor([int(seed) & (2**63 - 1)], dtype=torch.int64, device=_device(group))
    d.broadcast(t, src=d.get_global_rank(group, 0) if group is not None else 0, group=group)
    return int(t.item())


def all_reduce_sum(t, group=None):
    """Sum of an integer / float tensor over ranks (returned on the tensor's own device)."""
    d = _dist()
    if d is None or d.get_world_size(group) == 1:
        return t
    dev = t.device
    x = t.to(_device(group)).contiguous()
    d.all_reduce(x, op=d.ReduceOp.SUM, group=group)
    return x.to(dev)


def best_chain(post_local, lo, group=None):
    """Global arg-max of the log posterior; ties go to the lowest chain id (list.index(max(...)))
    -> (chain, value)."""
    post_local = np.asarray(post_local, np.float64)
    if post_local.size:
        i = int(np.argmax(post_local))  # first maximum
        cand = (float(post_local[i]), lo + i)
    else:
        cand = (-np.inf, np.iinfo(np.int64).max)
    d = _dist()
    if d is None or d.get_world_size(group) == 1:
        return cand[1], cand[0]
    import torch
    w = d.get_world_size(group)
    mine = torch.tensor([cand[0], float(cand[1])], dtype=torch.float64, device=_device(group))
    out = [torch.empty_like(mine) for _ in range(w)]
    d.all_gather(out, mine, group=group)
    vals = [(float(o[0]), int(o[1])) for o in out]
    best_v = max(v for v, _ in vals)
    best_c = min(c for v, c in vals if v == best_v)
    return best_c, best_v


def broadcast_arrays(arrays, src, group=None):
    """numpy arrays from rank `src` to every rank (None on the other ranks on entry)."""
    d = _dist()
    if d is None or d.get_world_size(group) == 1:
        return arrays
    import torch
    dev = _device(group)
    rank = d.get_rank(group)
    gsrc = d.get_global_rank(group, src) if group is not None else src
    if rank == src:
        meta = [(a.dtype.str, a.shape) for a in arrays]
    else:
        meta = None
    box = [meta]
    d.broadcast_object_list(box, src=gsrc, group=group, device=dev)
    meta = box[0]
    out = []
    for i, (dt, shape) in enumerate(meta):
        nbytes = int(np.prod(shape)) * np.dtype(dt).itemsize
        if rank == src:
            buf = torch.from_numpy(np.ascontiguousarray(arrays[i]).view(np.uint8).reshape(-1).copy()).to(dev)
        else:
            buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        if nbytes:
            d.broadcast(buf, src=gsrc, group=group)
        out.append(buf.cpu().numpy().view(np.dtype(dt)).reshape(shape))
    return out


def gather_to_root(local, n_total, group=None, sizes=None):
    """Every rank's shard (first dim = that rank's chains under shard_range, or `sizes[r]` rows of
    rank r) concatenated into the full tensor on rank 0 (on the shard's device), None on the other
    ranks: one gather of equal-size padded shards (RCCL over xGMI with the nccl backend), so only
    rank 0 ever holds the whole."""
    d = _dist()
    if d is None or d.get_world_size(group) == 1:
        return local
    import torch
    w = d.get_world_size(group)
    rank = d.get_rank(group)
    dev = _device(group)
    if sizes is None:
        sizes = [hi - lo for lo, hi in (shard_range(n_total, r, w) for r in range(w))]
    m = max(max(sizes), 1)
    pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    pad[:local.shape[0]] = local.to(dev)
    dst = d.get_global_rank(group, 0) if group is not None else 0
    bufs = [torch.empty_like(pad) for _ in range(w)] if rank == 0 else None
    d.gather(pad, gather_list=bufs, dst=dst, group=group)
    if rank != 0:
        return None
    parts = [bufs[r][:n] for r, n in enumerate(sizes)]
    return torch.cat(parts, 0)  # (on the collective's device: rank 0 copies it to the host)
