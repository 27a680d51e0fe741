"""Population sharding across GPUs (one process per GPU) and the fitness all-gather.

The reference's only parallelism is a single-node worker pool fed through
mp.Queue (tblup/evaluator.py:120-131, 236-241, 397-398).  Here every rank holds
the whole genotype panel in its own HBM, evaluates a contiguous block of the
population, and one all-gather of the float64 fitnesses (backend "nccl" = RCCL
over xGMI on a GPU node, "gloo" on CPU) gives every rank the full vector, so the
host-side DE step stays identical on every rank.
"""
import numpy as np


def world():
    """(rank, world_size) of the default process group, (0, 1) when not distributed."""
    try:
        import torch.distributed as dist
    except ImportError:  # pragma: no cover - torch is part of the image
        return 0, 1
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_range(n_items, rank, world_size):
    """Contiguous block [lo, hi) of n_items owned by `rank` (sizes differ by at most 1)."""
    base, rem = divmod(n_items, world_size)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def allgather_fitness(local, n_total):
    """All-gather the per-rank fitness blocks into the full float64 vector (rank order)."""
    import torch
    import torch.distributed as dist

    rank, ws = world()
    if ws == 1:
        return np.asarray(local, dtype=np.float64)
    sizes = [shard_range(n_total, r, ws) for r in range(ws)]
    maxc = max(hi - lo for lo, hi in sizes)
    backend = dist.get_backend()
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    buf = torch.full((maxc,), float("nan"), dtype=torch.float64, device=dev)
    if len(local):
        buf[:len(local)] = torch.as_tensor(np.asarray(local, dtype=np.float64), device=dev)
    out = [torch.empty_like(buf) for _ in range(ws)]
    dist.all_gather(out, buf)
    full = np.empty(n_total, dtype=np.float64)
    for r, (lo, hi) in enumerate(sizes):
        full[lo:hi] = out[r][:hi - lo].cpu().numpy()
    return full
