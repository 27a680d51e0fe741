"""Population sharding across GPUs (one process per GPU) and the fitness all-gather.

The reference's only parallelism is a single-node worker pool fed through
mp.Queue (tblup/evaluator.py:120-131, 236-241, 397-398).  Here every rank holds
the whole genotype panel in its own HBM, evaluates a contiguous block of the
population, and one all-gather of the float64 fitnesses (backend "nccl" = RCCL
over xGMI on a GPU node, "gloo" on CPU) gives every rank the full vector, so the
host-side DE step stays identical on every rank.

Under `torchrun main.py` nothing in the reference creates a process group, so the
evaluator does (`init_from_env`, called from ParallelEvaluator.__enter__ -- the
place where the reference starts its workers, evaluator.py:120-131): it binds the
process to GPU LOCAL_RANK and creates the default group ("nccl" = RCCL when a GPU
is visible, else "gloo"; TBLUP_DIST_BACKEND overrides).  bench.py uses the same
two functions for its N > 1 path.
"""
import os

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


def init_from_env(device=None):
    """Create the default process group from the torchrun environment (RANK, WORLD_SIZE,
    MASTER_ADDR, MASTER_PORT, LOCAL_RANK) when WORLD_SIZE > 1 and no group exists yet.

    With the nccl backend the process is first bound to its GPU (`device`, else LOCAL_RANK)
    so RCCL sees one device per rank.  Returns True when this call created the group (the
    caller then owns it and destroys it), False otherwise."""
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return False
    import torch
    import torch.distributed as dist
    if not dist.is_available() or dist.is_initialized():
        return False
    backend = os.environ.get("TBLUP_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    kwargs = {}
    if backend == "nccl":
        local = int(os.environ.get("LOCAL_RANK", "0")) if device is None else int(device)
        torch.cuda.set_device(local)
        kwargs["device_id"] = torch.device("cuda", local)
    dist.init_process_group(backend, **kwargs)
    return True


def backend_name():
    """'RCCL' for the nccl backend on ROCm, else the backend's own name ('' without a group)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return ""
    b = dist.get_backend()
    return "RCCL" if b == "nccl" else b


def destroy():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def shard_range(n_items, rank, world_size):
    """Contiguous block [lo, hi) of n_items owned by `rank` (sizes differ by at most 1)."""
    base, rem = divmod(n_items, world_size)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def allgather_fitness(local, n_total, device=None, status=None):
    """All-gather the per-rank fitness blocks into the full float64 vector (rank order).

    `local` is this rank's shard_range block of n_total individuals: a vector, or an
    (rows, block) matrix -- IntraGCV's per-fold fitnesses -- gathered in ONE collective into
    (rows, n_total).  With nccl the buffers live on `device` (the evaluating engine's GPU; default
    the current device), so each rank hands RCCL its own GPU's memory.

    `status` (a short sequence of small non-negative ints, e.g. this rank's device status words
    or an error code) travels in the same collective, appended to the block; the call then returns
    (full, status_max), the elementwise maximum over the ranks -- so every rank sees a failure on
    any rank and they all take the same decision (raise, or fall back) together."""
    import torch
    import torch.distributed as dist

    rank, ws = world()
    loc = np.asarray(local, dtype=np.float64)
    st = None if status is None else np.asarray(status, dtype=np.float64).ravel()
    if ws == 1:
        return loc if st is None else (loc, st.astype(np.int64))
    rows = loc.shape[0] if loc.ndim == 2 else None
    loc2 = loc.reshape(rows or 1, -1)
    R = loc2.shape[0]
    sizes = [shard_range(n_total, r, ws) for r in range(ws)]
    maxc = max(hi - lo for lo, hi in sizes)
    S = 0 if st is None else len(st)
    W = maxc + S
    if dist.get_backend() == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else int(device))
    else:
        dev = torch.device("cpu")
    buf = torch.full((R, W), float("nan"), dtype=torch.float64, device=dev)
    if loc2.shape[1]:
        buf[:, :loc2.shape[1]] = torch.as_tensor(loc2, device=dev)
    if S:
        buf[0, maxc:] = torch.as_tensor(st, device=dev)
    out = torch.empty(ws * R * W, dtype=torch.float64, device=dev)
    allgather_device(out, buf.reshape(-1))
    out = out.cpu().numpy().reshape(ws, R, W)
    full = np.empty((R, n_total), dtype=np.float64)
    for r, (lo, hi) in enumerate(sizes):
        full[:, lo:hi] = out[r, :, :hi - lo]
    full = full if rows is not None else full[0]
    if st is None:
        return full
    return full, out[:, 0, maxc:].max(axis=0).astype(np.int64)


def allgather_device(out, local):
    """out (world * len(local),) <- every rank's `local` block in rank order: the one
    collective per generation (RCCL all-gather over xGMI under nccl)."""
    import torch.distributed as dist
    if dist.get_backend() == "gloo":
        dist.all_gather(list(out.chunk(dist.get_world_size())), local)
    else:
        dist.all_gather_into_tensor(out, local)
