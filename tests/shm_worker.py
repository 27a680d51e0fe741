"""Rank process of tests/test_shmrows.py (gloo, CPU)."""
import json
import os
import sys


def run(rank, world, port, out_dir):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world))
    import gc

    import numpy as np
    import torch.distributed as dist

    from tblup_amd.distributed import shard_range
    from tblup_amd.shmrows import ShmRowRing

    dist.init_process_group("gloo", rank=rank, world_size=world)
    ring = ShmRowRing(extra=1)
    shape = (10, 7)
    log = []
    held = []
    for gen in range(6):
        blk = ring.acquire(shape, keep=2)          # 3 segments
        if blk is None:
            log.append(None)
            continue
        lo, hi = shard_range(shape[0], rank, world)
        blk[lo:hi] = gen * 100 + np.arange(lo, hi)[:, None] + 0.5 * np.arange(shape[1])[None, :]
        dist.barrier()
        seg = [i for i, w in enumerate(ring._rings[shape]["views"]) if w is not None and w() is blk][0]
        want = gen * 100 + np.arange(shape[0])[:, None] + 0.5 * np.arange(shape[1])[None, :]
        log.append({"seg": seg, "ok": bool(np.array_equal(blk, want))})
        # rank 1 keeps generation 1's rows alive longer than rank 0: the segment must not be reused
        # until both have dropped it
        if gen == 1 and rank == 1:
            held.append(blk[3])
        if gen == 4:
            held.clear()
        del blk
        gc.collect()
    json.dump(log, open(os.path.join(out_dir, f"shm{rank}.json"), "w"))
    dist.barrier()
    dist.destroy_process_group()
