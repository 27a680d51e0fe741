"""Node-shared host rows for the children's genomes of a multi-rank generation.

Under torch.distributed every rank holds the whole population (the reference's DE loop is
replicated: population.py:62-87 runs on each rank with identical RNG draws), and every rank's
GPU DE step produces the same children.  The reference's Individual objects need those genomes
on the host, so each rank used to copy ALL children from its GPU: at BASELINE config 3
(1024 x 50k float64) 410 MB per rank per generation over its PCIe link, while the rank
evaluates only its 1/N shard.

Here the ranks of one node share a ring of host memory segments (files in /dev/shm, mapped by
every rank and page-locked once with tblup_host_register so device-to-host copies land as DMA).
Per generation the ranks agree on a free segment, each rank copies only ITS shard's rows of the
children into it, and after one barrier every rank's genomes are read-only views of the one
segment: 1/N of the transfer per rank and one host copy of the children per node instead of N.

A segment is free when no rank still holds a genome in it.  Liveness is per rank (weak
references to the segment's block array, whose rows the genomes are); the ranks' masks are
combined by one all-reduce (MAX) so every rank picks the same segment.  The page-locked-block
compaction of tblup_amd.evolver (_RowBlocks.compact) moves the last survivors out of old blocks,
which frees their segments for reuse.  When no segment is free, or the ranks span several nodes,
acquire() returns None and the caller copies the whole population as before.
"""
import mmap
import os
import weakref

import numpy as np

from .distributed import world


def _single_node(ws):
    lws = os.environ.get("LOCAL_WORLD_SIZE")
    return lws is not None and int(lws) == ws


class ShmRowRing:
    """Ring of node-shared segments per children shape (see the module docstring)."""

    def __init__(self, extra=3):
        self.extra = extra     # segments beyond the page-locked blocks _RowBlocks keeps alive
        self._rings = {}       # shape -> {"maps": [mmap], "views": [weakref|None], "next": int, "reg": [ptr]}
        self._token = None

    def _collective_device(self):
        import torch
        import torch.distributed as dist
        if dist.get_backend() == "nccl":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def _job_token(self):
        if self._token is None:
            import torch.distributed as dist
            obj = [os.urandom(8).hex() if dist.get_rank() == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            self._token = obj[0]
        return self._token

    def _make_ring(self, shape, nseg):
        """Rank 0 creates the segment files, every rank maps them, rank 0 unlinks them once all
        have mapped (the mappings stay valid; nothing is left in /dev/shm)."""
        import torch.distributed as dist
        rank = dist.get_rank()
        nbytes = int(np.prod(shape)) * 8
        token = self._job_token()
        paths = [f"/dev/shm/tblup-{token}-{shape[0]}x{shape[1]}-{i}" for i in range(nseg)]
        # room for the ring in /dev/shm (a small tmpfs would SIGBUS on the writes): rank 0 checks,
        # every rank follows its decision
        ok = [None]
        if rank == 0:
            try:
                st = os.statvfs("/dev/shm")
                ok[0] = st.f_bavail * st.f_frsize >= 2 * nseg * nbytes
            except OSError:
                ok[0] = False
            if ok[0]:
                for p in paths:
                    with open(p, "wb") as f:
                        f.truncate(nbytes)
        dist.broadcast_object_list(ok, src=0)
        if not ok[0]:
            return None
        dist.barrier()
        maps = []
        for p in paths:
            with open(p, "r+b") as f:
                maps.append(mmap.mmap(f.fileno(), nbytes))
        dist.barrier()
        if rank == 0:
            for p in paths:
                os.unlink(p)
        reg = []
        if _gpu_available():
            from . import _native
            lib = _native.load()
            for m in maps:
                ptr = np.frombuffer(m, dtype=np.uint8).ctypes.data
                _native.check("tblup_host_register", lib.tblup_host_register(ptr, nbytes))
                reg.append(ptr)
        return {"maps": maps, "views": [None] * nseg, "next": 0, "reg": reg}

    def acquire(self, shape, keep):
        """A writable (n, L) float64 block over a segment no rank uses any more, the same segment
        on every rank (one all-reduce); None when there is none (or not one node)."""
        import torch
        import torch.distributed as dist
        rank, ws = world()
        if ws == 1 or not _single_node(ws):
            return None
        shape = (int(shape[0]), int(shape[1]))
        if shape not in self._rings:
            self._rings[shape] = self._make_ring(shape, keep + self.extra)
        ring = self._rings[shape]
        if ring is None:   # no room in /dev/shm: every rank copies the whole population
            return None
        n = len(ring["maps"])
        alive = torch.tensor([1 if (w is not None and w() is not None) else 0 for w in ring["views"]],
                             dtype=torch.int32, device=self._collective_device())
        dist.all_reduce(alive, op=dist.ReduceOp.MAX)
        alive = alive.cpu().tolist()
        for k in range(n):
            i = (ring["next"] + k) % n
            if not alive[i]:
                blk = np.ndarray(shape, dtype=np.float64, buffer=ring["maps"][i])
                ring["views"][i] = weakref.ref(blk)
                ring["next"] = (i + 1) % n
                return blk
        return None

    def close(self):
        from . import _native
        for ring in self._rings.values():
            if ring is not None and ring["reg"]:
                lib = _native.load()
                for ptr in ring["reg"]:
                    lib.tblup_host_unregister(ptr)
        self._rings.clear()


def _gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except ImportError:   # pragma: no cover
        return False


RING = ShmRowRing()
