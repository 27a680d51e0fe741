"""Genotype panel start-up: the reference's float64 .npy read once, in bounded chunks, into the
int8 {0,1,2} layout the GPU context takes -- and under torch.distributed once per node.

The reference hands every worker process its own full float64 copy of the panel
(tblup/evaluator.py:188 `np.load(data_path)`, :215-216 one copy per worker).  At BASELINE config 4
(5000 x 600k) that is 24 GB per copy; validating it with whole-array temporaries and converting
it added 12 GB more per rank.  Here:

* `read_panel_int8` streams the .npy file's rows through one fixed-size buffer (plain reads, no
  memory map, so no file page stays mapped into the process), checks {0,1,2} and writes int8:
  peak host memory is the int8 panel plus one chunk;
* `load_panel` (torch.distributed, every rank on one node): the node's rank 0 writes that int8
  panel once into a /dev/shm segment, every other rank maps it read-only, the segment name is
  unlinked as soon as every rank holds its mapping -- one int8 copy per node instead of one
  float64 copy per rank.  Each rank's `tblup_ctx_create` then copies the
  mapped rows to its own GPU.  Ranks spread over several nodes, or a failure to create the
  segment, fall back to every rank reading the file itself (still streamed).  A failure on any
  rank is exchanged with the other ranks before anyone proceeds, so no rank is left waiting.
"""
import os

import numpy as np

from .distributed import allgather_fitness, world

CHUNK_BYTES = 64 << 20   # host buffer for the streamed float64 rows


def _check_convert(blk, out_rows):
    """{0,1,2} check of one block of rows and its int8 conversion into out_rows."""
    if blk.dtype == np.int8:
        if blk.size and (int(blk.min()) < 0 or int(blk.max()) > 2):
            raise ValueError("genotypes must take values in {0, 1, 2} for the MI355X evaluator")
        out_rows[...] = blk
        return
    ok = (blk == 0)
    ok |= (blk == 1)
    ok |= (blk == 2)
    if not ok.all():
        raise ValueError("genotypes must take values in {0, 1, 2} for the MI355X evaluator")
    out_rows[...] = blk   # exact: integral values in [0, 2]


def convert_rows(g, out=None, chunk_bytes=CHUNK_BYTES):
    """int8 copy of a 2-D {0,1,2} array (any dtype, in memory or memory-mapped), converted in
    blocks of rows so no full-size temporary exists; ValueError for anything else."""
    if g.ndim != 2:
        raise ValueError("genotype matrix must be 2-D (animals x SNPs)")
    n, p = g.shape
    out = np.empty((n, p), dtype=np.int8) if out is None else out
    rows = max(1, chunk_bytes // max(1, p * g.itemsize))
    for r0 in range(0, n, rows):
        _check_convert(np.asarray(g[r0:r0 + rows]), out[r0:r0 + rows])
    return out


def read_panel_int8(path, out=None, chunk_bytes=CHUNK_BYTES):
    """The .npy panel at `path` as int8 (validated), read in chunks of rows into `out` (a new
    array, or e.g. a node-shared memory map).  C-ordered .npy files are streamed with plain reads;
    anything else (.npz, Fortran order) goes through numpy's own loader, converted by rows."""
    with open(path, "rb") as f:
        hdr = _npy_header(f)
        if hdr is not None and not hdr[1] and len(hdr[0]) == 2 and not hdr[2].hasobject:
            (n, p), dtype = hdr[0], hdr[2]
            out = np.empty((n, p), dtype=np.int8) if out is None else out
            row_bytes = p * dtype.itemsize
            rows = max(1, chunk_bytes // max(1, row_bytes))
            buf = np.empty(rows * p, dtype=dtype)
            for r0 in range(0, n, rows):
                m = min(rows, n - r0)
                view = buf[:m * p]
                got = f.readinto(memoryview(view).cast("B"))
                if got != m * row_bytes:
                    raise ValueError(f"{path}: truncated .npy data")
                _check_convert(view.reshape(m, p), out[r0:r0 + m])
            return out
    data = np.load(path, mmap_mode="r") if str(path).endswith(".npy") else np.load(path)
    if isinstance(data, np.lib.npyio.NpzFile):
        raise ValueError(f"{path}: expected one array, found an .npz archive")
    g = np.asarray(data)
    if g.ndim != 2:
        raise ValueError("genotype matrix must be 2-D (animals x SNPs)")
    return convert_rows(g, out, chunk_bytes)


def _single_node(ws):
    lws = os.environ.get("LOCAL_WORLD_SIZE")
    return lws is None or int(lws) == ws


def _exchange(code, device=None):
    """Element-wise max of every rank's error code (0 = ok): every rank learns of a failure."""
    _, st = allgather_fitness(np.zeros(0), 0, device, status=(code,))
    return int(st[0])


def _segment_name():
    import torch.distributed as dist
    obj = [os.urandom(8).hex() if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return f"/dev/shm/tblup_panel_{obj[0]}.npy"


def _npy_header(f):
    """(shape, fortran_order, dtype) of an open .npy file positioned at its start, or None."""
    try:
        version = np.lib.format.read_magic(f)
        if version == (1, 0):
            return np.lib.format.read_array_header_1_0(f)
        if version == (2, 0):
            return np.lib.format.read_array_header_2_0(f)
    except ValueError:
        pass
    return None


def load_panel(path, device=None):
    """The int8 panel for this process's GPU context (see the module docstring).  Returns an
    ndarray (single process, several nodes, or the shared segment unavailable) or a read-only
    memory map of the node's one shared copy."""
    rank, ws = world()
    if ws == 1 or not _single_node(ws):
        return read_panel_int8(path)
    name = _segment_name()
    err, arr = None, None
    if rank == 0:
        try:
            with open(path, "rb") as f:
                hdr = _npy_header(f)
            if hdr is None or len(hdr[0]) != 2:
                raise OSError(f"{path}: not a 2-D .npy panel (every rank loads it itself)")
            seg = np.lib.format.open_memmap(name, mode="w+", dtype=np.int8, shape=tuple(hdr[0]))
            read_panel_int8(path, out=seg)
            seg.flush()
            arr = seg
        except ValueError as e:     # not {0,1,2}: the same error on every rank
            err = e
        except Exception as e:      # noqa: BLE001 -- no segment: every rank reads the file itself
            err = e
    code = 0 if err is None else (1 if isinstance(err, ValueError) else 2)
    code = _exchange(code, device)
    if code == 1:
        if rank == 0 and os.path.exists(name):
            os.unlink(name)
        if isinstance(err, ValueError):
            raise err
        raise ValueError("genotypes must take values in {0, 1, 2} for the MI355X evaluator (rank 0)")
    if code == 2:
        if rank == 0 and os.path.exists(name):
            os.unlink(name)
        return read_panel_int8(path)
    if rank != 0:
        try:
            arr = np.load(name, mmap_mode="r")
        except Exception as e:      # noqa: BLE001
            err = e
    code = _exchange(0 if err is None else 2, device)
    if rank == 0:
        os.unlink(name)    # every rank holds its mapping (or failed): the name is no longer needed
    if code:
        return read_panel_int8(path) if arr is None else arr
    return arr
