"""Drop-in DE evolvers whose generation step runs on the GPU.

Mirrors `tblup/evolver.py` for the two classic strategies:

* `DERandOneEvolver` (evolver.py:86-157): mutant = a + F (b - c)
* `DECurrentToBestOneEvolver` (evolver.py:160-244): mutant = x + F (best - x) + F (a - b),
  always clipped (the reference's `evolve` never passes `self.clip`, evolver.py:239-244)

with the reference's binary crossover (evolver.py:63-82) and F = 5 on every 5th
generation.  The per-individual python-`random` draws (the donors through
`exclusive_randrange`, utils.py:21-36, and the forced crossover position,
evolver.py:76) stay on the host in the reference's order; numpy's global MT19937
stream, which the reference consumes with one `np.random.rand(L)` per individual,
is jumped ahead on the GPU (k_de.hip, mt_jump.cpp) so every individual's
uniforms, mutant, crossover and clip are computed in parallel.  The children's
genomes and the numpy / python RNG states afterwards are bit-identical to the
reference's sequential loop (tests/test_evolver.py, tests/test_gpu_evolver.py).

The adaptive evolvers keep the reference's bookkeeping (AdaptiveEvolver, evolver.py:297-404) on
the host.  SaDE (evolver.py:407-547) runs its generation on the GPU too: every individual's
strategy (python's random.random() < p) and crossover rate are drawn on the host in the
reference's order and the step takes them per individual (tblup_de_step_device_async_mix; numpy's
stream still holds one np.random.rand(L) per individual).  MDE_pBX (evolver.py:550-687) draws
np.random.choice (rejection-sampled randint) between the individuals' np.random.rand(L) calls, so
each individual's numpy stream offset depends on the draws before it; it runs its DE step on the
host, as the reference does, with the reference's RNG consumption.
There is no CPU fallback for the GPU steps: without the HIP library, `evolve` raises ImportError.
"""
import abc
import csv
import ctypes
import os
import random
from copy import deepcopy
from math import ceil

import numpy as np

from . import _native
from .distributed import shard_range, world
from .keystore import DeviceKeyStore, TrackedGenome, freeze_heap, track, track_rows, work_stream
from .shmrows import RING as _SHM


def get_evolver(args):
    """evolver.py:13-32 for the strategies this package runs on the GPU."""
    if args.de_strategy == "de_rand_1":
        return DERandOneEvolver(args.dimensionality, args.crossover_rate, args.mutation_intensity, args.clip)
    if args.de_strategy == "de_currenttobest_1":
        return DECurrentToBestOneEvolver(args.dimensionality, args.crossover_rate, args.mutation_intensity, args.clip)
    if args.de_strategy == "sade":
        return SaDE(args.dimensionality, args.clip)
    if args.de_strategy == "mde_pbx":
        return MDE_pBX(args.dimensionality, args.generations, args.clip)
    raise NotImplementedError("Evolver with config option {} is not implemented.".format(args.de_strategy))


def exclusive_randrange(begin, end, exclude):
    """utils.py:21-36, same python-`random` consumption (first draw before the assert)."""
    r = random.randrange(begin, end)
    exclude = set(exclude)
    assert len(exclude) < (end - begin), "Exclusion range larger than random range."
    while r in exclude:
        r = random.randrange(begin, end)
    return r


def _native_donors(strategy, n, L, best=-1):
    """One generation's donor / fixed-position draws (the python loops of _donors below) on
    CPython's MT19937 state in native code (tblup_de_donors): the same draws and the same
    `random` state afterwards, without 4n interpreted randrange calls.  None when the loop must
    stay in python (n < 4 raises the reference's assertion there; n > 65535 or L >= 2^32)."""
    if n < 4 or n > 65535 or L >= 1 << 32:
        return None
    version, internal, gauss = random.getstate()
    mt = np.array(internal[:624], dtype=np.uint32)
    idx = np.array([internal[624]], dtype=np.int32)
    donors = np.empty((n, 3), dtype=np.int32)
    fixed = np.empty(n, dtype=np.int64)
    lib = _native.load()
    _native.check("tblup_de_donors", lib.tblup_de_donors(
        strategy, n, L, best, mt.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
        idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), donors.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
        fixed.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
    random.setstate((version, tuple(mt.tolist()) + (int(idx[0]),), gauss))
    return donors, fixed


class GpuDEStep:
    """A panel-less GPU context running tblup_de_step (one per process and device)."""

    _instances = {}

    @classmethod
    def get(cls, device=None):
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        inst = cls._instances.get(device)
        if inst is None:
            inst = cls._instances[device] = cls(device)
        return inst

    def __init__(self, device=0):
        self._lib = _native.load()
        freeze_heap()
        ctx = ctypes.c_void_p()
        _native.check("tblup_ctx_create", self._lib.tblup_ctx_create(None, 0, 0, 0, None, int(device),
                                                                     ctypes.byref(ctx)))
        self._ctx = ctx
        self.device = int(device)

    def _rng_state(self):
        st = np.random.get_state()
        if st[0] != "MT19937":
            raise RuntimeError("numpy's global RandomState is not MT19937")
        return st, np.array(st[1], dtype=np.uint32), ctypes.c_int32(int(st[2]))

    def step(self, strategy, parents, donors, fixed, F, cr, clip, clip_hi):
        """children (pop x L) for the current numpy global state, which is advanced
        past the generation's pop x L uniforms exactly as the reference's loop does."""
        parents = np.ascontiguousarray(parents, dtype=np.float64)
        pop, L = parents.shape
        donors = np.ascontiguousarray(donors, dtype=np.int32)
        fixed = np.ascontiguousarray(fixed, dtype=np.int64)
        st, key, pos = self._rng_state()
        children = np.empty_like(parents)
        _native.check("tblup_de_step", self._lib.tblup_de_step(
            self._ctx, int(strategy), parents.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), pop, L,
            donors.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), fixed.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
            float(F), float(cr), 1 if clip else 0, float(clip_hi),
            key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(pos),
            children.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
        np.random.set_state(("MT19937", key, pos.value, st[3], st[4]))
        return children

    def step_device(self, strategy, parents, donors, fixed, F, cr, clip, clip_hi, defer=False):
        """Same on a device tensor of parents (pop x L float64, on this device); returns the
        children as a device tensor.  Runs on torch's current stream.  defer: return
        (children, finish) without waiting for the step; finish() waits for the new MT state
        only (tblup_de_state_wait) and hands it to numpy -- call it before numpy's global RNG is
        used again.  strategy / F / cr: scalars, or one per individual (SaDE)."""
        import torch
        pop, L = parents.shape
        donors = np.ascontiguousarray(donors, dtype=np.int32)
        fixed = np.ascontiguousarray(fixed, dtype=np.int64)
        cur = torch.cuda.current_stream(parents.device)
        ws = work_stream(self.device)
        ws.wait_stream(cur)   # parents may come from work queued on the caller's stream
        with torch.cuda.stream(ws):
            children = torch.empty_like(parents)
        st, key, pos = self._rng_state()
        stream = ws.cuda_stream
        if np.ndim(strategy) or np.ndim(F) or np.ndim(cr):
            strat_i = np.ascontiguousarray(np.broadcast_to(strategy, (pop,)), dtype=np.int32)
            F_i = np.ascontiguousarray(np.broadcast_to(F, (pop,)), dtype=np.float64)
            cr_i = np.ascontiguousarray(np.broadcast_to(cr, (pop,)), dtype=np.float64)
            _native.check("tblup_de_step_device_async_mix", self._lib.tblup_de_step_device_async_mix(
                self._ctx, strat_i.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                F_i.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), cr_i.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                ctypes.c_void_p(parents.data_ptr()), pop, L, parents.stride(0),
                donors.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                fixed.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), 1 if clip else 0, float(clip_hi),
                key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), pos.value,
                ctypes.c_void_p(children.data_ptr()), children.stride(0), ctypes.c_void_p(stream)))
        else:
            _native.check("tblup_de_step_device_async", self._lib.tblup_de_step_device_async(
                self._ctx, int(strategy), ctypes.c_void_p(parents.data_ptr()), pop, L, parents.stride(0),
                donors.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                fixed.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), float(F), float(cr), 1 if clip else 0,
                float(clip_hi), key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), pos.value,
                ctypes.c_void_p(children.data_ptr()), children.stride(0), ctypes.c_void_p(stream)))
        cur.wait_stream(ws)   # later caller work on the children is ordered behind the step

        def finish():
            _native.check("tblup_de_state_wait", self._lib.tblup_de_state_wait(
                self._ctx, key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(pos)))
            np.random.set_state(("MT19937", key, pos.value, st[3], st[4]))

        if defer:
            return children, finish
        finish()
        return children

    def gather_rows(self, out, ptrs):
        """out[i] = the device row at address ptrs[i] (this device), on torch's current stream."""
        import torch
        n, L = out.shape
        tab = np.array(ptrs, dtype=np.uint64)   # host array of n device addresses (one C conversion)
        _native.check("tblup_gather_rows", self._lib.tblup_gather_rows(
            self._ctx, ctypes.c_void_p(out.data_ptr()), n, L, out.stride(0), ctypes.c_void_p(tab.ctypes.data),
            ctypes.c_void_p(torch.cuda.current_stream(out.device).cuda_stream)))

    def close(self):
        if self._ctx:
            self._lib.tblup_ctx_destroy(self._ctx)
            self._ctx = None
            GpuDEStep._instances.pop(self.device, None)


_F64 = np.dtype(np.float64)


def _child_dtypes(genomes, donors, strategy, mi, clip):
    """Per-child dtype numpy gives the reference: np.where(mask, mutant, target) (+ np.clip);
    None when every child is float64 (the usual RandomKey case)."""
    dts = [g.dtype if isinstance(g, np.ndarray) else np.asarray(g).dtype for g in genomes]
    f64 = _F64
    if all(dt is f64 or dt == f64 for dt in dts):
        return None
    out = []
    e = np.zeros(0, dtype=bool)
    for i, (x, y, z) in enumerate(donors):
        t, a, b, c = (np.zeros(0, dtype=dts[j]) for j in (i, x, y, z))
        st = strategy[i] if np.ndim(strategy) else strategy
        m = mi[i] if np.ndim(mi) else mi
        mutant = a + m * (b - c) if st == 0 else t + m * (a - t) + m * (b - c)
        r = np.where(e, mutant, t)
        out.append((np.clip(r, 0, 1) if clip else r).dtype)
    return out


_POOL = None


def _pool(workers=8):
    global _POOL
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        _POOL = ThreadPoolExecutor(workers, thread_name_prefix="tblup-copy")
    return _POOL


def _copy_rows(host, dtypes, workers=8, ready=None, dest=None):
    """An own array per child: float64 rows as TrackedGenome views (the key store mirrors
    them on the device and must notice in-place writes), other dtypes as plain arrays.
    ready: per-chunk callables that block until that chunk of `host` has arrived (the
    device-to-host copy is chunked so the row copies of chunk c overlap the transfer of
    chunk c + 1).  dest: preallocated float64 rows to copy into (dtypes None).  (Splitting
    each chunk over all workers measured slower: 4.3 vs 3.0 ms at config 2.)"""
    n = host.shape[0]
    nchunk = workers if ready is None else len(ready)
    step = (n + nchunk - 1) // nchunk

    def chunk(c):
        lo, hi = c * step, min(n, (c + 1) * step)
        if ready is not None:
            ready[c]()
        if dtypes is None and dest is not None:
            for i in range(lo, hi):
                np.copyto(dest[i], host[i])
            return [track(dest[i]) for i in range(lo, hi)]
        if dtypes is None:
            return [track(np.array(host[i])) for i in range(lo, hi)]
        return [np.array(host[i], dtype=dtypes[i]) for i in range(lo, hi)]
    if ready is None and n * host.shape[1] < (1 << 20):
        return [a for c in range(nchunk) for a in chunk(c)]
    parts = _pool(workers).map(chunk, range(nchunk))
    return [a for part in parts for a in part]


_NO_GENOME = np.empty(0)

# diagnostics (tools/generation_bench.py): when a dict, evolve() adds its segment times (s)
PROFILE = None


def _mark(t0, name):
    import time
    t = time.perf_counter()
    if PROFILE is not None:
        PROFILE[name] = PROFILE.get(name, 0.0) + t - t0
    return t


class _RowBlocks:
    """Page-locked blocks (one per generation) whose rows are children's genomes.

    A row is a view, so a block stays allocated while any genome in it lives (the reference
    gives every child its own array, individual.py:110-118; a view is one as far as any
    reader can tell: disjoint rows, float64, written through the TrackedGenome paths).  DE selection leaves survivors spread
    over older blocks: when more than `keep` older blocks are still referenced by the
    population, the least-referenced ones are compacted -- those individuals' genomes are
    replaced by equal own copies (set_internal_genome, individual.py:100-101) -- so at most
    keep + 2 generations (about 2 GiB) stay page-locked.  The copies run on worker threads
    while the next generation's GPU work and transfers are in flight, and the genomes are
    swapped to them at the next compaction (an own array each: they are never DMA'd again,
    their device rows stay in the key store).  Freed blocks go back to torch's caching host
    allocator and are reused without new page-locking."""

    def __init__(self, keep=12):
        self.keep = keep
        self._reg = {}   # id(block) -> weakref(block)
        self._reserved = set()
        self._pending = []   # (individual, its genome when the copy started, future of the copy)

    def keep_for(self, nbytes):
        """Older blocks kept page-locked for blocks of nbytes (about 2 GiB in all)."""
        return max(1, min(self.keep, (2 << 30) // max(nbytes, 1)))

    def reserve(self, shape):
        """Pre-size torch's caching host allocator for blocks of `shape`: the steady state holds
        keep_for + 2 blocks at once (the kept older ones, the current population's, the one being
        filled), so page-lock that many once, on the first generation -- otherwise every
        generation until the pool is full pins a fresh block (~10 ms per 100 MB).  Synchronously:
        page-locking from a background thread (round 4) contended with the generation's own HIP
        calls and made generations 2-12 slower (18 ms vs 12 ms at config 2) than pinning them
        one by one."""
        key = tuple(int(x) for x in shape)
        if key in self._reserved:
            return
        self._reserved.add(key)
        import torch
        n = self.keep_for(8 * int(np.prod(key))) + 2
        bufs = [torch.empty(key, dtype=torch.float64, pin_memory=True) for _ in range(n)]
        del bufs   # back to the caching allocator, page-locked

    def rows(self, block):
        import weakref
        self._reg[id(block)] = weakref.ref(block)
        rows = track_rows(block)
        block.flags.writeable = False   # the rows' private aliases are the only writable ones
        return rows

    def _block_of(self, g):
        b = g._blk if type(g) is TrackedGenome else None   # set by track_rows: no base walk
        if b is not None:
            r = self._reg.get(id(b))
            if r is not None and r() is b:
                return b
        b = g
        while isinstance(b, np.ndarray):
            r = self._reg.get(id(b))
            if r is not None and r() is b:
                return b
            b = b.base
        return None

    def finish(self, store=None):
        """Swap the members whose copies the last compaction started to those copies: skipped
        for a genome replaced or written (TrackedGenome marks it stale) since the copy began --
        it stays where it is and a later compaction takes it."""
        pending, self._pending = self._pending, []
        for indv, old, fut in pending:
            new = fut.result()
            if getattr(indv, "_genome", None) is not old or old._stale:
                continue
            t = track(new)
            indv.set_internal_genome(t)
            if store is not None:
                store.rebind(indv, old, t)

    def compact(self, individuals, store=None):
        """Blocks that only a few members of the population still use (<= n / 64 rows), and
        the least-used ones beyond `keep`: those members' genomes are copied into own arrays on
        worker threads (np.copyto releases the GIL; the copies overlap the next generation's
        transfers) and swapped by the next call (finish); the key store keeps their device rows.
        (Round 4 copied them here, on the caller's thread, into page-locked buffers: 2-12 ms per
        generation at pop 1024.)"""
        self.finish(store)
        self._reg = {k: r for k, r in self._reg.items() if r() is not None}
        if not self._reg:
            return
        users = {}
        for indv in individuals:
            g = getattr(indv, "_genome", None)
            blk = self._block_of(g) if isinstance(g, np.ndarray) else None
            if blk is not None:
                users.setdefault(id(blk), []).append(indv)
        order = sorted(users, key=lambda k: len(users[k]))
        few = max(1, len(individuals) // 64)
        # at most `keep` older blocks, fewer when they are large (about 2 GiB page-locked)
        big = max(r().nbytes for r in self._reg.values())
        keep = self.keep_for(big) - 1   # the blocks dropped here are released at the next call (finish)
        drop = [k for i, k in enumerate(order) if len(users[k]) <= few or i < len(order) - keep]
        if not drop:
            return
        moved = [indv for k in drop for indv in users[k]
                 if indv.get_internal_genome() is indv._genome]   # RandomKey / Index semantics only
        pool = _pool()
        # runs of rows per job: few pool round trips, each copy large enough to release the GIL
        per = max(1, (len(moved) + 7) // 8)
        for j0 in range(0, len(moved), per):
            grp = moved[j0:j0 + per]
            fut = pool.submit(_copy_genomes, [indv._genome for indv in grp])
            for j, indv in enumerate(grp):
                self._pending.append((indv, indv._genome, _Part(fut, j)))


def _copy_genomes(genomes):
    return [np.array(g.view(np.ndarray)) for g in genomes]


class _Part:
    """Item j of a future's list result."""

    def __init__(self, fut, j):
        self.fut, self.j = fut, j

    def result(self):
        return self.fut.result()[self.j]


def _assigns_genome(indv):
    """Whether set_internal_genome only stores the array (IndexIndividual's, individual.py:100-101,
    inherited by RandomKey / Nullable): then a child may be bound to its row before the row's
    transfer has landed.  CoevolutionIndividual's reads the last element (individual.py:194-208)."""
    f = getattr(type(indv), "set_internal_genome", None)
    return getattr(f, "__qualname__", "") == "IndexIndividual.set_internal_genome"


_BLOCKS = _RowBlocks()

# a generation's float64 children up to this many bytes cross as one page-locked block
_BLOCK_MAX = int(os.environ.get("TBLUP_BLOCK_ROWS_MB", "1024")) << 20

# children of a generation up to this many bytes get page-locked genome buffers
_PINNED_ROWS_MAX = int(os.environ.get("TBLUP_PINNED_ROWS_MB", "2048")) << 20


_DC_INDEX = {}


def _deepcopy_is_index(dc):
    """Whether `dc` is IndexIndividual.__deepcopy__ (the reference's, individual.py:110-118)."""
    hit = _DC_INDEX.get(dc)
    if hit is None:
        hit = _DC_INDEX[dc] = getattr(dc, "__qualname__", "") == "IndexIndividual.__deepcopy__"
    return hit


def _copy_individual(indv):
    """deepcopy(indv) as the reference's evolvers take it (evolver.py:130, 208), without
    copying the internal genome the caller replaces right after (set_internal_genome):
    the reference's IndexIndividual.__deepcopy__ (individual.py:110-118) deep-copies
    `_genome`, a 400 KB array per child at L = 50k."""
    g = getattr(indv, "_genome", None)
    if not isinstance(g, np.ndarray):
        return deepcopy(indv)
    # the class's own __deepcopy__ (individual.py:43-59, 110-118) called directly: copy.deepcopy's
    # dispatch and throwaway memo bookkeeping cost a third of the time for the same object
    dc = getattr(type(indv), "__deepcopy__", None)
    # IndexIndividual.__deepcopy__ (individual.py:110-118) only deep-copies the placeholder: None is
    # an atomic for copy.deepcopy (returned as is), where an empty array's deepcopy took ~half the
    # copy's time; other classes' __deepcopy__ may read the genome, so they get an empty array
    indv._genome = None if _deepcopy_is_index(dc) else _NO_GENOME
    try:
        return dc(indv, {}) if dc is not None else deepcopy(indv)
    finally:
        indv._genome = g


def _members(population):
    """The population's individuals and their internal genomes, one pass, and the common genome
    length (DE needs one: numpy broadcasting in evolver.py:132)."""
    inds = [population[i] for i in range(len(population))]
    genomes = [x.get_internal_genome() for x in inds]
    L = len(genomes[0]) if genomes else 0
    if any(len(g) != L for g in genomes):
        raise ValueError("DE needs internal genomes of one length (numpy broadcasting in evolver.py:132)")
    return inds, genomes, L


def _common_length(population):
    return _members(population)[2]


class Evolver(abc.ABC):
    """evolver.py:35-44."""

    @abc.abstractmethod
    def evolve(self, population):
        raise NotImplementedError()


class _GpuDEEvolver(Evolver):
    strategy = None
    device = None

    def __init__(self, dimensionality, crossover_rate, mutation_intensity, clip=True):
        self.dimensionality = dimensionality
        self.crossover_rate = crossover_rate
        self.mutation_intensity = mutation_intensity
        self.clip = clip

    def _donors(self, population, L):
        raise NotImplementedError()

    def _clip(self):
        return self.clip

    def evolve(self, population):
        import time
        t = time.perf_counter()
        mi = 5 if population.generation % 5 == 0 else self.mutation_intensity
        members = _members(population)
        donors, fixed = self._donors(population, members[2])
        return self._gpu_generation(population, t, donors, fixed, self.strategy, mi, self.crossover_rate,
                                    self._clip(), members)

    def _gpu_generation(self, population, t, donors, fixed, strategy, mi, cr, clip, members=None):
        """The children of one generation (donors / fixed: the python-`random` draws already made;
        strategy, mi, cr: scalars or one per individual; members: _members(population) when the
        caller has it) through the GPU DE step."""
        import torch
        inds, genomes, L = members if members is not None else _members(population)
        n = len(inds)
        t = _mark(t, "ev_donors")
        step = GpuDEStep.get(self.device)
        store = DeviceKeyStore.get(step.device)
        with torch.cuda.device(step.device), torch.cuda.stream(work_stream(step.device)):
            parents = store.gather(inds, L, host_rows=lambda i: genomes[i],
                                   copy_rows=step.gather_rows)   # device-resident parents
            t = _mark(t, "ev_gather")
            children, rng_done = step.step_device(strategy, parents, donors, fixed, mi, cr, clip,
                                                  self.dimensionality - 1, defer=True)
            t = _mark(t, "ev_prepare_step")
            try:
                # the children's numpy dtypes (None: all float64), while the step runs
                dtypes = _child_dtypes(genomes, donors, strategy, mi, clip)
                # the population's evaluator (tblup_amd) may start evaluating the children on the GPU
                # now, while their genomes cross to the host (BlupParallelEvaluator._speculate)
                evaluator = getattr(population, "evaluator", None)
                spec = getattr(evaluator, "_speculate", None)
                speculated = bool(spec is not None and dtypes is None and spec(inds, children, population.generation))
                t = _mark(t, "ev_speculate")
                # float64 children: one DMA into a page-locked block whose rows become the children's
                # genomes (views: no host copy); otherwise chunks, each followed by an event, so the
                # per-row copies of one chunk overlap the transfer of the next
                block_rows = dtypes is None and n * L * 8 <= _BLOCK_MAX
                # several ranks of one node: a node-shared block, each rank copying its shard's rows
                shared = _SHM.acquire(children.shape, _BLOCKS.keep_for(n * L * 8)) if block_rows else None
                if shared is not None:
                    rank, ws = world()
                    lo, hi = shard_range(n, rank, ws)
                    host = torch.from_numpy(shared)
                    if lo < hi:
                        host[lo:hi].copy_(children[lo:hi], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record()
                    events = [ev]
                else:
                    if block_rows:
                        _BLOCKS.reserve(children.shape)
                    host = torch.empty(children.shape, dtype=torch.float64, pin_memory=True)
                    nchunk = 1 if block_rows else (8 if n >= 16 else 1)
                    rows = (n + nchunk - 1) // nchunk
                    events = []
                    for c in range(nchunk):
                        lo, hi = c * rows, min(n, (c + 1) * rows)
                        if lo < hi:
                            host[lo:hi].copy_(children[lo:hi], non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record()
                        events.append(ev)
            finally:
                rng_done()   # numpy's global state after the step's np.random.rand draws
        t = _mark(t, "ev_transfer_issue")
        # the candidates (new uids, the parent's other attributes) while the transfer runs
        next_pop = [_copy_individual(population[i]) for i in range(n)]
        t = _mark(t, "ev_candidates")
        if (shared is not None or block_rows) and all(_assigns_genome(c) for c in next_pop):
            # whole-block rows: every child is bound to its row (a view: nothing reads the values),
            # recorded, and the older blocks compacted while the rows are still in flight; the
            # children are returned once their rows have landed (every rank's, for a shared block)
            arrays = _BLOCKS.rows(shared if shared is not None else host.numpy())
            t = _mark(t, "ev_arrays")
            self._bind(next_pop, arrays, inds, genomes, children, parents, store, speculated, evaluator)
            t = _mark(t, "ev_bind_record")
            _BLOCKS.compact(inds, store)
            t = _mark(t, "ev_compact")
            events[-1].synchronize()
            if shared is not None:
                import torch.distributed as dist
                dist.barrier()   # every rank's shard of the rows has landed
            _mark(t, "ev_rows_landed")
            return next_pop
        if shared is not None:
            events[-1].synchronize()
            import torch.distributed as dist
            dist.barrier()   # every rank's shard of the rows has landed
            arrays = _BLOCKS.rows(shared)
        elif block_rows:
            events[-1].synchronize()
            arrays = _BLOCKS.rows(host.numpy())
        else:
            # an own array per child; float64 rows go into page-locked buffers from torch's caching
            # host allocator, which hands back the buffers of dead genomes: no page faults on the copy
            dest = None
            if dtypes is None and n * L * 8 <= _PINNED_ROWS_MAX:
                dest = [torch.empty(L, dtype=torch.float64, pin_memory=True).numpy() for _ in range(n)]
            arrays = _copy_rows(host.numpy(), dtypes, ready=[ev.synchronize for ev in events], dest=dest)
        t = _mark(t, "ev_arrays")
        self._bind(next_pop, arrays, inds, genomes, children, parents, store, speculated, evaluator, dtypes)
        t = _mark(t, "ev_bind_record")
        # older blocks the parents leave sparsely used, while the GPU still evaluates the children
        _BLOCKS.compact(inds, store)
        _mark(t, "ev_compact")
        return next_pop

    @staticmethod
    def _bind(next_pop, arrays, inds, genomes, children, parents, store, speculated, evaluator, dtypes=None):
        for i in range(len(next_pop)):
            next_pop[i].set_internal_genome(arrays[i])
        if speculated:
            evaluator._spec_bind(next_pop)
        if dtypes is None:   # float64 internal genomes: the device rows are the children's exact values
            store.record_rows(children, next_pop, arrays)
            store.record(parents, inds, genomes, adopt=True)
        store.prune([x.uid for x in inds] + [x.uid for x in next_pop])


class DERandOneEvolver(_GpuDEEvolver):
    """DE/rand/1 (evolver.py:86-157)."""

    strategy = _native.DE_STRATEGY["de_rand_1"]

    def _donors(self, population, L):
        n = len(population)
        drawn = _native_donors(self.strategy, n, L)
        if drawn is not None:
            return drawn
        donors = np.empty((n, 3), dtype=np.int32)
        fixed = np.empty(n, dtype=np.int64)
        for i in range(n):   # de_rand_one (evolver.py:118-121) then crossover (evolver.py:76)
            a = exclusive_randrange(0, n, [i])
            b = exclusive_randrange(0, n, [i, a])
            c = exclusive_randrange(0, n, [i, a, b])
            donors[i] = (a, b, c)
            fixed[i] = random.randrange(0, L)
        return donors, fixed


class DECurrentToBestOneEvolver(_GpuDEEvolver):
    """DE/current-to-best/1 (evolver.py:160-244)."""

    strategy = _native.DE_STRATEGY["de_currenttobest_1"]

    def _clip(self):
        return True   # evolve() calls de_currenttobest_one without clip (default True)

    def _donors(self, population, L):
        n = len(population)
        best = max(population, key=lambda individual: individual.fitness)   # evolver.py:235
        best_index = population.population.index(best)                      # evolver.py:194
        drawn = _native_donors(self.strategy, n, L, best_index)
        if drawn is not None:
            return drawn
        donors = np.empty((n, 3), dtype=np.int32)
        fixed = np.empty(n, dtype=np.int64)
        for i in range(n):   # evolver.py:199-203, then crossover (evolver.py:76)
            exclusion_list = [i, best_index]
            a = exclusive_randrange(0, n, exclusion_list)
            exclusion_list.append(a)
            b = exclusive_randrange(0, n, exclusion_list)
            donors[i] = (best_index, a, b)
            fixed[i] = random.randrange(0, L)
        return donors, fixed


# ---------------------------------------------------------------------------------------------
# Adaptive evolvers (evolver.py:297-687)
# ---------------------------------------------------------------------------------------------
class AdaptiveEvolver(Evolver):
    """Bookkeeping of the F / CR values whose candidates entered the population (evolver.py:297-404),
    with the reference's parameter report (a `_params` CSV beside the monitor's results file)."""

    def __init__(self):
        self.successful_fs = []
        self.successful_crs = []
        self.previous_pop_uids = None
        self.crs = []
        self.fs = []

    def should_report(self):
        return True

    def report(self, population):
        stem, ext = os.path.splitext(os.path.basename(population.monitor.results_file))
        path = os.path.join(os.path.dirname(population.monitor.results_file), stem + "_params" + ext)
        if population.generation == 1:
            with open(path, "w") as f:
                csv.writer(f).writerow(self.get_header())
        with open(path, "a") as f:
            csv.writer(f).writerow(self.get_params_row())

    @abc.abstractmethod
    def get_header(self):
        raise NotImplementedError()

    @abc.abstractmethod
    def get_params_row(self):
        raise NotImplementedError()

    def evolve(self, population):
        """The per-generation adaptation step subclasses run first (evolver.py:336-356)."""
        if self.should_report():
            self.report(population)
        if self.previous_pop_uids is None:
            self.previous_pop_uids = [x.uid for x in population]
        self.count_outcomes(population)
        if self.should_regenerate_crs(population):
            self.regenerate_crs(population)
        if self.should_regenerate_fs(population):
            self.regenerate_fs(population)
        self.previous_pop_uids = [x.uid for x in population]

    def count_outcomes(self, population):
        """A changed uid at position i: the candidate made with crs[i] / fs[i] entered the population."""
        for i, (old, cur) in enumerate(zip(self.previous_pop_uids, population)):
            if old != cur.uid:
                if i < len(self.crs):
                    self.successful_crs.append(self.crs[i])
                if i < len(self.fs):
                    self.successful_fs.append(self.fs[i])

    @abc.abstractmethod
    def should_regenerate_crs(self, population):
        raise NotImplementedError()

    @abc.abstractmethod
    def generate_cr(self):
        raise NotImplementedError()

    def regenerate_crs(self, population):
        self.crs = [self.generate_cr() for _ in range(len(population))]

    @abc.abstractmethod
    def should_regenerate_fs(self, population):
        raise NotImplementedError()

    @abc.abstractmethod
    def generate_f(self):
        raise NotImplementedError()

    def regenerate_fs(self, population):
        self.fs = [self.generate_f() for _ in range(len(population))]


class SaDE(AdaptiveEvolver, _GpuDEEvolver):
    """Self-adaptive DE (Qin & Suganthan 2005; evolver.py:407-547), its generation on the GPU.

    Per generation: cr_m re-estimated every 25 generations, the crossover rates redrawn every 5
    (N(cr_m, 0.1) clipped to [0, 1]), one F ~ N(0.5, 0.3) clipped to [0, 2], and per individual
    DE/rand/1 with probability p, else DE/current-to-best/1, p learnt from the strategies' success
    counts after a 50-generation learning period.  The host draws what the reference draws, in its
    order (numpy's normal() calls, then per individual random.random(), the donors and the forced
    crossover position); the GPU step computes every child with its own strategy and rate."""

    f_m = 0.5
    f_std = 0.3
    cr_std = 0.1
    recalculate_mean_interval = 25
    regenerate_crs_interval = 5
    initial_learning_period = 50

    def __init__(self, dimensionality, clip=True):
        AdaptiveEvolver.__init__(self)
        self.dimensionality = dimensionality
        self.clip = clip
        self.cr_m = 0.5
        self.p = 0.5
        self.strategy_one_indices = set()
        self.ns_1, self.ns_2, self.nf_1, self.nf_2 = 0, 0, 0, 0

    def get_header(self):
        return ["cr_m", "p"]

    def get_params_row(self):
        return [self.cr_m, self.p]

    def should_regenerate_crs(self, population):
        return len(self.crs) == 0 or population.generation % self.regenerate_crs_interval == 0

    def should_recalculate_cr_m(self, generation):
        return generation != 0 and generation % self.recalculate_mean_interval == 0

    def recalculate_cr_m(self):
        if self.successful_crs:
            self.cr_m = np.mean(self.successful_crs)

    def generate_f(self):
        return np.clip(np.random.normal(self.f_m, self.f_std), 0, 2)

    def generate_cr(self):
        return np.clip(np.random.normal(self.cr_m, self.cr_std), 0, 1)

    def should_regenerate_fs(self, population):
        return False

    def recalculate_p(self, population):
        if population.generation >= self.initial_learning_period and (self.ns_1 or self.ns_2):
            num = self.ns_1 * (self.ns_2 + self.nf_2)
            self.p = num / (self.ns_2 * (self.ns_1 + self.nf_1) + num)

    def count_outcomes(self, population):
        AdaptiveEvolver.count_outcomes(self, population)
        if population.generation == self.initial_learning_period:
            # learning period over: counters restart from one success each (evolver.py:479-484)
            self.ns_1, self.ns_2, self.nf_1, self.nf_2 = 1, 1, 0, 0
        for i, (old, cur) in enumerate(zip(self.previous_pop_uids, population)):
            one = i in self.strategy_one_indices
            if old == cur.uid:
                if one:
                    self.nf_1 += 1
                else:
                    self.nf_2 += 1
            elif one:
                self.ns_1 += 1
            else:
                self.ns_2 += 1

    def evolve(self, population):
        import time
        t = time.perf_counter()
        if self.should_recalculate_cr_m(population.generation):
            self.recalculate_cr_m()
        AdaptiveEvolver.evolve(self, population)
        self.recalculate_p(population)
        f = self.generate_f()
        n = len(population)
        members = _members(population)
        L = members[2]
        best = max(population, key=lambda indv: indv.fitness)
        best_index = population.population.index(best)
        strategies = np.empty(n, dtype=np.int32)
        donors = np.empty((n, 3), dtype=np.int32)
        fixed = np.empty(n, dtype=np.int64)
        self.strategy_one_indices = set()
        for i in range(n):
            if random.random() < self.p:   # DE/rand/1 (evolver.py:118-121)
                self.strategy_one_indices.add(i)
                strategies[i] = 0
                a = exclusive_randrange(0, n, [i])
                b = exclusive_randrange(0, n, [i, a])
                donors[i] = (a, b, exclusive_randrange(0, n, [i, a, b]))
            else:                          # DE/current-to-best/1 (evolver.py:199-203)
                strategies[i] = 1
                a = exclusive_randrange(0, n, [i, best_index])
                donors[i] = (best_index, a, exclusive_randrange(0, n, [i, best_index, a]))
            fixed[i] = random.randrange(0, L)   # the crossover's forced position (evolver.py:76)
        crs = np.array([float(c) for c in self.crs[:n]], dtype=np.float64)
        return self._gpu_generation(population, t, donors, fixed, strategies, f, crs, self.clip, members)


class MDE_pBX(AdaptiveEvolver):
    """MDE_pBX (Islam et al. 2012; evolver.py:550-687), the DE step on the host.

    Each individual draws its group best and its parent with np.random.choice -- rejection-sampled
    integers, a data-dependent number of MT19937 words -- between the individuals' np.random.rand(L)
    calls, so an individual's numpy stream offset depends on every draw before it and cannot be
    jumped to in parallel as the GPU step does.  The generation therefore runs as the reference's
    loop: the same draws in the same order, DE/current-to-best/1 with the chosen best and parent,
    binary crossover, optional clip."""

    f_scale = 0.1
    cr_std = 0.1
    group_q = 0.15

    def __init__(self, dimensionality, generations, clip=True):
        AdaptiveEvolver.__init__(self)
        self.dimensionality = dimensionality
        self.clip = clip
        self.g_max = generations
        self.cr_m = 0.6
        self.f_m = 0.5
        self.p = None

    def get_header(self):
        return ["cr_m", "f_m"]

    def get_params_row(self):
        return [self.cr_m, self.f_m]

    def should_regenerate_fs(self, population):
        return True

    def should_regenerate_crs(self, population):
        return True

    def generate_cr(self):
        """N(cr_m, 0.1), redrawn until in [0, 1]."""
        while True:
            cr = np.random.normal(self.cr_m, self.cr_std)
            if 0 <= cr <= 1:
                return cr

    def generate_f(self):
        """Cauchy(f_m, 0.1) (scipy.stats.cauchy on numpy's global RandomState), redrawn until in [0, 1]."""
        from scipy.stats import cauchy
        while True:
            f = cauchy.rvs(loc=self.f_m, scale=self.f_scale)
            if 0 <= f <= 1:
                return f

    @staticmethod
    def mean_pow(vals, n=1.5):
        """The power mean of formula (10), simplified for positive values as the reference does."""
        assert n > 0, "n must be a positive number."
        return sum(vals) / pow(1 / len(vals), -n)

    @staticmethod
    def get_weight_factor(p, q):
        return p + q * random.random()

    def recalculate_cr_m(self):
        if self.successful_crs:
            w = self.get_weight_factor(0.9, 0.1)
            self.cr_m = w * self.cr_m + (1 - w) * self.mean_pow(self.successful_crs)
            self.successful_crs = []

    def recalculate_f_m(self):
        if self.successful_fs:
            w = self.get_weight_factor(0.8, 0.2)
            self.f_m = w * self.f_m + (1 - w) * self.mean_pow(self.successful_fs)
            self.successful_fs = []

    def recalculate_p(self, population):
        self.p = ceil((len(population) / 2) * (1 - (population.generation / self.g_max)))

    def evolve(self, population):
        self.recalculate_cr_m()
        self.recalculate_f_m()
        self.recalculate_p(population)
        AdaptiveEvolver.evolve(self, population)
        order = np.argsort([x.fitness for x in population])
        q_best = order[-int(len(population) * self.group_q):]
        p_best = order[-self.p:]
        n = len(population)
        out = []
        for i in range(n):
            best = population[np.random.choice(q_best, 1).item()]
            parent_idx = np.random.choice(p_best, 1).item()
            out.append(_host_current_to_best(population, self.fs[i], self.crs[i], self.dimensionality, parent_idx,
                                             best, self.clip))
        return out


def _host_current_to_best(population, mi, cr, dimensionality, parent_idx, best, clip):
    """DECurrentToBestOneEvolver.de_currenttobest_one with binary crossover (evolver.py:63-82,
    179-221) on the host: the reference's draws (exclusive_randrange x 2, random.randrange, one
    np.random.rand(L)) and its float arithmetic order."""
    n = len(population)
    best_index = population.population.index(best)
    excl = [parent_idx, best_index]
    a = exclusive_randrange(0, n, excl)
    excl.append(a)
    b = exclusive_randrange(0, n, excl)
    ga, gb = population[a].get_internal_genome(), population[b].get_internal_genome()
    child = deepcopy(population[parent_idx])
    x = child.get_internal_genome()
    mutant = x + mi * (best.get_internal_genome() - x) + mi * (ga - gb)
    L = len(x)
    fixed = random.randrange(0, L)
    take = np.random.rand(L) < cr
    take[fixed] = True
    child.set_internal_genome(np.where(take, mutant, x))
    if clip:
        child.set_internal_genome(np.clip(child.get_internal_genome(), 0, dimensionality - 1))
    return child
