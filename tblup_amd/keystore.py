"""Device-resident internal genomes of recent individuals, keyed by uid.

The GPU DE step (tblup_amd.evolver) leaves each generation's children on the
device; the evaluator decodes them there (k_decode_topk) and the next
generation's DE step reads its parents there, so the population's keys cross
PCIe once per generation (children to the host, for the reference's
Individual objects) instead of three times (parents up, children down, keys up
again for the decode).

An entry is valid while the individual still holds the very numpy array the
entry was recorded with (`indv._genome is <recorded array>`), that array has not
been written since, and the individual has the same `length`.
`set_internal_genome` and `fill` (individual.py:103-130, 187-208,
scheduler.py:209-251) replace the array or change the length.  In-place writes
are allowed, as the reference allows them (`Individual.__setitem__`,
individual.py:119-120), but never silently: a recorded array is a `TrackedGenome`,
a READ-ONLY view whose memory has no other writable numpy alias (the page-locked
block it lives in, or an adopted initial genome, is made read-only too).  Every
numpy write path it intercepts -- item assignment, in-place ufuncs and `out=`,
`ufunc.at`, the writing methods (`fill`, `sort`, `put`, `partition`, `byteswap`,
`setfield`, `itemset`) and the writing functions (`np.copyto`, `np.put`, `np.place`,
`np.putmask`, `np.put_along_axis`, `np.fill_diagonal`, any `out=`) -- marks the
array stale and then writes through a private writable alias; every other write
(`np.random.shuffle`, writes through `np.asarray(g)` or `g.view(np.ndarray)`, the
buffer protocol) meets a read-only array and raises.  A stale or replaced genome is
read from the host.  Device memory is plumbing here: torch tensors on the context's
device.
"""
import os
import weakref

import numpy as np


class TrackedGenome(np.ndarray):
    """A genome array the key store mirrors on the device: read-only to numpy, written only
    through the paths below, each of which first marks the owning array stale.  Views of it
    are TrackedGenomes of the same owner; copies and results of computations are plain
    (writable, untracked) arrays."""

    _owner = None    # the recorded array this view belongs to (None: it is the owner)
    _stale = False
    _w = None        # owner only: a writable plain alias of its memory, held by nobody else
    _blk = None      # track_rows: the 2-D block this row belongs to (the evolver's page-locked blocks)

    def __array_finalize__(self, obj):
        if isinstance(obj, TrackedGenome) and obj._tracked() and not self.flags.owndata:
            self._owner = obj._owner if obj._owner is not None else obj
        else:                      # a copy: behaves as a plain array
            self._owner = None
            self._w = None

    def _tracked(self):
        return self._owner is not None or self._w is not None

    def _root(self):
        return self._owner if self._owner is not None else self

    def _writable(self):
        """A writable plain view of exactly this array's elements (marks the owner stale)."""
        root = self._root()
        if root._w is None:        # untracked copy
            return self.view(np.ndarray)
        root._stale = True
        base = root._w
        off = self.__array_interface__["data"][0] - base.__array_interface__["data"][0]
        return np.ndarray(self.shape, dtype=self.dtype, buffer=base, offset=off, strides=self.strides)

    def _touch(self):
        if self._tracked():
            self._root()._stale = True

    # -- item assignment and the writing methods
    def __setitem__(self, key, value):
        if not self._tracked():
            return super().__setitem__(key, value)
        self._writable()[key] = value

    def fill(self, value):
        (self._writable() if self._tracked() else super()).fill(value)

    def sort(self, *a, **k):
        (self._writable() if self._tracked() else super()).sort(*a, **k)

    def partition(self, *a, **k):
        (self._writable() if self._tracked() else super()).partition(*a, **k)

    def put(self, *a, **k):
        (self._writable() if self._tracked() else super()).put(*a, **k)

    def setfield(self, *a, **k):
        (self._writable() if self._tracked() else super()).setfield(*a, **k)

    def itemset(self, *a):
        w = self._writable() if self._tracked() else self.view(np.ndarray)
        w[a[:-1] if len(a) > 2 else a[0]] = a[-1]

    def byteswap(self, inplace=False):
        if inplace and self._tracked():
            self._writable().byteswap(inplace=True)
            return self
        return super().byteswap(inplace).view(np.ndarray)

    # -- ufuncs: in place (out=) and ufunc.at write; everything else computes plain arrays
    def __array_ufunc__(self, ufunc, method, *inputs, out=None, **kwargs):
        def plain(x):
            return x.view(np.ndarray) if isinstance(x, TrackedGenome) else x
        if method == "at" and isinstance(inputs[0], TrackedGenome):
            inputs = (inputs[0]._writable(),) + tuple(plain(x) for x in inputs[1:])
        else:
            inputs = tuple(plain(x) for x in inputs)
        if out is not None:
            kwargs["out"] = tuple(o._writable() if isinstance(o, TrackedGenome) else o for o in out)
        res = getattr(ufunc, method)(*inputs, **kwargs)
        if out is not None:
            return out[0] if len(out) == 1 else out
        return res

    # -- numpy functions that write into an argument
    _WRITERS = {np.copyto: 0, np.put: 0, np.place: 0, np.putmask: 0, np.put_along_axis: 0, np.fill_diagonal: 0}

    def __array_function__(self, func, types, args, kwargs):
        pos = TrackedGenome._WRITERS.get(func)
        if pos is not None and len(args) > pos and isinstance(args[pos], TrackedGenome):
            args = list(args)
            args[pos] = args[pos]._writable()
        o = kwargs.get("out")
        if isinstance(o, TrackedGenome):
            kwargs = dict(kwargs, out=o._writable())
        elif isinstance(o, tuple) and any(isinstance(x, TrackedGenome) for x in o):
            kwargs = dict(kwargs, out=tuple(x._writable() if isinstance(x, TrackedGenome) else x for x in o))
        args = tuple(a.view(np.ndarray) if isinstance(a, TrackedGenome) else a for a in args)
        res = super().__array_function__(func, types, args, kwargs)
        if o is not None:
            return o
        return res

    def __reduce__(self):   # pickles / deep-copies as a plain ndarray
        return self.view(np.ndarray).__reduce__()

    def __deepcopy__(self, memo):
        return self.view(np.ndarray).copy()

    def __copy__(self):
        return self.view(np.ndarray).copy()


def track(a, lock=True):
    """A TrackedGenome over the float64 array `a`'s memory (no copy).  `a` itself is made
    read-only (lock=False: the caller locks the memory's owner, e.g. a whole block, after
    tracking all of its rows), so the only writable alias left is the TrackedGenome's own."""
    w = a.view(np.ndarray)
    t = a.view(TrackedGenome)
    t._w = w
    t._owner = None
    t.flags.writeable = False
    if lock:
        a.flags.writeable = False
    return t


def track_rows(block):
    """track() for every row of a 2-D float64 block in one pass: each row its own owner (marking
    one row stale leaves the others alone) with a writable alias taken from one writable view of
    the block (list(view) slices the rows without per-row indexing: 2.8 -> 1.0 ms for 1024 rows).
    The caller locks the block itself afterwards, as with track(lock=False)."""
    wl = list(block.view(np.ndarray))
    tb = block.view(TrackedGenome)
    tb.flags.writeable = False      # the rows inherit it
    rows = list(tb)
    for t, w in zip(rows, wl):
        t._w = w
        t._blk = block
    return rows


_FROZEN = False


def freeze_heap():
    """Once per process: move every object that exists now -- the imported modules (torch,
    scipy, sklearn, numpy: ~10^6 container objects) -- into the collector's permanent generation
    (gc.freeze), so python's full collections stop traversing them.  A full collection over that
    heap took 93 ms, every ~15 DE generations at pop 1024 (profiles/r05_generation_gc.jsonl); after
    the freeze it walks only the objects created since (the population, its genomes).  Called
    where the drop-ins start up (ParallelEvaluator.__enter__, the first GPU DE step); objects alive
    at that moment are never collected as cyclic garbage (reference counting still frees them).

    A process-wide side effect, so it can be switched off (TBLUP_GC_FREEZE=0) and is undone by
    thaw_heap() -- ParallelEvaluator.__exit__ calls it -- which moves the frozen objects back into
    the collected generations.  Returns True when this call froze the heap."""
    global _FROZEN
    if _FROZEN or os.environ.get("TBLUP_GC_FREEZE", "1") == "0":
        return False
    import gc
    _FROZEN = True
    gc.collect()
    gc.freeze()
    return True


def thaw_heap():
    """Undo freeze_heap (gc.unfreeze): the permanent generation back into the oldest collected
    one, so the host application's objects frozen with the imports are collectable again."""
    global _FROZEN
    if _FROZEN:
        import gc
        gc.unfreeze()
        _FROZEN = False


_STREAMS = {}


def work_stream(device):
    """A dedicated (non-default) torch stream per device for the device-resident DE /
    decode plumbing: its handle is passed to the C ABI, so the library's kernels and
    torch's copies of the same tensors are ordered on one stream (the legacy default
    stream does not order against the library's non-blocking context stream)."""
    import torch
    s = _STREAMS.get(device)
    if s is None:
        s = _STREAMS[device] = torch.cuda.Stream(device=device)
    return s


class DeviceKeyStore:
    _instances = {}

    @classmethod
    def get(cls, device):
        inst = cls._instances.get(device)
        if inst is None:
            inst = cls._instances[device] = cls(device)
        return inst

    def __init__(self, device):
        self.device = int(device)
        # uid -> (tensor, row, weakref(genome array), length, row address, row length): the row's
        # device address (0 unless the tensor is a plain row-major float64 matrix) taken when the
        # row is recorded, so the DE step's gather reads addresses instead of tensor geometry
        self._entries = {}

    @staticmethod
    def _geo(tensor):
        """(base address, row pitch in bytes, row length) of a plain row-major float64 (., L) device
        matrix, else (0, 0, -1)."""
        import torch
        if tensor.dim() == 2 and tensor.stride(1) == 1 and tensor.dtype == torch.float64:
            return tensor.data_ptr(), 8 * tensor.stride(0), tensor.shape[1]
        return 0, 0, -1

    @staticmethod
    def _key_array(indv):
        g = getattr(indv, "_genome", None)
        return g if isinstance(g, np.ndarray) else None

    def record_rows(self, tensor, individuals, arrays):
        """record() for a generation's children that the evolver has just bound to fresh TrackedGenome
        rows (every individual's genome IS arrays[i]): one dict update."""
        p0, pitch, nc = self._geo(tensor)
        self._entries.update({indv.uid: (tensor, i, weakref.ref(g), getattr(indv, "length", None),
                                         p0 + pitch * i if p0 else 0, nc)
                              for i, (indv, g) in enumerate(zip(individuals, arrays))
                              if getattr(indv, "_genome", None) is g})

    def record(self, tensor, individuals, arrays, adopt=False):
        """Row i of `tensor` (pop x L, on the device) holds arrays[i]; recorded for individuals
        whose internal genome IS that array (RandomKey / Index semantics: get_internal_genome()
        returns `_genome`) and a TrackedGenome (the evolver hands its children such views;
        parents recorded from other arrays are not tracked and are read from the host).
        Individuals that derive their internal genome (Coevolution appends its length) are not
        recorded and are read from the host."""
        ent = self._entries
        p0, pitch, nc = self._geo(tensor)
        for i, (indv, a) in enumerate(zip(individuals, arrays)):
            g = getattr(indv, "_genome", None)
            if g is not a or g is None:
                continue
            if type(g) is TrackedGenome and not g._stale:   # the common case, inlined
                ent[indv.uid] = (tensor, i, weakref.ref(g), getattr(indv, "length", None), p0 + pitch * i if p0 else 0, nc)
                continue
            if not isinstance(g, np.ndarray):
                continue
            if not isinstance(g, TrackedGenome):
                # a genome the evolver did not create (the initial population): adopt it as a
                # tracked view of the same buffer when nothing else views that buffer
                if not adopt or g.base is not None or g.dtype != np.float64 or not g.flags.c_contiguous:
                    continue
                g = track(g)
                indv._genome = g
            if g._stale:
                continue
            ent[indv.uid] = (tensor, i, weakref.ref(g), getattr(indv, "length", None), p0 + pitch * i if p0 else 0, nc)

    def lookup(self, indv):
        e = self._entries.get(indv.uid)
        if e is None:
            return None
        g = e[2]()
        if g is None or g is not self._key_array(indv) or g._stale or getattr(indv, "length", None) != e[3]:
            del self._entries[indv.uid]
            return None
        return e[0], e[1]

    def rebind(self, indv, old, new):
        """indv's genome array `old` was replaced by the equal-valued TrackedGenome `new`
        (the evolver compacting page-locked blocks): keep its device row."""
        e = self._entries.get(indv.uid)
        if e is not None and e[2]() is old and not old._stale:
            self._entries[indv.uid] = (e[0], e[1], weakref.ref(new)) + e[3:]

    def rows(self, individuals):
        """(tensor, row) per individual (None where absent): lookup() inlined over the batch."""
        ent = self._entries
        out = []
        for indv in individuals:
            e = ent.get(indv.uid)
            if e is not None:
                g = e[2]()
                k = getattr(indv, "_genome", None)
                if (g is not None and g is k and isinstance(k, np.ndarray) and not g._stale
                        and getattr(indv, "length", None) == e[3]):
                    out.append((e[0], e[1]))
                    continue
                del ent[indv.uid]
            out.append(None)
        return out

    def gather(self, individuals, L, host_rows=None, copy_rows=None):
        """A contiguous (len(individuals) x L) float64 device tensor of their internal genomes;
        rows not in the store come from host_rows(i) (None -> return None if any is missing).
        No copy when the individuals are exactly one recorded block in order.  copy_rows(out,
        pointers): one native gather of the recorded rows (pointer 0 = row to skip)."""
        import torch
        n = len(individuals)
        if copy_rows is not None and n:
            out = self._gather_ptrs(individuals, L, host_rows, copy_rows)
            if out is not False:
                return out
        hits = self.rows(individuals)
        if n and all(h is not None for h in hits):
            t0 = hits[0][0]
            if t0.shape == (n, L) and all(h[0] is t0 and h[1] == i for i, h in enumerate(hits)):
                return t0
        if host_rows is None and any(h is None for h in hits):
            return None
        out = torch.empty((n, L), dtype=torch.float64, device="cuda:%d" % self.device)
        # every row's device address in one pass: (base address, row pitch in bytes) per distinct
        # device tensor (torch's accessors once per tensor, not per row), None if that tensor is not
        # a plain row-major (., L) float64 matrix
        if copy_rows is not None:
            geo = {}
            ptrs = [0] * n
            missing = []
            plain = True
            for i, h in enumerate(hits):
                if h is None:
                    missing.append(i)
                    continue
                t, row = h
                g = geo.get(id(t))
                if g is None:
                    g = geo[id(t)] = ((t.data_ptr(), 8 * t.stride(0))
                                      if t.dim() == 2 and t.shape[1] == L and t.stride(1) == 1 else ())
                if not g:
                    plain = False
                    break
                ptrs[i] = g[0] + g[1] * row
            if plain:
                if len(missing) < n:
                    if missing:   # missing slots: any recorded row, overwritten below
                        any_row = next(q for q in ptrs if q)
                        for i in missing:
                            ptrs[i] = any_row
                    copy_rows(out, ptrs)
                if missing:
                    self._fill_missing(out, missing, host_rows)
                return out
        by_tensor = {}
        missing = []
        for i, h in enumerate(hits):
            if h is None:
                missing.append(i)
            elif h[0].shape[1] != L:
                return None if host_rows is None else self._fill_missing(out, list(range(n)), host_rows)
            else:
                by_tensor.setdefault(id(h[0]), (h[0], [], []))
                by_tensor[id(h[0])][1].append(i)
                by_tensor[id(h[0])][2].append(h[1])
        for t, dst, src in by_tensor.values():
            di = torch.tensor(dst, device=out.device)
            si = torch.tensor(src, device=out.device)
            out.index_copy_(0, di, t.index_select(0, si))
        if missing:
            self._fill_missing(out, missing, host_rows)
        return out

    def _gather_ptrs(self, individuals, L, host_rows, copy_rows):
        """gather() from the recorded row addresses in one pass (rows() inlined); False when some
        recorded tensor is not a plain (., L) matrix (the caller's general path)."""
        import torch
        ent = self._entries
        n = len(individuals)
        ptrs = [0] * n
        missing = []
        t0 = None
        block = True   # exactly rows 0 .. n-1 of one recorded (n, L) tensor, in order
        for i, indv in enumerate(individuals):
            e = ent.get(indv.uid)
            if e is not None:
                g = e[2]()
                if (g is not None and g is getattr(indv, "_genome", None) and not g._stale
                        and getattr(indv, "length", None) == e[3]):
                    if not e[4] or e[5] != L:
                        return False
                    ptrs[i] = e[4]
                    if block:
                        if t0 is None:
                            t0 = e[0]
                        block = e[0] is t0 and e[1] == i
                    continue
                del ent[indv.uid]
            missing.append(i)
            block = False
        if block and t0 is not None and t0.shape[0] == n:
            return t0
        if missing and host_rows is None:
            return None
        out = torch.empty((n, L), dtype=torch.float64, device="cuda:%d" % self.device)
        if len(missing) < n:
            if missing:   # missing slots: any recorded row, overwritten below
                any_row = next(q for q in ptrs if q)
                for i in missing:
                    ptrs[i] = any_row
            copy_rows(out, ptrs)
        if missing:
            self._fill_missing(out, missing, host_rows)
        return out

    @staticmethod
    def _fill_missing(out, idx, host_rows):
        import torch
        host = torch.from_numpy(np.stack([np.asarray(host_rows(i), dtype=np.float64) for i in idx]))
        out.index_copy_(0, torch.tensor(idx, device=out.device), host.to(out.device, non_blocking=False))
        return out

    def prune(self, keep_uids):
        keep = set(keep_uids)
        for uid in [u for u in self._entries if u not in keep]:
            del self._entries[uid]

    def clear(self):
        self._entries.clear()
