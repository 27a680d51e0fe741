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
scheduler.py:209-251) replace the array or change the length; an in-place write
(`Individual.__setitem__`, individual.py:119-120, or any numpy write through the
array or a view of it) marks the recorded array stale -- recorded arrays are
`TrackedGenome` views (an ndarray subclass that notices item assignment and
in-place ufuncs) and stay writable, as the reference allows.  A stale or replaced
genome is read from the host.  Device memory is plumbing here: torch tensors on
the context's device.
"""
import weakref

import numpy as np


class TrackedGenome(np.ndarray):
    """A genome array the key store mirrors on the device.  Writes through it or through
    any view of it (item assignment, in-place ufuncs / `out=`) mark the owning array
    stale; values and semantics are otherwise those of the ndarray it views.  Results of
    computations on it are plain ndarrays."""

    _owner = None
    _stale = False

    def __array_finalize__(self, obj):
        if isinstance(obj, TrackedGenome):
            self._owner = obj._owner if obj._owner is not None else obj

    def _touch(self):
        (self._owner if self._owner is not None else self)._stale = True

    def __setitem__(self, key, value):
        self._touch()
        super().__setitem__(key, value)

    def __array_ufunc__(self, ufunc, method, *inputs, out=None, **kwargs):
        plain = tuple(x.view(np.ndarray) if isinstance(x, TrackedGenome) else x for x in inputs)
        if out is not None:
            for o in out:
                if isinstance(o, TrackedGenome):
                    o._touch()
            kwargs["out"] = tuple(o.view(np.ndarray) if isinstance(o, TrackedGenome) else o for o in out)
        res = getattr(ufunc, method)(*plain, **kwargs)
        if out is not None:
            return out[0] if len(out) == 1 else out
        return res

    def __reduce__(self):   # pickles / deep-copies as a plain ndarray
        return self.view(np.ndarray).__reduce__()

    def __deepcopy__(self, memo):
        return self.view(np.ndarray).copy()

    def __copy__(self):
        return self.view(np.ndarray).copy()


def track(a):
    """A TrackedGenome view of the float64 array `a` (no copy)."""
    return a.view(TrackedGenome)


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
        self._entries = {}   # uid -> (tensor, row, weakref(genome array), length)

    @staticmethod
    def _key_array(indv):
        g = getattr(indv, "_genome", None)
        return g if isinstance(g, np.ndarray) else None

    def record(self, tensor, individuals, arrays, adopt=False):
        """Row i of `tensor` (pop x L, on the device) holds arrays[i]; recorded for individuals
        whose internal genome IS that array (RandomKey / Index semantics: get_internal_genome()
        returns `_genome`) and a TrackedGenome (the evolver hands its children such views;
        parents recorded from other arrays are not tracked and are read from the host).
        Individuals that derive their internal genome (Coevolution appends its length) are not
        recorded and are read from the host."""
        for i, indv in enumerate(individuals):
            g = self._key_array(indv)
            if g is None or g is not arrays[i]:
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
            self._entries[indv.uid] = (tensor, i, weakref.ref(g), getattr(indv, "length", None))

    def lookup(self, indv):
        e = self._entries.get(indv.uid)
        if e is None:
            return None
        tensor, row, ref, length = e
        g = ref()
        if g is None or g is not self._key_array(indv) or g._stale or getattr(indv, "length", None) != length:
            del self._entries[indv.uid]
            return None
        return tensor, row

    def rebind(self, indv, old, new):
        """indv's genome array `old` was replaced by the equal-valued TrackedGenome `new`
        (the evolver compacting page-locked blocks): keep its device row."""
        e = self._entries.get(indv.uid)
        if e is not None and e[2]() is old and not old._stale:
            self._entries[indv.uid] = (e[0], e[1], weakref.ref(new), e[3])

    def rows(self, individuals):
        """(tensor, row) per individual (None where absent)."""
        return [self.lookup(i) for i in individuals]

    def gather(self, individuals, L, host_rows=None, copy_rows=None):
        """A contiguous (len(individuals) x L) float64 device tensor of their internal genomes;
        rows not in the store come from host_rows(i) (None -> return None if any is missing).
        No copy when the individuals are exactly one recorded block in order.  copy_rows(out,
        pointers): one native gather of the recorded rows (pointer 0 = row to skip)."""
        import torch
        hits = self.rows(individuals)
        n = len(individuals)
        if n and all(h is not None for h in hits):
            t0 = hits[0][0]
            if t0.shape == (n, L) and all(h[0] is t0 and h[1] == i for i, h in enumerate(hits)):
                return t0
        if host_rows is None and any(h is None for h in hits):
            return None
        out = torch.empty((n, L), dtype=torch.float64, device="cuda:%d" % self.device)
        # (base address, row pitch in bytes) per distinct device tensor, None if not a plain
        # row-major (., L) float64 matrix: torch's accessors once per tensor, not per row
        geo = {}
        for h in hits:
            if h is not None and id(h[0]) not in geo:
                t = h[0]
                geo[id(t)] = ((t.data_ptr(), 8 * t.stride(0))
                              if t.dim() == 2 and t.shape[1] == L and t.stride(1) == 1 else None)
        if copy_rows is not None and all(g is not None for g in geo.values()):
            ptrs = []
            for h in hits:
                if h is None:
                    ptrs.append(0)
                else:
                    base, pitch = geo[id(h[0])]
                    ptrs.append(base + pitch * h[1])
            missing = [i for i, q in enumerate(ptrs) if not q]
            if len(missing) < n:
                any_row = next(q for q in ptrs if q)
                copy_rows(out, [q if q else any_row for q in ptrs])   # missing slots overwritten below
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
