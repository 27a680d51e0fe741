"""GpuBlupEngine: one MI355X context holding the genotype panel in HBM.

This is the compute leg that replaces the reference's worker pool
(tblup/evaluator.py:205-241): instead of pickling one `blup` job per
individual onto an mp.Queue, a whole batch of selected-index sets goes to
`tblup_eval_batch` in one call.  Splits (train/validation animal lists) are
registered once and cached by content, so InterGCV folds, the testing split
and Monte-Carlo splits each pay the split build only when they change.
"""
import ctypes
import hashlib
from collections import OrderedDict

import numpy as np

from . import _native


def _as_int64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.int64))


def _ptr(a, ctype):
    return a.ctypes.data_as(ctypes.POINTER(ctype))


def validate_genotypes(data):
    """The GPU path stores genotypes as int8 {0,1,2} (SURVEY.md section 8a data contract).

    Raises ValueError for anything else (e.g. imputed dosages), instead of
    silently changing the arithmetic.
    """
    from .panel import convert_rows
    g = data if isinstance(data, np.ndarray) else np.asarray(data)
    if g.ndim != 2:
        raise ValueError("genotype matrix must be 2-D (animals x SNPs)")
    if g.dtype == np.int8:
        if g.size and (int(g.min()) < 0 or int(g.max()) > 2):
            raise ValueError("genotypes must take values in {0, 1, 2} for the MI355X evaluator")
        return np.ascontiguousarray(g)
    # converted by blocks of rows (tblup_amd.panel): no full-size boolean or float temporaries
    return convert_rows(g)


def concat_genomes(genomes):
    """Concatenate ragged index arrays -> (idx int64, offsets int64[B+1])."""
    lens = np.fromiter((len(g) for g in genomes), dtype=np.int64, count=len(genomes))
    offsets = np.zeros(len(genomes) + 1, dtype=np.int64)
    np.cumsum(lens, out=offsets[1:])
    if len(genomes):
        idx = np.concatenate([np.asarray(g, dtype=np.int64).ravel() for g in genomes])
    else:
        idx = np.zeros(0, dtype=np.int64)
    return np.ascontiguousarray(idx), offsets


class GpuBlupEngine:
    """Genotypes + phenotypes resident on one GPU; batched BLUP fitness."""

    MAX_SPLITS = 16   # a cached split is ~100 MB at config 2; IntraGCV holds k of them

    def __init__(self, data, labels, device=0, snp_major=False):
        """labels: (n,) phenotypes, or (n, t) for multi-trait evaluation (t <= 4, BASELINE
        config 5): one Cholesky per individual serves every trait, fitness = mean |r|."""
        self._lib = _native.load()
        geno = validate_genotypes(data)
        labels = np.asarray(labels, dtype=np.float64)
        if labels.ndim == 2 and labels.shape[1] == 1:
            labels = labels[:, 0]
        if labels.ndim not in (1, 2) or (labels.ndim == 2 and not 1 <= labels.shape[1] <= _native.MAX_TRAITS):
            raise ValueError(f"phenotypes must be (n,) or (n, t) with t <= {_native.MAX_TRAITS}")
        self.n_traits = 1 if labels.ndim == 1 else labels.shape[1]
        pheno = np.ascontiguousarray(labels[:, 0] if labels.ndim == 2 else labels)
        if snp_major:
            n_snps, n = geno.shape
            layout = _native.LAYOUT_SNP_MAJOR
        else:
            n, n_snps = geno.shape
            layout = _native.LAYOUT_ANIMAL_MAJOR
        if pheno.shape[0] != n:
            raise ValueError(f"phenotype length {pheno.shape[0]} != number of animals {n}")
        self.n_animals, self.n_snps, self.device = n, n_snps, int(device)
        ctx = ctypes.c_void_p()
        _native.check("tblup_ctx_create", self._lib.tblup_ctx_create(
            geno.ctypes.data_as(ctypes.c_void_p), n, n_snps, layout, _ptr(pheno, ctypes.c_double), self.device,
            ctypes.byref(ctx)))
        self._ctx = ctx
        if self.n_traits > 1:
            mt = np.ascontiguousarray(labels)
            _native.check("tblup_set_traits", self._lib.tblup_set_traits(
                self._ctx, _ptr(mt, ctypes.c_double), self.n_traits))
        self._splits = OrderedDict()   # key -> (split_id, n_valid)
        self._next_split = 0
        self._pending = None           # (event, keep-alive) of asynchronous work using the workspace
        self._spec_stream = None

    def _settle(self):
        """Wait for asynchronous work (eval_keys_async) that uses the context's workspace; every
        other entry point (the device-pointer ones included) calls this first, so calls stay
        serialised on the context whatever stream they are enqueued on."""
        p = self._pending
        if p is not None:
            self._pending = None
            p[0].synchronize()

    # ------------------------------------------------------------------ splits
    def split_id(self, train, valid, pinned=()):
        """Device id of the (train, valid) split, registered on first use; the cache keeps the
        MAX_SPLITS most recently used splits, never evicting the keys in `pinned` (the other
        splits of the same call: evaluate_folds)."""
        self._settle()
        t = _as_int64(train)
        v = _as_int64(valid)
        key = self._split_key(t, v)
        hit = self._splits.get(key)
        if hit is not None:
            self._splits.move_to_end(key)
            return hit[0]
        while len(self._splits) >= self.MAX_SPLITS:
            victim = next((k for k in self._splits if k not in pinned), None)
            if victim is None:   # every cached split belongs to this call: let the cache grow
                break
            old_id, _ = self._splits.pop(victim)
            _native.check("tblup_drop_split", self._lib.tblup_drop_split(self._ctx, old_id))
        sid = self._next_split
        self._next_split += 1
        _native.check("tblup_set_split", self._lib.tblup_set_split(
            self._ctx, sid, _ptr(t, ctypes.c_int64), len(t), _ptr(v, ctypes.c_int64), len(v)))
        self._splits[key] = (sid, len(v))
        return sid

    @staticmethod
    def _split_key(train, valid):
        return hashlib.sha1(_as_int64(train).tobytes() + b"|" + _as_int64(valid).tobytes()).hexdigest()

    def split_ids(self, splits):
        """split_id for every (train, valid) pair of one call; none of them evicts another, however
        many there are (the cache shrinks back to MAX_SPLITS on later registrations)."""
        pinned = {self._split_key(t, v) for t, v in splits}
        return [self.split_id(t, v, pinned) for t, v in splits]

    # -------------------------------------------------------------- evaluation
    def evaluate(self, genomes, train, valid, h2, branch="auto", return_ebv=False):
        """Fitness |pearson(EBV_V, y_V)| for each selected-index set (evaluator.py:244-314);
        multi-trait: the mean over traits, EBVs (B, t, n_valid)."""
        self._settle()
        sid = self.split_id(train, valid)
        idx, offsets = concat_genomes(genomes)
        B = len(genomes)
        fit = np.empty(B, dtype=np.float64)
        n_valid = len(valid)
        shape = (B, n_valid) if self.n_traits == 1 else (B, self.n_traits, n_valid)
        ebv = np.empty(shape, dtype=np.float64) if return_ebv else None
        if B:
            _native.check("tblup_eval_batch", self._lib.tblup_eval_batch(
                self._ctx, sid, _ptr(idx, ctypes.c_int64), _ptr(offsets, ctypes.c_int64), B, float(h2),
                _native.BRANCH[branch], _ptr(fit, ctypes.c_double),
                _ptr(ebv, ctypes.c_double) if return_ebv else None))
        return (fit, ebv) if return_ebv else fit

    def evaluate_folds(self, genomes, splits, h2, branch="auto"):
        """Every genome against each (train, valid) split in one call (tblup_eval_folds: the
        splits' evaluations back to back on the GPU, one round trip): (n_splits, B) fitness, row f
        bit-identical to evaluate(genomes, *splits[f]).  IntraGCV's k folds (evaluator.py:509-537)."""
        self._settle()
        sids = np.array(self.split_ids(splits), dtype=np.int32)
        idx, offsets = concat_genomes(genomes)
        B = len(genomes)
        fit = np.empty((len(sids), B), dtype=np.float64)
        if B:
            _native.check("tblup_eval_folds", self._lib.tblup_eval_folds(
                self._ctx, _ptr(sids, ctypes.c_int32), len(sids), _ptr(idx, ctypes.c_int64),
                _ptr(offsets, ctypes.c_int64), B, float(h2), _native.BRANCH[branch], _ptr(fit, ctypes.c_double)))
        return fit

    def evaluate_folds_device(self, split_ids, d_idx_ptr, d_off_ptr, h_offsets, h2, d_fit_ptr, stream_ptr=None,
                              branch="auto"):
        """Asynchronous evaluate_folds on device-resident buffers (d_fit: n_splits x B)."""
        self._settle()
        sids = np.ascontiguousarray(split_ids, dtype=np.int32)
        h_off = _as_int64(h_offsets)
        _native.check("tblup_eval_folds_device", self._lib.tblup_eval_folds_device(
            self._ctx, _ptr(sids, ctypes.c_int32), len(sids), ctypes.c_void_p(d_idx_ptr), ctypes.c_void_p(d_off_ptr),
            _ptr(h_off, ctypes.c_int64), len(h_off) - 1, float(h2), _native.BRANCH[branch],
            ctypes.c_void_p(d_fit_ptr), ctypes.c_void_p(stream_ptr) if stream_ptr else None))

    def evaluate_device(self, split_id, d_idx_ptr, d_off_ptr, h_offsets, h2, d_fit_ptr, d_ebv_ptr=None,
                        stream_ptr=None, branch="auto"):
        """Asynchronous evaluation on device-resident buffers (raw device pointers)."""
        self._settle()
        h_off = _as_int64(h_offsets)
        B = len(h_off) - 1
        _native.check("tblup_eval_batch_device", self._lib.tblup_eval_batch_device(
            self._ctx, split_id, ctypes.c_void_p(d_idx_ptr), ctypes.c_void_p(d_off_ptr),
            _ptr(h_off, ctypes.c_int64), B, float(h2), _native.BRANCH[branch], ctypes.c_void_p(d_fit_ptr),
            ctypes.c_void_p(d_ebv_ptr) if d_ebv_ptr else None,
            ctypes.c_void_p(stream_ptr) if stream_ptr else None))

    def index_error(self, stream_ptr=None):
        """True if an individual evaluated through evaluate_device since the last call had an
        index outside [-P, P) (its fitness is NaN); synchronises the stream, clears the flag."""
        self._settle()
        flag = ctypes.c_int(0)
        _native.check("tblup_index_error", self._lib.tblup_index_error(
            self._ctx, ctypes.c_void_p(stream_ptr) if stream_ptr else None, ctypes.byref(flag)))
        return bool(flag.value)

    def solve_error(self, stream_ptr=None):
        """True if a chained-solve hand-off wait expired in a device-entry evaluation since the
        last call (those fitnesses are invalid); synchronises the stream, clears the flag."""
        self._settle()
        flag = ctypes.c_int(0)
        _native.check("tblup_solve_error", self._lib.tblup_solve_error(
            self._ctx, ctypes.c_void_p(stream_ptr) if stream_ptr else None, ctypes.byref(flag)))
        return bool(flag.value)

    def check_device_status(self, stream_ptr=None):
        """Raise for a device-entry evaluation that failed: TblupIndexError for an index outside
        [-P, P) (numpy's IndexError), TblupError for an expired chained-solve wait."""
        if self.index_error(stream_ptr):
            raise _native.TblupIndexError("tblup_eval_batch_device", _native.ERR_INDEX,
                                          "an index is out of bounds for axis 1 with size %d" % self.n_snps)
        if self.solve_error(stream_ptr):
            raise _native.TblupError("tblup_eval_batch_device", _native.ERR_STATE, _native.CHAIN_EXPIRED)

    def status_async(self, host_status, stream_ptr=None):
        """Enqueue the copy of the device status words {index error, solve error} into the
        page-locked int32 tensor `host_status` (and clear them); read it after the stream's event."""
        _native.check("tblup_status_async", self._lib.tblup_status_async(
            self._ctx, ctypes.c_void_p(stream_ptr) if stream_ptr else None, ctypes.c_void_p(host_status.data_ptr())))

    def chain_recoveries(self):
        """Chunks the synchronous entries re-solved through k_solve after a chained-solve wait
        expired (tblup_chain_recoveries); the speculative path's fallbacks are counted by the
        evaluator (BlupParallelEvaluator.spec_fallbacks)."""
        v = ctypes.c_int64(0)
        _native.check("tblup_chain_recoveries", self._lib.tblup_chain_recoveries(self._ctx, ctypes.byref(v)))
        return v.value

    @staticmethod
    def raise_status(status, fn="tblup_eval_batch_device", n_snps=None):
        """Raise for nonzero status words read through status_async."""
        if int(status[0]):
            raise _native.TblupIndexError(fn, _native.ERR_INDEX, "an index is out of bounds for axis 1"
                                          + ("" if n_snps is None else " with size %d" % n_snps))
        if int(status[1]):
            raise _native.TblupError(fn, _native.ERR_STATE, _native.CHAIN_EXPIRED)

    def decode_randkey(self, keys, lengths):
        """RandomKeyIndividual.genome for a batch (individual.py:154-156) on the GPU:
        row i -> np.argsort(keys[i])[-int(lengths[i]):] (ascending key order; equal keys
        ordered by index, as a stable argsort).  Returns (idx, offsets) for evaluate_concat."""
        self._settle()
        kk = np.ascontiguousarray(np.asarray(keys, dtype=np.float64))
        if kk.ndim != 2:
            raise ValueError("keys must be (batch, d)")
        B, d = kk.shape
        lens = np.broadcast_to(np.asarray(lengths), (B,)).astype(np.int64)
        offsets = np.zeros(B + 1, dtype=np.int64)
        np.cumsum(lens, out=offsets[1:])
        idx = np.empty(int(offsets[-1]), dtype=np.int64)
        if B:
            _native.check("tblup_decode_topk", self._lib.tblup_decode_topk(
                self._ctx, _ptr(kk, ctypes.c_double), B, d, _ptr(offsets, ctypes.c_int64), _ptr(idx, ctypes.c_int64)))
        return idx, offsets

    def decode_randkey_device(self, d_keys_ptr, B, d, ld, d_off_ptr, h_offsets, d_idx_ptr, stream_ptr=None):
        """Device-resident decode: keys (B x ld doubles) -> idx at offsets (device pointers)."""
        self._settle()
        h_off = _as_int64(h_offsets)
        _native.check("tblup_decode_topk_device", self._lib.tblup_decode_topk_device(
            self._ctx, ctypes.c_void_p(d_keys_ptr), B, d, ld, ctypes.c_void_p(d_off_ptr), _ptr(h_off, ctypes.c_int64),
            ctypes.c_void_p(d_idx_ptr), ctypes.c_void_p(stream_ptr) if stream_ptr else None))

    def grm(self, indices=None):
        """make_grm(data[:, indices]) over all animals (tblup/utils.py:7-18) on the GPU:
        n x n float64.  indices=None: every SNP of the panel."""
        self._settle()
        idx = _as_int64(np.arange(self.n_snps) if indices is None else indices)
        G = np.empty((self.n_animals, self.n_animals), dtype=np.float64)
        _native.check("tblup_grm", self._lib.tblup_grm(self._ctx, _ptr(idx, ctypes.c_int64), len(idx),
                                                       _ptr(G, ctypes.c_double)))
        return G

    def snp_scan(self, rows, yc):
        """Per-SNP (sum x, sum x^2, sum x*yc) over animal `rows` (k_snp_scan)."""
        self._settle()
        r = _as_int64(rows)
        y = np.ascontiguousarray(yc, dtype=np.float64)
        if y.shape != r.shape:
            raise ValueError("yc must have one value per row")
        sx = np.empty(self.n_snps, dtype=np.int64)
        sxx = np.empty(self.n_snps, dtype=np.int64)
        sxy = np.empty(self.n_snps, dtype=np.float64)
        _native.check("tblup_snp_scan", self._lib.tblup_snp_scan(
            self._ctx, _ptr(r, ctypes.c_int64), len(r), _ptr(y, ctypes.c_double), _ptr(sx, ctypes.c_int64),
            _ptr(sxx, ctypes.c_int64), _ptr(sxy, ctypes.c_double)))
        return sx, sxx, sxy

    def decode_randkey_tensor(self, keys, d, lengths):
        """decode_randkey on a device tensor of key rows (B x ld float64, ld >= d, on this
        context's device) on torch's current stream; returns host (idx, offsets)."""
        self._settle()
        import torch
        from .keystore import work_stream
        B, ld = keys.shape
        lens = np.broadcast_to(np.asarray(lengths), (B,)).astype(np.int64)
        offsets = np.zeros(B + 1, dtype=np.int64)
        np.cumsum(lens, out=offsets[1:])
        ws = work_stream(keys.device.index)
        ws.wait_stream(torch.cuda.current_stream(keys.device))
        with torch.cuda.stream(ws):   # one stream for the copies and the library's kernel
            d_off = torch.from_numpy(offsets).to(keys.device)
            d_idx = torch.empty(int(offsets[-1]), dtype=torch.int64, device=keys.device)
            if B:
                self.decode_randkey_device(keys.data_ptr(), B, d, keys.stride(0), d_off.data_ptr(), offsets,
                                           d_idx.data_ptr(), ws.cuda_stream)
            out = d_idx.cpu().numpy()
        return out, offsets

    def evaluate_concat(self, idx, offsets, train, valid, h2, branch="auto"):
        """evaluate() on an already-concatenated (idx, offsets) batch."""
        self._settle()
        sid = self.split_id(train, valid)
        idx = _as_int64(idx)
        offsets = _as_int64(offsets)
        B = len(offsets) - 1
        fit = np.empty(B, dtype=np.float64)
        if B:
            _native.check("tblup_eval_batch", self._lib.tblup_eval_batch(
                self._ctx, sid, _ptr(idx, ctypes.c_int64), _ptr(offsets, ctypes.c_int64), B, float(h2),
                _native.BRANCH[branch], _ptr(fit, ctypes.c_double), None))
        return fit

    def debug_grm(self, indices, train, valid, h2, branch="auto", stage=1):
        """K_{R,T} (stage 1) or the factored block (stage 2) and z for one individual."""
        self._settle()
        sid = self.split_id(train, valid)
        idx = _as_int64(indices)
        nT, nV = len(train), len(valid)
        out = np.empty((nT + nV, nT), dtype=np.float64)
        z = np.empty(nT, dtype=np.float64)
        _native.check("tblup_debug_grm", self._lib.tblup_debug_grm(
            self._ctx, sid, _ptr(idx, ctypes.c_int64), len(idx), float(h2), _native.BRANCH[branch], int(stage),
            _ptr(out, ctypes.c_double), _ptr(z, ctypes.c_double)))
        return out, z

    def eval_keys_async(self, keys, lengths, train, valid, h2):
        """RandomKey individuals' fitness straight from a device tensor of their keys (B x ld
        float64 on this context's device): decode (k_decode_topk) and evaluation enqueued on a
        stream of this engine without waiting.  Returns (event, pinned host fitness tensor, pinned
        status words); both are valid once the event has completed (raise_status(status) then
        raises for a failed evaluation).  Later calls on the engine wait for it."""
        import torch
        self._settle()
        B, ld = keys.shape
        lens = np.asarray(lengths, dtype=np.int64)
        offsets = np.zeros(B + 1, dtype=np.int64)
        np.cumsum(lens, out=offsets[1:])
        sid = self.split_id(train, valid)
        dev = keys.device
        if self._spec_stream is None:
            self._spec_stream = torch.cuda.Stream(device=dev)
        st = self._spec_stream
        st.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.device(dev), torch.cuda.stream(st):
            d_off = torch.from_numpy(offsets).to(dev, non_blocking=True)
            d_idx = torch.empty(int(offsets[-1]), dtype=torch.int64, device=dev)
            d_fit = torch.empty(B, dtype=torch.float64, device=dev)
            self.decode_randkey_device(keys.data_ptr(), B, ld, keys.stride(0), d_off.data_ptr(), offsets,
                                       d_idx.data_ptr(), st.cuda_stream)
            self.evaluate_device(sid, d_idx.data_ptr(), d_off.data_ptr(), offsets, h2, d_fit.data_ptr(),
                                 stream_ptr=st.cuda_stream)
            host = torch.empty(B, dtype=torch.float64, pin_memory=True)
            host.copy_(d_fit, non_blocking=True)
            status = torch.zeros(2, dtype=torch.int32, pin_memory=True)
            self.status_async(status, st.cuda_stream)
            ev = torch.cuda.Event()
            ev.record(st)
        self._pending = (ev, (keys, d_off, d_idx, d_fit, offsets))
        return ev, host, status

    # --------------------------------------------------------------- profiling
    def set_profiling(self, enable=True):
        _native.check("tblup_set_profiling", self._lib.tblup_set_profiling(self._ctx, 1 if enable else 0))

    def reset_profile(self):
        _native.check("tblup_reset_profile", self._lib.tblup_reset_profile(self._ctx))

    def profile(self):
        n = _native.N_KCLASS
        ms = np.zeros(n)
        la = np.zeros(n, dtype=np.int64)
        fl = np.zeros(n)
        by = np.zeros(n)
        _native.check("tblup_get_profile", self._lib.tblup_get_profile(
            self._ctx, _ptr(ms, ctypes.c_double), _ptr(la, ctypes.c_int64), _ptr(fl, ctypes.c_double),
            _ptr(by, ctypes.c_double)))
        return {name: {"ms": float(ms[i]), "launches": int(la[i]), "flops": float(fl[i]), "bytes": float(by[i])}
                for i, name in enumerate(_native.KCLASS_NAMES)}

    def wg_trace(self, raw=False):
        """Per-workgroup records of the last evaluation's Cholesky launches and chained solve
        (TBLUP_WG_TRACE=1): structured array (start, end [s], kind, J, I, b, wait [s]); raw=True: the (n, 4) uint64 records
        (including each diagonal launch's phase-stamp block, kind 0)."""
        n = ctypes.c_int64(0)
        _native.check("tblup_get_wg_trace", self._lib.tblup_get_wg_trace(self._ctx, None, 0, ctypes.byref(n)))
        raw_out = raw
        raw = np.zeros((n.value, 4), dtype=np.uint64)
        if n.value:
            _native.check("tblup_get_wg_trace", self._lib.tblup_get_wg_trace(
                self._ctx, raw.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n.value, ctypes.byref(n)))
        if raw_out:
            return raw
        out = np.zeros(len(raw), dtype=[("start", "f8"), ("end", "f8"), ("kind", "i4"), ("J", "i4"), ("I", "i4"),
                                        ("b", "i8"), ("wait", "f8")])
        out["start"] = raw[:, 0] / 1e8
        out["end"] = raw[:, 1] / 1e8
        out["kind"] = (raw[:, 2] >> np.uint64(56)).astype(np.int32)
        out["I"] = ((raw[:, 2] >> np.uint64(40)) & np.uint64(0xFFFF)).astype(np.int32)
        out["b"] = (raw[:, 2] & np.uint64((1 << 40) - 1)).astype(np.int64)
        out["J"] = (raw[:, 3] & np.uint64(0xFFFF)).astype(np.int32)
        out["wait"] = (raw[:, 3] >> np.uint64(16)) / 1e8      # chained-solve units: first wait done - start
        return out[out["kind"] != 0]

    def mem_in_use(self):
        v = ctypes.c_int64(0)
        _native.check("tblup_mem_info", self._lib.tblup_mem_info(self._ctx, ctypes.byref(v)))
        return v.value

    # ----------------------------------------------------------------- cleanup
    def close(self):
        if getattr(self, "_pending", None) is not None:
            self._settle()
        if getattr(self, "_ctx", None):
            self._lib.tblup_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
