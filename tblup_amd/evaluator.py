"""Drop-in evaluators for TBLUP's fitness plugin API, computed on MI355X.

Mirrors the reference module `tblup/evaluator.py` (ianwhale/tblup): the same
class names, constructor signatures, attributes the rest of TBLUP reads
(`training_indices`, `validation_indices`, `testing_indices`, `snp_remover`,
`data_path`, `labels_path`, `h2`, `archive`), the same RNG consumption for the
splits, the same archive/SNP-removal semantics and error behaviour.  What
changes is the compute leg: instead of `n_procs` worker processes each
running `blup()` on a private copy of the data (evaluator.py:120-131,
205-241), `__enter__` opens a GPU context (tblup_amd.engine.GpuBlupEngine) and
every `_evaluate` sends the whole batch of selected-index sets to the HIP
pipeline in one call.  Under torch.distributed (one process per GPU) the batch
is sharded across ranks and the fitnesses are all-gathered.

There is no CPU fallback: without the HIP library, entering the evaluator
raises ImportError.
"""
import abc
import os
import random
import weakref
from math import sqrt

import numpy as np

from . import _native
from .distributed import allgather_fitness, destroy, init_from_env, shard_range, world


def get_evaluator(args):
    """Factory with the reference's flag semantics (evaluator.py:14-55)."""
    splitter = None
    if args.splitter == "pca":
        # evaluator.py:22-24: decorate the splitter so only the data is passed later
        splitter = lambda data: pca_splitter(data, outliers=args.pca_outliers)  # noqa: E731
    r = args.features if args.removal_r is None else args.removal_r
    remover = SNPRemovalHandler(r, args.h2_alpha, args.heritability, args.remove_snps)
    common = dict(n_procs=args.processes, splitter=splitter, snp_remover=remover)
    pos = (args.geno, args.pheno, args.heritability)
    kind = args.regressor
    if kind == args.REGRESSOR_TYPE_BLUP:
        return BlupParallelEvaluator(*pos, **common)
    if kind == args.REGRESSOR_TYPE_INTRACV_BLUP:
        return IntraGCVBlupParallelEvaluator(*pos, n_folds=args.cv_folds, **common)
    if kind == args.REGRESSOR_TYPE_INTERCV_BLUP:
        return InterGCVBlupParallelEvaluator(*pos, n_folds=args.cv_folds, **common)
    if kind == args.REGRESSOR_TYPE_MONTECV_BLUP:
        return MonteCarloCVBlupParallelEvaluator(*pos, **common)
    raise NotImplementedError("Regressor with config option {} not implemented.".format(kind))


# ---------------------------------------------------------------------------
# Base classes
# ---------------------------------------------------------------------------
class Evaluator(abc.ABC):
    """Evaluator plugin interface (evaluator.py:63-99)."""

    def __init__(self, data_path, labels_path):
        assert os.path.isfile(data_path), "Argument for data_path {} not found.".format(data_path)
        assert os.path.isfile(labels_path), "Argument for labels_path {} not found.".format(labels_path)
        self.data_path = data_path
        self.labels_path = labels_path

    @abc.abstractmethod
    def __enter__(self):
        pass

    @abc.abstractmethod
    def __exit__(self, exc_type, exc_val, exc_tb):
        pass

    @abc.abstractmethod
    def evaluate(self, previous_population, next_population, generation):
        raise NotImplementedError()

    @abc.abstractmethod
    def genomes_to_evaluate(self, population):
        raise NotImplementedError()


class ParallelEvaluator(Evaluator):
    """Context-managed compute resource (evaluator.py:102-155).

    The reference spawns `n_procs` workers in __enter__; here __enter__ opens
    the GPU context for this process (device = `device`, else LOCAL_RANK, else 0).
    Launched one process per GPU (`torchrun main.py`, WORLD_SIZE > 1) it first creates
    the default process group (RCCL) unless the caller already has one, and then every
    batch of individuals is sharded across the ranks; __exit__ destroys a group it created.
    `n_procs` is kept for signature compatibility.
    """

    def __init__(self, data_path, labels_path, n_procs=-1, device=None):
        super().__init__(data_path, labels_path)
        self.n_procs = n_procs
        self.device = device
        self.engine = None
        self._owns_group = False

    def _device(self):
        if self.device is not None:
            return int(self.device)
        return int(os.environ.get("LOCAL_RANK", "0"))

    def _open_engine(self):
        from .engine import GpuBlupEngine  # loads libtblup_gpu.so or raises ImportError
        from .panel import load_panel
        # the float64 .npy streamed into int8 once per node (a /dev/shm segment every rank maps),
        # not a float64 copy per rank as evaluator.py:188 / 215-216 load it
        data = load_panel(self.data_path, self._device() if self._nccl() else None)
        labels = np.load(self.labels_path)
        return GpuBlupEngine(data, labels, device=self._device())

    @staticmethod
    def _nccl():
        import torch.distributed as dist
        return dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl"

    def __enter__(self):
        if init_from_env(self._device()):
            self._owns_group = True
        if self.engine is None:
            self.engine = self._open_engine()
        from .keystore import freeze_heap
        # the imported modules out of python's full collections (a 93 ms pause); undone in __exit__
        self._froze_heap = freeze_heap()
        return self

    def __exit__(self, exc_type, exc_val, exc_tb):
        if self.engine is not None:
            self.engine.close()
            self.engine = None
        if self._owns_group:
            self._owns_group = False
            destroy()
        if getattr(self, "_froze_heap", False):
            from .keystore import thaw_heap
            self._froze_heap = False
            thaw_heap()

    def genomes_to_evaluate(self, population):
        raise NotImplementedError()

    def evaluate(self, previous_population, next_population, generation):
        if self.engine is None:
            raise AttributeError("Workers are not set up.")


# ---------------------------------------------------------------------------
# BLUP evaluators
# ---------------------------------------------------------------------------
def _default_split(n_samples, train_test, train_valid):
    """Shuffled split with the reference's RNG consumption (evaluator.py:196-203):
    python `random.sample` for the shuffle, then two sklearn train_test_split
    calls drawing from numpy's global RNG."""
    from sklearn.model_selection import train_test_split

    order = random.sample(range(n_samples), n_samples)
    train, test = train_test_split(order, train_size=train_test, test_size=1 - train_test)
    train, valid = train_test_split(train, train_size=train_valid, test_size=1 - train_valid)
    return train, valid, test


class BlupParallelEvaluator(ParallelEvaluator):
    """GBLUP / SNP-BLUP fitness on MI355X (reference: evaluator.py:158-431)."""

    TRAIN_TEST_SPLIT = 0.8
    TRAIN_VALID_SPLIT = 0.8

    def __init__(self, data_path, labels_path, h2, n_procs=-1, splitter=None, snp_remover=None, device=None):
        super().__init__(data_path, labels_path, n_procs=n_procs, device=device)
        self.archive = {}
        self.snp_remover = snp_remover
        self.h2 = h2
        self._spec = None   # speculative evaluation of the last GPU DE generation (see _speculate)
        self.spec_fallbacks = 0   # speculative evaluations dropped after a chained-solve expiry
        data = np.load(data_path, mmap_mode="r")
        self.n_samples, self.n_columns = data.shape[0], data.shape[1]
        if splitter:
            self.training_indices, self.testing_indices = splitter(np.asarray(data))
            from sklearn.model_selection import train_test_split
            self.training_indices, self.validation_indices = train_test_split(
                self.training_indices, train_size=self.TRAIN_VALID_SPLIT, test_size=1 - self.TRAIN_VALID_SPLIT)
        else:
            self.training_indices, self.validation_indices, self.testing_indices = _default_split(
                self.n_samples, self.TRAIN_TEST_SPLIT, self.TRAIN_VALID_SPLIT)

    # -- the hot path -------------------------------------------------------
    def _fitness(self, genomes, train_indices, validation_indices):
        """Batched blup() over `genomes`; sharded across ranks under torch.distributed."""
        rank, ws = world()
        total = len(genomes)
        if ws == 1:
            return self.engine.evaluate(genomes, train_indices, validation_indices, self.h2)
        lo, hi = shard_range(total, rank, ws)
        return _gather_or_raise(lambda: self.engine.evaluate(genomes[lo:hi], train_indices, validation_indices,
                                                             self.h2),
                                (hi - lo,), total, getattr(self.engine, "device", None))

    @staticmethod
    def blup(indices, train_indices, validation_indices, data, labels, h2):
        """Single-individual blup (evaluator.py:244-263), used in-process by local search.

        Runs on the GPU through an engine cached per (data, labels) array pair.
        """
        eng = _static_engine(data, labels)
        return float(eng.evaluate([np.asarray(indices)], train_indices, validation_indices, h2)[0])

    @staticmethod
    def gblup(indices, train_indices, validation_indices, data, labels, h2):
        eng = _static_engine(data, labels)
        return float(eng.evaluate([np.asarray(indices)], train_indices, validation_indices, h2, branch="gblup")[0])

    @staticmethod
    def snp_blup(indices, train_indices, validation_indices, data, labels, h2):
        eng = _static_engine(data, labels)
        return float(eng.evaluate([np.asarray(indices)], train_indices, validation_indices, h2, branch="snp")[0])

    # -- reference control flow ---------------------------------------------
    def train_validation_indices(self, generation):
        return self.training_indices, self.validation_indices

    def __getstate__(self):
        return {k: v for k, v in self.__dict__.items()
                if k not in ("archive", "pool", "engine", "_owns_group", "_spec")}

    def genomes_to_evaluate(self, population):
        """Individuals whose uid is not archived (evaluator.py:339-357)."""
        if self.snp_remover is not None and self.snp_remover.should_remove():
            return self.snp_remover.genomes_to_evaluate(population, self.archive)
        todo, where = [], []
        for i, indv in enumerate(population):
            if indv.uid not in self.archive:
                where.append(i)
                todo.append(indv)
        return self._batch_genomes(todo), where, False

    _GPU_DECODE_TYPES = ("RandomKeyIndividual", "CoevolutionIndividual")

    def _batch_genomes(self, individuals):
        """`indv.genome` for a batch.  RandomKey / Coevolution individuals
        (individual.py:154-156: argsort(keys)[-int(length):]) are decoded on the GPU in one
        call (k_decode_topk); equal keys order by index, the set numpy returns unless a tie
        straddles the k-th key (continuous keys; DE clipping only creates ties at 0)."""
        dec = getattr(self.engine, "decode_randkey", None)
        if dec is not None and individuals and all(
                type(i).__name__ in self._GPU_DECODE_TYPES and hasattr(i, "_genome") for i in individuals):
            keys = [np.asarray(i._genome, dtype=np.float64) for i in individuals]
            d = keys[0].shape[0]
            lens = [int(i.length) for i in individuals]
            if all(k.ndim == 1 and k.shape[0] == d for k in keys) and all(1 <= n <= min(d, 8192) for n in lens):
                # keys the GPU DE step left on the device (tblup_amd.keystore) decode in place
                from .keystore import DeviceKeyStore
                import torch
                with torch.cuda.device(self.engine.device):
                    dev = DeviceKeyStore.get(self.engine.device).gather(individuals, d)
                    if dev is not None:
                        idx, off = self.engine.decode_randkey_tensor(dev, d, lens)
                    else:
                        idx, off = dec(np.stack(keys), lens)
                return [idx[off[j]:off[j + 1]] for j in range(len(individuals))]
        return [i.genome for i in individuals]

    # -- speculative evaluation of a GPU DE generation -----------------------------
    _SPEC_TYPES = ("RandomKeyIndividual",)

    def _speculate(self, parents, keys, generation):
        """Called by tblup_amd.evolver right after its DE kernel, with the children's keys still
        on the device: enqueue their decode and evaluation now (GpuBlupEngine.eval_keys_async)
        so the GPU computes the fitnesses while the host copies the children's genomes.
        evaluate() takes the result only when it is asked for exactly these children,
        unchanged, at this generation; otherwise it is dropped and evaluate() runs as usual.
        Only where evaluate() is a pure function of the genomes: the fixed split or InterGCV
        folds (no RNG draws), no SNP removal, RandomKey individuals.  Under torch.distributed
        every rank holds the same children (the DE step is replicated) and evaluates its own
        shard of them; evaluate() all-gathers the shards, as _fitness does."""
        self._spec = None
        if self.engine is None or type(self) not in (BlupParallelEvaluator, InterGCVBlupParallelEvaluator):
            return False
        if not hasattr(self.engine, "eval_keys_async") or not parents:
            return False
        if self.snp_remover is not None and self.snp_remover.should_remove():
            return False
        if not all(type(p).__name__ in self._SPEC_TYPES for p in parents):
            return False
        L = keys.shape[1]
        lens = [int(p.length) for p in parents]
        if not all(1 <= k <= min(L, 8192) for k in lens) or keys.device.index != self.engine.device:
            return False
        train, valid = self.train_validation_indices(generation)
        rank, ws = world()
        lo, hi = shard_range(len(lens), rank, ws)
        if hi > lo:
            event, host, status = self.engine.eval_keys_async(keys[lo:hi], lens[lo:hi], train, valid, self.h2)
        else:   # more ranks than children: nothing to evaluate here, the all-gather still runs
            event, host, status = None, None, None
        self._spec = {"generation": generation, "keys": keys, "lens": lens, "event": event, "host": host,
                      "status": status, "inds": None, "shard": (lo, hi)}
        return True

    def _spec_bind(self, children):
        if self._spec is not None:
            self._spec["inds"] = list(children)

    def _take_spec(self, population, generation):
        spec, self._spec = self._spec, None
        if spec is None or spec["inds"] is None or spec["generation"] != generation:
            return None
        inds = [population[i] for i in range(len(population))]
        if len(inds) != len(spec["inds"]) or any(a is not b for a, b in zip(inds, spec["inds"])):
            return None
        if any(i.uid in self.archive or int(i.length) != k for i, k in zip(inds, spec["lens"])):
            return None
        # genomes untouched since the DE step: the key store still maps child i to row i of the keys
        from .keystore import DeviceKeyStore
        hits = DeviceKeyStore.get(self.engine.device).rows(inds)
        if any(h is None or h[0] is not spec["keys"] or h[1] != i for i, h in enumerate(hits)):
            return None
        status = np.zeros(2, dtype=np.int64)
        if spec["event"] is not None:
            spec["event"].synchronize()
            status = spec["status"].numpy().astype(np.int64)
            local = spec["host"].numpy().copy()
        else:
            local = np.zeros(0, dtype=np.float64)
        if world()[1] > 1:
            # every rank takes the same decision here (replicated state): one all-gather, which carries
            # every rank's status words, so a failure on any rank is seen by all of them
            local, status = allgather_fitness(local, len(inds), getattr(self.engine, "device", None), status=status)
        if status[0]:   # an index outside [-P, P): numpy's IndexError, on every rank
            self.engine.raise_status((status[0], 0), n_snps=self.engine.n_snps)
        if status[1]:
            # a chained-solve wait expired in the speculative (device-entry) evaluation: drop it;
            # evaluate() then evaluates these children through the synchronous entry, which
            # re-solves an expired chunk by itself (tblup_chain_recoveries) -- same bits
            self.spec_fallbacks += 1
            return None
        return local

    def evaluate(self, previous_population, next_population, generation):
        """evaluator.py:359-378."""
        super().evaluate(previous_population, next_population, generation)
        fits = self._take_spec(next_population, generation)
        if fits is not None:   # the children's fitnesses, computed while their genomes were copied
            for i, f in enumerate(fits):
                next_population[i].set_fitness(f)
                self.archive[next_population[i].uid] = next_population[i].fitness
            return next_population
        todo, where, reevaluate = self.genomes_to_evaluate(next_population)
        next_population = self._evaluate(next_population, todo, where, generation)
        if reevaluate:
            todo, where, _ = self.genomes_to_evaluate(previous_population)
            self._evaluate(previous_population, todo, where, generation)
            previous_population.monitor.log_snp_removal_event(generation)
        return next_population

    def _evaluate(self, population, to_evaluate, indices, generation):
        """evaluator.py:380-405, one batched GPU call instead of the queue fan-out."""
        train, valid = self.train_validation_indices(generation)
        fits = self._fitness(list(to_evaluate), train, valid) if to_evaluate else []
        for i, f in zip(indices, fits):
            population[i].set_fitness(f)
            self.archive[population[i].uid] = population[i].fitness
        return population

    def evaluate_testing(self, population):
        """Testing accuracy with train = T u V and the genome merged with removed SNPs
        (evaluator.py:407-431); returned in population order."""
        if self.engine is None:
            raise AttributeError("Workers are not set up.")
        train = np.concatenate((self.training_indices, self.validation_indices))
        genomes = []
        for indv in population:
            if self.snp_remover is not None:
                genomes.append(self.snp_remover.combine_with_removed(indv.genome))
            else:   # same sorted-unique genome the reference's empty remover yields
                genomes.append(np.union1d(indv.genome, np.array([])).astype(int))
        return list(self._fitness(genomes, train, self.testing_indices))


class InterGCVBlupParallelEvaluator(BlupParallelEvaluator):
    """Validation fold rotates with the generation (evaluator.py:434-491)."""

    def __init__(self, data_path, labels_path, h2, n_procs=-1, n_folds=5, splitter=None, snp_remover=None,
                 device=None):
        super().__init__(data_path, labels_path, h2, n_procs=n_procs, splitter=splitter, snp_remover=snp_remover,
                         device=device)
        self.n_folds = n_folds
        self.fold_indices = self.make_fold_indices(self.training_indices, self.n_folds)

    @staticmethod
    def make_fold_indices(indices, n_folds):
        """Contiguous folds, the first len % n_folds one element longer; fold i is the
        validation set and the others, in order, the training set (evaluator.py:454-483)."""
        n = len(indices)
        sizes = [n // n_folds + (1 if i < n % n_folds else 0) for i in range(n_folds)]
        bounds = np.concatenate(([0], np.cumsum(sizes))).astype(int)
        folds = [list(indices[bounds[i]:bounds[i + 1]]) for i in range(n_folds)]
        out = []
        for i in range(n_folds):
            train = []
            for j in range(n_folds):
                if j != i:
                    train += folds[j]
            out.append([train, folds[i]])
        return out

    def train_validation_indices(self, generation):
        return self.fold_indices[generation % self.n_folds]


class IntraGCVBlupParallelEvaluator(InterGCVBlupParallelEvaluator):
    """k-fold CV inside every fitness evaluation; fitness = mean over folds (evaluator.py:494-537).
    The k folds' evaluations go to the GPU as one batch (GpuBlupEngine.evaluate_folds)."""

    def _fold_fitness(self, genomes):
        """(n_folds, len(genomes)) fitness; sharded across ranks like _fitness."""
        splits = [self.train_validation_indices(k) for k in range(self.n_folds)]
        folds = getattr(self.engine, "evaluate_folds", None)
        if folds is None:   # engines without the batched entry (test stand-ins): one call per fold
            return np.array([self._fitness(genomes, t, v) for t, v in splits])
        rank, ws = world()
        if ws == 1:
            return folds(genomes, splits, self.h2)
        lo, hi = shard_range(len(genomes), rank, ws)
        # every fold's block in one all-gather
        return _gather_or_raise(lambda: np.asarray(folds(genomes[lo:hi], splits, self.h2)).reshape(self.n_folds, hi - lo),
                                (self.n_folds, hi - lo), len(genomes), getattr(self.engine, "device", None))

    def _evaluate(self, population, to_evaluate, indices, generation):
        sums = {i: 0 for i in indices}
        per_fold = self._fold_fitness(list(to_evaluate)) if to_evaluate else [[] for _ in range(self.n_folds)]
        for k in range(self.n_folds):
            for i, f in zip(indices, per_fold[k]):
                sums[i] += f
        for i, s in sums.items():
            population[i].set_fitness(s / self.n_folds)
            self.archive[population[i].uid] = population[i].fitness
        return population


class MonteCarloCVBlupParallelEvaluator(BlupParallelEvaluator):
    """Fresh random 80/20 split of T u V on every _evaluate (evaluator.py:540-561)."""

    def __init__(self, data_path, labels_path, h2, n_procs=-1, splitter=None, snp_remover=None, device=None):
        super().__init__(data_path, labels_path, h2, n_procs=n_procs, splitter=splitter, snp_remover=snp_remover,
                         device=device)
        self.indices = np.concatenate((self.training_indices, self.validation_indices))

    def train_validation_indices(self, generation):
        from sklearn.model_selection import train_test_split
        return train_test_split(self.indices, test_size=0.2)


def _gather_or_raise(evaluate, shape, n_total, device):
    """This rank's shard evaluated, then the all-gather (torch.distributed).  A failure of the
    shard's evaluation -- an index outside [-P, P) in one rank's genomes, or any other exception
    (a torch / ctypes error, a ValueError from a genome's shape, device memory) -- would otherwise
    raise on that rank only and leave its peers waiting in the collective: the error code travels
    in the same all-gather, every rank leaves it together, the failing rank re-raises its own
    exception and the others raise TblupError (TblupIndexError for an index error)."""
    err = None
    try:
        local = evaluate()
    except Exception as e:   # noqa: BLE001 -- re-raised below, after the collective
        err = e
        local = np.full(shape, np.nan)
    code = 0 if err is None else (1 if isinstance(err, IndexError) else 2)
    full, st = allgather_fitness(local, n_total, device, status=(code,))
    if st[0]:
        if err is not None:
            raise err
        cls = _native.TblupIndexError if st[0] == 1 else _native.TblupError
        raise cls("tblup_eval_batch", _native.ERR_INDEX if st[0] == 1 else _native.ERR_STATE,
                  "the evaluation failed on another rank" + (" (an index is out of bounds for axis 1)"
                                                            if st[0] == 1 else ""))
    return full


# ---------------------------------------------------------------------------
# SNP removal (evaluator.py:569-633)
# ---------------------------------------------------------------------------
class SNPRemovalHandler:
    """Removes the best individual's SNPs from evaluation once its fitness passes
    sqrt(h2) * (1 + alpha)."""

    def __init__(self, r, alpha, h2, remove_snps):
        self.r = r
        self.threshold = sqrt(h2) * (1 + alpha)
        self.removed = np.array([])
        self.remove_snps = remove_snps

    def should_remove(self):
        return self.remove_snps

    def genomes_to_evaluate(self, population, archive):
        todo, where = [], []
        best = max(population, key=lambda x: x.fitness)
        triggered = best.fitness > self.threshold
        if triggered:
            count = len(best) if self.r < len(best) else self.r
            self.removed = np.union1d(self.removed, best.genome[-count:])
            for key in list(archive.keys()):   # flush in place: the evaluator keeps its reference
                del archive[key]
        for i, indv in enumerate(population):
            if indv.uid in archive:
                continue
            kept = np.setdiff1d(indv.genome, self.removed)
            if len(kept) == 0:   # every selected SNP removed: fitness 0 without evaluation
                archive[indv.uid] = 0.0
                indv.set_fitness(0.0)
            else:
                where.append(i)
                todo.append(kept)
        return todo, where, triggered

    def combine_with_removed(self, genome):
        return np.union1d(genome, self.removed).astype(int)


# ---------------------------------------------------------------------------
# engine cache for the static blup() entry points
# ---------------------------------------------------------------------------
_STATIC = {}


def _static_engine(data, labels):
    key = (id(data), id(labels))
    hit = _STATIC.get(key)
    if hit is not None:
        dref, lref, eng = hit
        if dref() is data and lref() is labels:
            return eng
    from .engine import GpuBlupEngine
    eng = GpuBlupEngine(data, labels, device=int(os.environ.get("LOCAL_RANK", "0")))
    try:
        dref, lref = weakref.ref(data), weakref.ref(labels)
    except TypeError:
        dref = lref = (lambda: None)
    # drop engines whose arrays are gone
    for k in [k for k, (d, l, _) in _STATIC.items() if d() is None or l() is None]:
        _STATIC.pop(k)[2].close()
    _STATIC[key] = (dref, lref, eng)
    return eng


# ---------------------------------------------------------------------------
# Splitters (evaluator.py:636-663)
# ---------------------------------------------------------------------------
def gpu_grm(data):
    """make_grm(data) (tblup/utils.py:7-18) over every SNP, on the GPU (int8 MFMA, exact
    integer A A^T + fp64 centring): a panel context opened for the call."""
    from .engine import GpuBlupEngine
    data = np.asarray(data)
    eng = GpuBlupEngine(data, np.zeros(data.shape[0]), device=int(os.environ.get("LOCAL_RANK", "0")))
    try:
        return eng.grm()
    finally:
        eng.close()


def pca_splitter(data, split=0.8, outliers=False, grm=None):
    """PCA splitter (evaluator.py:641-663): project the GRM onto its first two principal
    components (sklearn PCA, as the reference, including its use of numpy's global RNG by
    the randomized solver), sort animals by squared distance from the projected mean
    (descending when `outliers`), the first int(n * split) are the training animals.
    The n^2 P GRM runs on the GPU (`grm` overrides it: the tests pass the oracle's)."""
    from sklearn.decomposition import PCA
    G = gpu_grm(data) if grm is None else grm(data)
    proj = PCA(n_components=2)
    x = proj.fit_transform(G)
    centred = x - x.mean(axis=0)
    dist = centred[:, 0] ** 2 + centred[:, 1] ** 2
    # list.sort(key=dist, reverse=outliers) is stable in both directions: ties keep index order
    order = np.argsort(-dist if outliers else dist, kind="stable")
    cut = int(len(order) * split)
    return [int(i) for i in order[:cut]], [int(i) for i in order[cut:]]
