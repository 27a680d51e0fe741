"""Drop-in population seeder (tblup/seeder.py) whose GWAS metric runs on the GPU.

The reference ranks every SNP once at start-up by a univariate regression
metric cross-validated over 5 folds of the training animals
(`SeedStrategy.get_sorted_indices`, seeder.py:144-160): sklearn `f_regression`
on `X[train]` per fold, i.e. a full n x P pass over the genotypes in float64 per
fold.  Here the data pass is `k_snp_scan` (per-SNP exact sum x, sum x^2 and fp64
sum x*yc over the fold's animals, int8 genotypes resident on the GPU) and the
F statistic / p-value are formed on the host exactly as sklearn 1.7.2 forms
them from those moments (`r_regression`/`f_regression`, center=True,
force_finite=True; p from scipy's F survival function).  The seeders and the
top-SNPs strategy keep the reference's classes, RNG use and quirks (the fold
positions index X directly, seeder.py:157-158).

The scores match the reference to ~1e-15 relative (the y @ X product is summed
in a different order than BLAS); the SNP ranking is identical unless two SNPs'
scores differ by less than that (tests/test_seeder.py).
"""
import abc
import os

import numpy as np


def get_seeder(args, evaluator):
    """seeder.py:7-42."""
    if args.seeder is None:
        return None
    length = args.features if args.initial_features is None else args.initial_features
    metric = None
    if args.seeder_metric == args.SEED_METRIC_P_VALUE:
        metric = p_value
    if metric is None:
        raise NotImplementedError("Metric {} not implemented.".format(args.seeder_metric))
    strategy = None
    if args.seeder == args.SEED_STRATEGY_TOP_SNPS:
        strategy = TopSNPsSeedStrategy(evaluator, metric, args.geno, args.pheno)
    if strategy is None:
        raise NotImplementedError("Strategy {} not implemented.".format(args.seeder))
    if args.individual in (args.INDIVIDUAL_TYPE_INDEX, args.INDIVIDUAL_TYPE_NULLABLE):
        return IndexSeeder(strategy, length)
    if args.individual in (args.INDIVIDUAL_TYPE_RANDOM_KEYS, args.INDIVIDUAL_TYPE_COEVOLE):
        return RandomKeySeeder(strategy, length, args.dimensionality)
    raise NotImplementedError("Seeder {} not implemented.".format(args.seeder))


# --------------------------------------------------------------------- seeders
class Seeder(abc.ABC):
    """Iterator of initial genomes (seeder.py:49-71)."""

    def __init__(self, strategy, length):
        assert isinstance(strategy, SeedStrategy)
        self.strategy = strategy
        self.length = length

    @abc.abstractmethod
    def __next__(self):
        raise NotImplementedError()

    def __iter__(self):
        self.strategy.reset()
        return self


class IndexSeeder(Seeder):
    """seeder.py:74-80."""

    def __next__(self):
        return self.strategy.get_next_indices(self.length)


class RandomKeySeeder(Seeder):
    """Random keys with the next best SNPs' keys set to 1 (seeder.py:83-103)."""

    def __init__(self, strategy, length, dimensionality):
        super().__init__(strategy, length)
        self.dimensionality = dimensionality

    def __next__(self):
        genome = np.random.rand(self.dimensionality)
        genome[self.strategy.get_next_indices(self.length)] = 1
        return genome


# ------------------------------------------------------------------ strategies
class SeedStrategy(abc.ABC):
    """seeder.py:110-160."""

    N_SPLITS = 5

    def __init__(self, evaluator, metric, geno_path, pheno_path):
        try:
            self.training_indices = evaluator.training_indices
        except AttributeError:
            raise AttributeError("The provided evaluator {} does not calculate training indices, which are needed "
                                 "for a seeder to filter the data.".format(evaluator.__class__.__name__))
        self.metric = metric
        self.indices = self.get_sorted_indices(geno_path, pheno_path)

    @abc.abstractmethod
    def get_next_indices(self, length):
        raise NotImplementedError()

    @abc.abstractmethod
    def reset(self):
        raise NotImplementedError()

    def get_sorted_indices(self, geno_path, pheno_path):
        """Scores summed over KFold(5) of the training positions, SNPs in descending score
        order (np.flip of np.argsort, as the reference).  The fold positions index the
        genotype rows directly, like the reference's X[train] (seeder.py:157-158)."""
        from sklearn.model_selection import KFold
        from .engine import GpuBlupEngine
        X, y = np.load(geno_path), np.load(pheno_path)
        y = np.asarray(y)
        scores = np.zeros(X.shape[1])
        eng = GpuBlupEngine(X, np.zeros(X.shape[0]), device=int(os.environ.get("LOCAL_RANK", "0")))
        try:
            for train, _ in KFold(n_splits=self.N_SPLITS).split(self.training_indices):
                scores += self.metric(eng, train, y[train].ravel())
        finally:
            eng.close()
        return np.flip(np.argsort(scores, axis=0), 0)


class TopSNPsSeedStrategy(SeedStrategy):
    """seeder.py:163-199."""

    def __init__(self, evaluator, metric, geno_path, pheno_path):
        super().__init__(evaluator, metric, geno_path, pheno_path)
        self.current_index = 0

    def get_next_indices(self, length):
        n = self.current_index
        self.current_index += length
        if self.current_index > len(self.indices):
            return np.random.choice(self.indices, length, replace=False)
        return self.indices[n:n + length]

    def reset(self):
        self.current_index = 0


# ---------------------------------------------------------------------- metrics
def f_regression_rows(engine, rows, y):
    """sklearn f_regression(X[rows], y) (1.7.2, center=True, force_finite=True) with X the
    engine's genotype panel: the moments come from the GPU scan; the rest is sklearn's
    arithmetic in sklearn's order."""
    from scipy import stats
    y = np.asarray(y, dtype=np.float64).ravel()
    rows = np.asarray(rows, dtype=np.int64)
    n = rows.shape[0]
    yc = y - np.mean(y)
    sx, sxx, sxy = engine.snp_scan(rows, yc)
    x_means = sx.astype(np.float64) / n
    x_norms = np.sqrt(sxx.astype(np.float64) - n * x_means ** 2)
    r = sxy.copy()
    with np.errstate(divide="ignore", invalid="ignore"):
        r /= x_norms
        r /= np.linalg.norm(yc)
    r[np.isnan(r)] = 0.0
    dof = y.size - 2
    r2 = r ** 2
    with np.errstate(divide="ignore", invalid="ignore"):
        f = r2 / (1 - r2) * dof
        p = stats.f.sf(f, 1, dof)
    if not np.isfinite(f).all():
        f[np.isinf(f)] = np.finfo(f.dtype).max
        nan = np.isnan(f)
        f[nan] = 0.0
        p[nan] = 1.0
    return f, p


def p_value(engine, rows, y):
    """Negated p-values: a smaller p-value scores higher (seeder.py:200-209)."""
    return -1 * f_regression_rows(engine, rows, y)[1]


def f_score(engine, rows, y):
    """F statistics (seeder.py:211-220)."""
    return f_regression_rows(engine, rows, y)[0]
