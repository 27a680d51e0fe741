"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

A numpy restatement of the reference's GBLUP/SNP-BLUP fitness path
(ianwhale/tblup).  Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may import this module, and only as the
checker / the timed CPU baseline.  The product path (`tblup_amd`) never
imports it and fails loudly if its HIP library is missing.

Pinning: every function here is checked against golden vectors produced by
running the reference itself in the build container
(`tests/golden/make_golden.py` -> `tests/golden/*.npz`, test
`tests/test_oracle.py`).  Third-party arithmetic the reference delegates to
(numpy 2.2.6 / scipy 1.15.3 / scikit-learn 1.7.2, unpinned `>=` bounds in the
reference's requirements.txt:1-3) is restated from its published algorithm:

* `scipy.stats.pearsonr` (scipy 1.15.3 `_stats_py.py`): exact-equality
  constant check -> NaN, mean-centre, max-abs scaled norms, clip to [-1, 1],
  round when n == 2.
* `sklearn.linear_model.Ridge(alpha).fit/predict` with fit_intercept=True,
  solver 'auto' -> 'cholesky' on dense input (scikit-learn 1.7.2
  `_ridge.py::_solve_cholesky` when n_features <= n_samples, else
  `_solve_cholesky_kernel`): centre X and y by their training means, solve
  (X^T X + alpha I) w = X^T y (or the kernel form), intercept = ybar - xbar.w.
"""
import numpy as np
import scipy.linalg


# ----------------------------------------------------------------------------
# GRM (tblup/utils.py:7-18)
# ----------------------------------------------------------------------------
def make_grm(geno):
    """VanRaden GRM with p = column mean / 2 over all rows passed in.

    Follows tblup/utils.py:7-18: W = (Z - 1) - (2p - 1) = Z - 2p and
    G = W W^T / (2 sum p (1 - p)).
    """
    z = np.asarray(geno, dtype=np.float64)
    p = z.mean(axis=0) / 2.0
    w = z - 2.0 * p
    return (w @ w.T) / (2.0 * np.sum(p * (1.0 - p)))


# ----------------------------------------------------------------------------
# Pearson correlation (scipy.stats.pearsonr restated)
# ----------------------------------------------------------------------------
def pearson_r(x, y):
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    n = x.shape[0]
    if n < 2:
        raise ValueError("x and y must have length at least 2.")
    if np.all(x == x[0]) or np.all(y == y[0]):
        return float("nan")
    xm = x - x.mean()
    ym = y - y.mean()
    xmax = np.max(np.abs(xm))
    ymax = np.max(np.abs(ym))
    nx = xmax * np.linalg.norm(xm / xmax)
    ny = ymax * np.linalg.norm(ym / ymax)
    r = float(np.sum((xm / nx) * (ym / ny)))
    r = min(max(r, -1.0), 1.0)
    if n == 2:
        r = float(np.round(r))
    return r


# ----------------------------------------------------------------------------
# The two BLUP branches (tblup/evaluator.py:244-314)
# ----------------------------------------------------------------------------
def gblup(indices, train, valid, data, labels, h2, return_ebv=False):
    """GBLUP branch, tblup/evaluator.py:265-286.

    GRM over all n rows, Ginv = inv(G_TT + lambda I), pred = G[:, T] Ginv y_T,
    fitness = |pearson(y_V, pred_V)|.  The LU inverse is replaced by a
    Cholesky solve of the same SPD system (same solution to rounding).
    """
    train = np.asarray(train)
    valid = np.asarray(valid)
    G = make_grm(np.asarray(data)[:, np.asarray(indices)])
    lam = (1.0 - h2) / h2
    A = G[np.ix_(train, train)].copy()
    A.flat[:: A.shape[0] + 1] += lam
    y_t = np.asarray(labels, dtype=np.float64)[train]
    with np.errstate(all="ignore"):
        try:
            alpha = scipy.linalg.solve(A, y_t, assume_a="pos")
        except (np.linalg.LinAlgError, ValueError):
            alpha = np.full(len(train), np.nan)
        ebv = G[np.ix_(valid, train)] @ alpha
    fit = abs(pearson_r(np.asarray(labels, dtype=np.float64)[valid], ebv))
    return (fit, ebv) if return_ebv else fit


def _ridge_predict(x_train, y_train, x_valid, alpha):
    """sklearn Ridge(alpha, fit_intercept=True, solver='cholesky') restated."""
    x_off = x_train.mean(axis=0)
    y_off = y_train.mean()
    xc = x_train - x_off
    yc = y_train - y_off
    n_samples, n_features = xc.shape
    with np.errstate(all="ignore"):
        if n_features > n_samples:
            K = xc @ xc.T
            K.flat[:: n_samples + 1] += alpha
            try:
                dual = scipy.linalg.solve(K, yc, assume_a="pos")
            except (np.linalg.LinAlgError, ValueError):
                dual = np.full(n_samples, np.nan)
            coef = xc.T @ dual
        else:
            A = xc.T @ xc
            A.flat[:: n_features + 1] += alpha
            try:
                coef = scipy.linalg.solve(A, xc.T @ yc, assume_a="pos")
            except (np.linalg.LinAlgError, ValueError):
                coef = np.full(n_features, np.nan)
        intercept = y_off - x_off @ coef
        return x_valid @ coef + intercept


def snp_blup(indices, train, valid, data, labels, h2, return_ebv=False):
    """SNP-BLUP branch, tblup/evaluator.py:288-314.

    p from the training rows only, X_T -= 2p and X_V -= 2p,
    Ridge(alpha = (1-h2)/(h2/d)) with d = 2 sum p(1-p),
    fitness = |pearson(pred_V, y_V)|.
    """
    train = np.asarray(train)
    valid = np.asarray(valid)
    x = np.asarray(data, dtype=np.float64)[:, np.asarray(indices)]
    y = np.asarray(labels, dtype=np.float64)
    x_t, x_v = x[train], x[valid]
    p = x_t.mean(axis=0) / 2.0
    d = 2.0 * np.sum(p * (1.0 - p))
    with np.errstate(all="ignore"):
        alpha = (1.0 - h2) / (h2 / d)
    x_t = x_t - 2.0 * p
    x_v = x_v - 2.0 * p
    ebv = _ridge_predict(x_t, y[train], x_v, alpha)
    fit = abs(pearson_r(ebv, y[valid]))
    return (fit, ebv) if return_ebv else fit


def blup(indices, train, valid, data, labels, h2, return_ebv=False):
    """Branch dispatch of tblup/evaluator.py:257: GBLUP iff k > n (total rows)."""
    if len(indices) > np.asarray(data).shape[0]:
        return gblup(indices, train, valid, data, labels, h2, return_ebv)
    return snp_blup(indices, train, valid, data, labels, h2, return_ebv)


# ----------------------------------------------------------------------------
# Unified GRM-form restatement (the identity the GPU pipeline implements)
# ----------------------------------------------------------------------------
def blup_grm_form(indices, train, valid, geno, labels, h2, branch="auto"):
    """Both branches as one kernel-form system, in exact integer arithmetic.

    With A the gathered {0,1,2} columns, m_s the column sums over the
    reference rows (all n rows for gblup, train rows for snp) and N their
    count:  K d = A_R A_T^T - (u_R + u_T)/N + q/N^2, u = A m, q = sum m^2,
    d = sum m/N - q/(2 N^2).  Solve (K_TT + lambda I) a = y_T - mu with
    mu = 0 (gblup) or mean(y_T) (snp); EBV_V = K_VT a + mu.
    """
    geno = np.asarray(geno)
    idx = np.asarray(indices, dtype=np.int64)
    n = geno.shape[0]
    if branch == "auto":
        branch = "gblup" if len(idx) > n else "snp"
    train = np.asarray(train)
    valid = np.asarray(valid)
    # float64 products of {0,1,2} data are exact integers here (all sums < 2^53),
    # so BLAS gives the same exact values as integer arithmetic, much faster.
    a = geno[:, idx].astype(np.float64)
    ref = np.arange(n) if branch == "gblup" else train
    N = float(len(ref))
    m = a[ref].sum(axis=0)                       # exact integer column sums
    u = a @ m                                    # exact integer row dots
    q = float(np.sum(m * m))
    d = float(np.sum(m)) / N - q / (2.0 * N * N)
    at, av = a[train], a[valid]
    with np.errstate(all="ignore"):
        ktt = ((at @ at.T) - (u[train][:, None] + u[train][None, :]) / N + q / (N * N)) / d
        kvt = ((av @ at.T) - (u[valid][:, None] + u[train][None, :]) / N + q / (N * N)) / d
        lam = (1.0 - h2) / h2
        ktt.flat[:: ktt.shape[0] + 1] += lam
        y = np.asarray(labels, dtype=np.float64)
        mu = 0.0 if branch == "gblup" else float(np.mean(y[train]))
        try:
            alpha = scipy.linalg.solve(ktt, y[train] - mu, assume_a="pos")
        except (np.linalg.LinAlgError, ValueError):
            alpha = np.full(len(train), np.nan)
        ebv = kvt @ alpha + mu
    return abs(pearson_r(ebv, y[valid])), ebv


def grm_block(indices, train, valid, geno, branch="auto"):
    """K_{R,T} (R = T then V) of the unified form, without the lambda shift."""
    geno = np.asarray(geno)
    idx = np.asarray(indices, dtype=np.int64)
    n = geno.shape[0]
    if branch == "auto":
        branch = "gblup" if len(idx) > n else "snp"
    a = geno[:, idx].astype(np.float64)
    ref = np.arange(n) if branch == "gblup" else np.asarray(train)
    N = float(len(ref))
    m = a[ref].sum(axis=0)
    u = a @ m
    q = float(np.sum(m * m))
    d = float(np.sum(m)) / N - q / (2.0 * N * N)
    rows = np.concatenate([np.asarray(train), np.asarray(valid)])
    ar, at = a[rows], a[np.asarray(train)]
    return ((ar @ at.T) - (u[rows][:, None] + u[np.asarray(train)][None, :]) / N
            + q / (N * N)) / d


# ----------------------------------------------------------------------------
# Genome decode (tblup/individual.py)
# ----------------------------------------------------------------------------
def decode_randkeys(keys, length):
    """RandomKeyIndividual.genome, individual.py:154-156."""
    return np.argsort(np.asarray(keys))[-int(length):]


def decode_index(genome):
    """IndexIndividual.genome, individual.py:93-95 (truncation, duplicates kept)."""
    return np.asarray(genome).astype(int)


def decode_nullable(genome, dimensionality):
    """NullableIndexIndividual.genome, individual.py:230-237."""
    g = np.asarray(genome)
    keep = np.logical_and(0 <= g, g < dimensionality)
    return np.extract(keep, g).astype(int)


def coevolution_fitness(fitness, gamma, length, dimensionality):
    """CoevolutionIndividual.set_fitness penalty, individual.py:215-222."""
    return fitness - gamma * (length / dimensionality)


# ----------------------------------------------------------------------------
# Synthetic data
# ----------------------------------------------------------------------------
def synth_geno(rng, n, p, maf_lo=0.05, maf_hi=0.5, dtype=np.int8):
    maf = rng.uniform(maf_lo, maf_hi, size=p)
    return rng.binomial(2, maf, size=(n, p)).astype(dtype)
