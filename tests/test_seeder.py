"""Top-SNPs seeder (tblup/seeder.py): the host arithmetic on oracle moments (CPU) and the
GPU scan (k_snp_scan through tblup_snp_scan) against the reference's goldens."""
import os

import numpy as np
import pytest

from tblup_amd import seeder as S

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "seed.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


class OracleScan:
    """TEST INFRASTRUCTURE: the per-SNP moments in numpy (stands in for the GPU scan)."""

    def __init__(self, X, labels=None, device=0):
        self.X = np.asarray(X)

    def snp_scan(self, rows, yc):
        x = self.X[np.asarray(rows)].astype(np.float64)
        return x.sum(0).astype(np.int64), (x * x).sum(0).astype(np.int64), yc @ x

    def close(self):
        pass


class Ev:
    def __init__(self, t):
        self.training_indices = list(t)


def _paths(gold, tmp_path):
    gp, pp = tmp_path / "g.npy", tmp_path / "y.npy"
    np.save(gp, gold["geno"])
    np.save(pp, gold["pheno"])
    return str(gp), str(pp)


def _check_f(gold, eng):
    rows = gold["f_rows"]
    F, p = S.f_regression_rows(eng, rows, gold["pheno"][rows])
    assert np.allclose(F, gold["f_F"], rtol=1e-12, atol=0) and np.allclose(p, gold["f_p"], rtol=1e-10, atol=1e-300)
    assert F[7] == 0.0 and p[7] == 1.0   # monomorphic SNP: sklearn's force_finite values
    assert np.allclose(S.f_score(eng, rows, gold["pheno"][rows]), gold["f_score"], rtol=1e-12, atol=0)


def _check_seeders(gold, gp, pp):
    strat = S.TopSNPsSeedStrategy(Ev(gold["training_indices"]), S.p_value, gp, pp)
    assert np.array_equal(strat.indices, gold["sorted_indices"])
    np.random.seed(8)
    it = iter(S.RandomKeySeeder(strat, 40, gold["geno"].shape[1]))
    assert np.array_equal(np.stack([next(it) for _ in range(3)]), gold["rk_genomes"])
    it = iter(S.IndexSeeder(strat, 900))
    assert np.array_equal(np.stack([next(it) for _ in range(2)]), gold["index_genomes"])
    assert np.array_equal(next(it), gold["index_random_tail"])
    assert np.array_equal(np.asarray(np.random.get_state()[1], np.uint32), gold["mt_key"])


def test_f_regression_host_arithmetic(gold):
    _check_f(gold, OracleScan(gold["geno"]))


def test_seeders_host_logic(gold, tmp_path, monkeypatch):
    import tblup_amd.engine as E
    monkeypatch.setattr(E, "GpuBlupEngine", OracleScan)
    _check_seeders(gold, *_paths(gold, tmp_path))


def test_get_seeder_factory(gold, tmp_path, monkeypatch):
    import tblup_amd.engine as E
    from types import SimpleNamespace
    monkeypatch.setattr(E, "GpuBlupEngine", OracleScan)
    gp, pp = _paths(gold, tmp_path)
    a = SimpleNamespace(seeder=None)
    assert S.get_seeder(a, Ev(gold["training_indices"])) is None
    a = SimpleNamespace(seeder="top_snps", seeder_metric="p_value", SEED_METRIC_P_VALUE="p_value",
                        SEED_STRATEGY_TOP_SNPS="top_snps", features=40, initial_features=None, geno=gp, pheno=pp,
                        individual="randkeys", INDIVIDUAL_TYPE_INDEX="index", INDIVIDUAL_TYPE_NULLABLE="nullable",
                        INDIVIDUAL_TYPE_RANDOM_KEYS="randkeys", INDIVIDUAL_TYPE_COEVOLE="coevolve",
                        dimensionality=gold["geno"].shape[1])
    sd = S.get_seeder(a, Ev(gold["training_indices"]))
    assert isinstance(sd, S.RandomKeySeeder) and sd.length == 40
    a.seeder_metric = "nope"
    with pytest.raises(NotImplementedError):
        S.get_seeder(a, Ev(gold["training_indices"]))


@pytest.mark.gpu
def test_f_regression_gpu_scan(gold, gpu):
    from tblup_amd.engine import GpuBlupEngine
    with GpuBlupEngine(gold["geno"], gold["pheno"]) as eng:
        _check_f(gold, eng)
        rows = np.random.default_rng(0).integers(0, 300, size=5000)   # repeats, > one LDS stage
        yc = np.random.default_rng(1).standard_normal(5000)
        sx, sxx, sxy = eng.snp_scan(rows, yc)
        x = gold["geno"][rows].astype(np.float64)
        assert np.array_equal(sx, x.sum(0)) and np.array_equal(sxx, (x * x).sum(0))
        assert np.allclose(sxy, yc @ x, rtol=1e-12, atol=1e-9)


@pytest.mark.gpu
def test_seeders_gpu(gold, gpu, tmp_path):
    _check_seeders(gold, *_paths(gold, tmp_path))
