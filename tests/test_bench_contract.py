"""bench.py's self-check: the timed GPU fitnesses against the oracle fitnesses
the CPU baseline computed for the same genomes -- the comparison itself, on the CPU."""
import numpy as np

import bench


def test_fitness_parity_covers_and_flags():
    fit = np.array([0.1, 0.2, np.nan, 0.4])
    ok = bench.fitness_parity(fit, {0: 0.1, 1: 0.2 + 1e-13, 2: float("nan"), 3: 0.4}, 4)
    assert ok["covered"] == 4 and ok["of"] == 4
    assert ok["max_abs_fit"] <= 1e-12 and ok["max_abs_fit"] <= bench.PARITY_ATOL
    bad = bench.fitness_parity(fit, {0: 0.1, 2: 0.3}, 4)   # a NaN against a number: a mismatch
    assert bad["covered"] == 2 and bad["max_abs_fit"] == float("inf")
    off = bench.fitness_parity(fit, {1: 0.2 + 2e-9}, 4)
    assert off["max_abs_fit"] > bench.PARITY_ATOL
    assert bench.fitness_parity(fit, {}, 4)["max_abs_fit"] is None


def test_cpu_baseline_keeps_its_oracle_fitnesses(monkeypatch):
    """cpu_baseline's sample covers individual i % pop at evaluation i and returns their fitnesses."""
    rng = np.random.default_rng(0)
    n, P, k = 60, 300, 20
    geno = rng.integers(0, 3, size=(n, P)).astype(np.int8)
    pheno = rng.standard_normal(n)
    T, V = np.arange(40), np.arange(40, 55)
    genomes = np.stack([rng.choice(P, k, replace=False) for _ in range(3)])
    cpu = bench.cpu_baseline(geno, pheno, T, V, genomes, 0.4, 0.2)
    of = cpu["_oracle_fit"]
    assert sorted(of) == [0, 1, 2]
    from oracle.blup_oracle import blup
    for i in range(3):
        assert abs(of[i] - blup(genomes[i], T, V, geno.astype(np.float64), pheno, 0.4)) == 0.0
    assert cpu["host_cpus_affinity"] >= 1 and cpu["cores"] >= 1
