"""BASELINE config 4 at full size: 5000 animals x 600k SNPs (3 GB of int8 genotypes), panel
k = 5000 (the snp branch in the kernel form: k = n, n_T = 3200 < k).

P * n = 3.0e9 > 2^31, so this exercises the 64-bit offsets of the panel transpose
(k_transpose_geno), the split build (k_build_split: (P+1) x nRp = 2.5e9 bytes), the packed
rows and the gather of SNPs whose rows start beyond 2^31 bytes.  Parity against the
oracle's exact kernel form (oracle.blup_grm_form, evaluator.py:288-314) for individuals
drawn over the whole panel, from its last 100k SNPs only (all offsets > 2^31), with
duplicates and with negative (numpy-wrapped) indices; plus bit-determinism and
index-order invariance.
"""
import numpy as np
import pytest

from oracle import blup_oracle as O

N, P, K, NT, NV = 5000, 600_000, 5000, 3200, 800


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_config4_full_size_parity(gpu):
    from tblup_amd.engine import GpuBlupEngine
    rng = np.random.default_rng(44)
    geno = rng.integers(0, 3, size=(N, P), dtype=np.int8)
    pheno = rng.standard_normal(N)
    perm = rng.permutation(N)
    T, V = perm[:NT], perm[NT:NT + NV]
    whole = rng.choice(P, K, replace=False)
    tail = P - 100_000 + rng.choice(100_000, K, replace=False)          # rows at byte offsets > 2^31
    dup = np.concatenate([tail[:K // 2], tail[:K // 2]])                  # numpy gathers duplicates twice
    neg = whole.copy()
    neg[::3] -= P                                                        # -P <= i < 0 wraps to i + P
    genomes = [whole, tail, dup, neg]
    with GpuBlupEngine(geno, pheno, device=0) as eng:
        fit, ebv = eng.evaluate(genomes, T, V, 0.4, return_ebv=True)
        fit2 = eng.evaluate(genomes, T, V, 0.4)
        shuffled = [g[rng.permutation(len(g))] for g in genomes[:2]]
        fit_sh = eng.evaluate(shuffled, T, V, 0.4)
    np.testing.assert_array_equal(fit, fit2)                             # bit-deterministic
    np.testing.assert_allclose(fit_sh, fit[:2], rtol=0, atol=1e-12)      # index order is irrelevant
    assert fit[3] == fit[0]                                              # wrapped ids = the same columns
    for i in (0, 1, 2):
        f, e = O.blup_grm_form(genomes[i], T, V, geno, pheno, 0.4)
        assert abs(fit[i] - f) < 1e-9, (i, fit[i], f)
        assert np.max(np.abs(ebv[i] - e)) <= 1e-9 * np.max(np.abs(e)), i
