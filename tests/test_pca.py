"""PCA splitter (evaluator.py:641-663): host logic with the oracle GRM against the
reference's goldens (CPU), and the GPU GRM path (tblup_grm) against them (GPU)."""
import os

import numpy as np
import pytest

from oracle import blup_oracle as O
from tblup_amd.evaluator import pca_splitter

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pca.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def _check(gold, n, outl, grm):
    np.random.seed(50 + n)
    tr, te = pca_splitter(gold["pca_%d_geno" % n], outliers=outl, grm=grm)
    tag = "pca_%d_%s_" % (n, "out" if outl else "in")
    assert tr == list(gold[tag + "train"]) and te == list(gold[tag + "test"])
    st = np.random.get_state()   # the randomized solver draws from numpy's global RNG like the reference
    assert np.array_equal(np.asarray(st[1], np.uint32), gold[tag + "mt_key"]) and st[2] == int(gold[tag + "mt_pos"])


def test_oracle_grm_matches_reference(gold):
    for n in (200, 600):
        G = O.make_grm(gold["pca_%d_geno" % n])
        assert np.max(np.abs(G - gold["pca_%d_grm" % n])) <= 1e-12 * np.max(np.abs(gold["pca_%d_grm" % n]))


@pytest.mark.parametrize("n", [200, 600])
@pytest.mark.parametrize("outl", [False, True])
def test_pca_splitter_host_logic(gold, n, outl):
    _check(gold, n, outl, O.make_grm)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [200, 600])
@pytest.mark.parametrize("outl", [False, True])
def test_pca_splitter_gpu_grm(gold, gpu, n, outl):
    _check(gold, n, outl, None)


@pytest.mark.gpu
def test_gpu_grm_matches_make_grm(gold, gpu):
    from tblup_amd.engine import GpuBlupEngine
    for n in (200, 600):
        geno = gold["pca_%d_geno" % n]
        with GpuBlupEngine(geno, np.zeros(n)) as eng:
            G = eng.grm()
            sub = np.random.default_rng(n).choice(geno.shape[1], 300, replace=True)
            Gs = eng.grm(sub)
        ref = gold["pca_%d_grm" % n]
        assert np.max(np.abs(G - ref)) <= 1e-12 * np.max(np.abs(ref))
        assert np.array_equal(G, G.T)
        ref_s = O.make_grm(geno[:, sub])
        assert np.max(np.abs(Gs - ref_s)) <= 1e-12 * np.max(np.abs(ref_s))


@pytest.mark.gpu
def test_gpu_grm_config2_scale(gpu):
    """2000 x 50k (BASELINE config 2 panel): full GRM vs the oracle on a row sample."""
    from tblup_amd.engine import GpuBlupEngine
    rng = np.random.default_rng(2)
    geno = O.synth_geno(rng, 2000, 50000)
    with GpuBlupEngine(geno, np.zeros(2000)) as eng:
        G = eng.grm()
    z = geno.astype(np.float64)
    p = z.mean(axis=0) / 2
    rows = rng.choice(2000, 16, replace=False)
    W = z - 2 * p
    ref = W[rows] @ W.T / (2 * np.sum(p * (1 - p)))
    assert np.max(np.abs(G[rows] - ref)) <= 1e-11 * np.max(np.abs(ref))
