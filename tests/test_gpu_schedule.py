"""Cholesky schedule invariance: the classic column schedule and the ahead schedule (partial sums
of the next column's tiles computed one launch early, in 1 / 2 / 4 row slices, the diagonal
target's in 1 / 2 block slices) redistribute the same MFMA chains over workgroups and launches,
the two solve kernels (k_solve: one workgroup per individual; k_solve_chain: an individual's
block rows and tiles over the chip, chosen for small batches) share one arithmetic, and the
diagonal tile's last SYRK term runs the same MFMA chains whether the diagonal launch or the
previous launch's tile (J, J-1) workgroup computes it, the diagonal target's partial sum runs in
the off-diagonal launch or beside the diagonal one, and a tile's GEMM1 term L = Ls0 runs in its
T-unit or in an E-unit beside the diagonal launch, so fitness
and EBVs must be bit-identical under every setting, for both system forms and for system sizes
from 1 to 9 tile columns; and equal to the oracle.  (TBLUP_AHEAD / TBLUP_NRS / TBLUP_SOLVE_CHAIN /
TBLUP_SOLVE_PULL / TBLUP_LAST_TERM / TBLUP_PAD_FIRST / TBLUP_DIAG_D / TBLUP_DIAG_E are read when a context is created.)"""
import os

import numpy as np
import pytest

from oracle import blup_oracle as O

pytestmark = pytest.mark.gpu

SETTINGS = [
    {"TBLUP_AHEAD": "0"},                           # the classic (round-2) schedule
    {"TBLUP_AHEAD": "1", "TBLUP_NRS": "1"},
    {"TBLUP_AHEAD": "1", "TBLUP_NRS": "2"},
    {"TBLUP_AHEAD": "1", "TBLUP_NRS": "4"},
    {"TBLUP_AHEAD": "1", "TBLUP_NRS": "0"},
    {"TBLUP_AHEAD": "-1", "TBLUP_NRS": "0"},        # the defaults
    {"TBLUP_SOLVE_CHAIN": "1"},                     # SNP form: chained solve at every batch size
    {"TBLUP_SOLVE_CHAIN": "1", "TBLUP_SOLVE_PULL": "0"},   # ... its push units (block rows)
    {"TBLUP_SOLVE_CHAIN": "1", "TBLUP_SOLVE_PULL": "1"},   # ... its pull units (block columns), every trait count
    {"TBLUP_SOLVE_CHAIN": "0"},                     # one solve workgroup per individual
    {"TBLUP_LAST_TERM": "1"},                       # diagonal's last SYRK term in the previous launch
    {"TBLUP_LAST_TERM": "0"},                       # ... in the diagonal launch
    {"TBLUP_DIAG_D": "1"},                          # diagonal-target partials in the diagonal launches
    {"TBLUP_DIAG_D": "0"},                          # ... in the off-diagonal launches
    {"TBLUP_DIAG_E": "1"},                          # a GEMM1 term of every tile in the diagonal launch
    {"TBLUP_DIAG_E": "0"},                          # ... of none
    {"TBLUP_AHEAD": "0", "TBLUP_DIAG_E": "1"},      # ... from K (term L = 0) at every column
]


def _evaluate(geno, pheno, genomes, T, V, env, form=None, multi=None):
    from tblup_amd.engine import GpuBlupEngine
    keys = list(env) + ["TBLUP_FORM"]
    old = {k: os.environ.get(k) for k in keys}
    try:
        os.environ.update(env)
        if form is not None:
            os.environ["TBLUP_FORM"] = str(form)
        with GpuBlupEngine(geno, pheno if multi is None else multi, device=0) as eng:
            groups = genomes if isinstance(genomes[0], list) else [genomes]
            out = [eng.evaluate(g, T, V, 0.4, return_ebv=True) for g in groups]
            return np.concatenate([o[0] for o in out]), np.concatenate([o[1] for o in out])
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def panel():
    rng = np.random.default_rng(21)
    n, p = 2000, 20_000
    geno = O.synth_geno(rng, n, p)
    pheno = rng.standard_normal(n)
    perm = rng.permutation(n)
    return {"geno": geno, "pheno": pheno, "T": perm[:1280], "V": perm[1280:1600], "rng": rng}


@pytest.mark.parametrize("form", [None, 1])
def test_schedules_are_bit_identical(panel, gpu, form):
    """k from 100 (1 tile column) to 1100 (9): SNP form (default) and kernel form (TBLUP_FORM=1:
    int8 K inside the units, whole-tile partials) -- every setting gives the same bits."""
    rng = np.random.default_rng(5)
    # one batch per system size (the batch's largest k sets the tile columns) and a mixed one
    groups = [[rng.choice(20_000, k, replace=False) for _ in range(6)] for k in (100, 250, 640, 1000, 1100)]
    groups.append([rng.choice(20_000, k, replace=False) for k in (383, 1000, 777, 900, 128, 1024)])
    genomes = [g for grp in groups for g in grp]
    ref = None
    for env in SETTINGS:
        fit, ebv = _evaluate(panel["geno"], panel["pheno"], groups, panel["T"], panel["V"], env, form)
        if ref is None:
            ref = (fit, ebv)
            continue
        np.testing.assert_array_equal(fit, ref[0], err_msg=str(env))
        np.testing.assert_array_equal(ebv, ref[1], err_msg=str(env))
    for i in (0, 14, 25, 31):
        f, e = O.blup_grm_form(genomes[i], panel["T"], panel["V"], panel["geno"], panel["pheno"], 0.4)
        assert abs(ref[0][i] - f) <= 1e-9


def test_schedules_small_batches_and_traits(panel, gpu):
    """Batches of 1, 3 and 40 individuals (the ahead schedule's auto row slicing changes with B),
    3 traits: identical to the round-2 schedule."""
    rng = np.random.default_rng(6)
    multi = np.stack([panel["pheno"], rng.standard_normal(2000), rng.standard_normal(2000)], axis=1)
    for B in (1, 3, 40):
        genomes = [rng.choice(20_000, 1000, replace=False) for _ in range(B)]
        a = _evaluate(panel["geno"], None, genomes, panel["T"], panel["V"], SETTINGS[0], multi=multi)
        for env in SETTINGS[-5:]:
            b = _evaluate(panel["geno"], None, genomes, panel["T"], panel["V"], env, multi=multi)
            np.testing.assert_array_equal(a[0], b[0], err_msg=str(env))
            np.testing.assert_array_equal(a[1], b[1], err_msg=str(env))


def test_leading_padding_matches_trailing(panel, gpu):
    """SNP form: padding rows leading the system (the default: the contractions over block column 0
    skip them) or trailing it (TBLUP_PAD_FIRST=0) -- the same systems with moved block boundaries,
    so equal up to rounding, and both equal to the oracle.  Batches with one k (pad 24 < 128) and
    with mixed k (pads up to 896: whole padding tiles skipped)."""
    rng = np.random.default_rng(8)
    groups = [[rng.choice(20_000, 1000, replace=False) for _ in range(5)],
              [rng.choice(20_000, k, replace=False) for k in (128, 1000, 777, 1024, 901, 420)]]
    genomes = [g for grp in groups for g in grp]
    lead = _evaluate(panel["geno"], panel["pheno"], groups, panel["T"], panel["V"], {})
    trail = _evaluate(panel["geno"], panel["pheno"], groups, panel["T"], panel["V"], {"TBLUP_PAD_FIRST": "0"})
    np.testing.assert_allclose(lead[0], trail[0], rtol=0, atol=1e-11)
    np.testing.assert_allclose(lead[1], trail[1], rtol=1e-9, atol=1e-9)
    for i in range(len(genomes)):
        f, _ = O.blup_grm_form(genomes[i], panel["T"], panel["V"], panel["geno"], panel["pheno"], 0.4)
        assert abs(lead[0][i] - f) <= 1e-9, i


def test_last_term_mask_past_32_columns(gpu):
    """a kernel-form system with more than 32 tile columns (n_T = 4224: NT = 33) at
    B <= 64, where the automatic last-term mask is every diagonal launch J >= 1 -- including
    J = 32, whose bit a 32-bit shift used to wrap to bit 0.  Every setting gives the same bits
    (the last term moves between launches on the same MFMA chains), equal to the oracle."""
    rng = np.random.default_rng(33)
    n, p = 4400, 6000
    geno = O.synth_geno(rng, n, p)
    pheno = rng.standard_normal(n)
    perm = rng.permutation(n)
    T, V = perm[:4224], perm[4224:4324]
    genomes = [rng.choice(p, 4300, replace=False), rng.choice(p, 4250, replace=False)]   # k > n_T: kernel form
    ref = _evaluate(geno, pheno, genomes, T, V, {"TBLUP_LAST_TERM": "0"})
    for env in ({"TBLUP_LAST_TERM": "-1"}, {"TBLUP_LAST_TERM": "1"}):
        got = _evaluate(geno, pheno, genomes, T, V, env)
        np.testing.assert_array_equal(got[0], ref[0])
        np.testing.assert_array_equal(got[1], ref[1])
    f, e = O.blup(genomes[0], T, V, geno.astype(np.float64), pheno, 0.4, return_ebv=True)
    assert abs(ref[0][0] - f) <= 1e-9
    assert np.max(np.abs(ref[1][0] - e)) <= 1e-9 * np.max(np.abs(e))
