"""GPU parity: the HIP pipeline (through the C ABI) against the reference goldens and the oracle.

Tolerances (north star: EBVs within 1e-5 relative of the numpy reference):
  * GRM block K_{R,T}: max |dK| <= 1e-12 * max |K| (exact-integer A A^T + fp64 centring)
  * Cholesky factor / forward solve: <= 1e-10 relative
  * EBV_V: max |dEBV| <= 1e-9 * max |EBV| (well inside the 1e-5 bar); fitness |df| <= 1e-9
"""
import hashlib
import os

import numpy as np
import pytest

from oracle import blup_oracle as O

pytestmark = pytest.mark.gpu

EBV_RTOL = 1e-9
FIT_ATOL = 1e-9


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def _cases(z):
    return [(str(z["names"][i]), z["idx"][z["offsets"][i]:z["offsets"][i + 1]]) for i in range(len(z["names"]))]


@pytest.fixture(scope="module")
def small(golden_dir, gpu):
    from tblup_amd.engine import GpuBlupEngine
    z = _load(golden_dir, "blup_200x1000.npz")
    eng = GpuBlupEngine(z["geno"], z["pheno"], device=0)
    yield z, eng
    eng.close()


def _relmax(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def test_grm_block_matches_oracle(small):
    z, eng = small
    T, V, g = z["T"], z["V"], z["geno"]
    lam = (1 - 0.4) / 0.4
    for name, idx in _cases(z):
        K, _ = eng.debug_grm(idx, T, V, 0.4, stage=1)
        ref = O.grm_block(idx, T, V, g)
        ref[np.arange(len(T)), np.arange(len(T))] += lam
        assert _relmax(K, ref) <= 1e-12, name


def test_cholesky_factor_and_forward_solve(small):
    z, eng = small
    T, V, g, y = z["T"], z["V"], z["geno"], z["pheno"]
    lam = (1 - 0.4) / 0.4
    nT = len(T)
    for name, idx in _cases(z):
        F, zz = eng.debug_grm(idx, T, V, 0.4, stage=2)
        K = O.grm_block(idx, T, V, g)[:nT]
        K[np.arange(nT), np.arange(nT)] += lam
        L = np.linalg.cholesky(K)
        assert _relmax(np.tril(F[:nT]), L) <= 1e-10, name
        branch = "gblup" if len(idx) > g.shape[0] else "snp"
        mu = 0.0 if branch == "gblup" else float(np.mean(y[T]))
        zref = np.linalg.solve(L, y[T] - mu)
        assert _relmax(zz, zref) <= 1e-10, name


def test_fitness_and_ebv_vs_reference_goldens(small):
    """All cases in ONE ragged batch: mixed k, duplicates, both branches."""
    z, eng = small
    genomes = [idx for _, idx in _cases(z)]
    fit, ebv = eng.evaluate(genomes, z["T"], z["V"], float(z["h2"]), return_ebv=True)
    for i, (name, _) in enumerate(_cases(z)):
        assert abs(fit[i] - z["fitness"][i]) <= FIT_ATOL, name
        assert _relmax(ebv[i], z["ebv"][i]) <= EBV_RTOL, name


def test_testing_split_goldens(small):
    z, eng = small
    genomes = [idx for _, idx in _cases(z)]
    TV = np.concatenate([z["T"], z["V"]])
    fit, ebv = eng.evaluate(genomes, TV, z["X"], float(z["h2"]), return_ebv=True)
    for i, (name, _) in enumerate(_cases(z)):
        assert abs(fit[i] - z["test_fitness"][i]) <= FIT_ATOL, name
        assert _relmax(ebv[i], z["test_ebv"][i]) <= EBV_RTOL, name


def test_h2_sweep(small):
    z, eng = small
    c = _cases(z)
    for h, (fs, fg) in zip(z["h2_sweep"], z["h2_sweep_fitness"]):
        f = eng.evaluate([c[0][1], c[8][1]], z["T"], z["V"], float(h))
        assert abs(f[0] - fs) <= FIT_ATOL and abs(f[1] - fg) <= FIT_ATOL


def test_forced_branches_match_oracle(small):
    z, eng = small
    g, y, T, V = z["geno"].astype(np.float64), z["pheno"], z["T"], z["V"]
    idx = _cases(z)[0][1]
    f_g = eng.evaluate([idx], T, V, 0.4, branch="gblup")[0]
    f_s = eng.evaluate([idx], T, V, 0.4, branch="snp")[0]
    assert abs(f_g - O.gblup(idx, T, V, g, y, 0.4)) <= FIT_ATOL
    assert abs(f_s - O.snp_blup(idx, T, V, g, y, 0.4)) <= FIT_ATOL


def test_degenerate_panels_give_nan(golden_dir, gpu):
    from tblup_amd.engine import GpuBlupEngine
    z = _load(golden_dir, "blup_edge.npz")
    with GpuBlupEngine(z["geno"], z["pheno"]) as eng:
        sel = [np.arange(10, 20), np.tile(np.arange(10, 20), 21), np.arange(0, 10)]
        f = eng.evaluate(sel, z["T"], z["V"], 0.4)
        assert np.all(np.isnan(f)), f


def test_config2_shape_golden(golden_dir, gpu):
    from tblup_amd.engine import GpuBlupEngine
    z = _load(golden_dir, "blup_2000x4000.npz")
    geno = O.synth_geno(np.random.default_rng(int(z["seed"])), int(z["n"]), int(z["p"]))
    assert hashlib.sha256(geno.tobytes()).hexdigest() == str(z["geno_sha256"])
    genomes = [z["idx"][z["offsets"][i]:z["offsets"][i + 1]] for i in range(len(z["offsets"]) - 1)]
    with GpuBlupEngine(geno, z["pheno"]) as eng:
        fit, ebv = eng.evaluate(genomes, z["T"], z["V"], 0.4, return_ebv=True)
    for i in range(4):
        assert abs(fit[i] - z["fitness"][i]) <= FIT_ATOL
        ref = z["ebv"][i] if i < 3 else z["ebv_gblup"]
        assert _relmax(ebv[i], ref) <= EBV_RTOL


def test_chunked_workspace_is_identical(golden_dir, gpu, monkeypatch):
    """A tiny workspace budget forces many chunks; results must be bit-identical."""
    from tblup_amd.engine import GpuBlupEngine
    z = _load(golden_dir, "blup_200x1000.npz")
    genomes = [idx for _, idx in _cases(z)] * 3
    with GpuBlupEngine(z["geno"], z["pheno"]) as eng:
        ref = eng.evaluate(genomes, z["T"], z["V"], 0.4)
    monkeypatch.setenv("TBLUP_WORKSPACE_MB", "1")
    with GpuBlupEngine(z["geno"], z["pheno"]) as eng:
        got = eng.evaluate(genomes, z["T"], z["V"], 0.4)
    np.testing.assert_array_equal(got, ref)


def test_device_pointer_path_matches_host_path(small):
    import torch
    z, eng = small
    genomes = [idx for _, idx in _cases(z)]
    ref = eng.evaluate(genomes, z["T"], z["V"], 0.4)
    from tblup_amd.engine import concat_genomes
    idx, off = concat_genomes(genomes)
    sid = eng.split_id(z["T"], z["V"])
    d_idx = torch.from_numpy(idx).cuda()
    d_off = torch.from_numpy(off).cuda()
    d_fit = torch.empty(len(genomes), dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream()
    eng.evaluate_device(sid, d_idx.data_ptr(), d_off.data_ptr(), off, 0.4, d_fit.data_ptr(),
                        stream_ptr=stream.cuda_stream)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d_fit.cpu().numpy(), ref)


# ---------------------------------------------------------------------------
# Full BASELINE config-2 size: 2000 animals x 50k SNPs, k = 1000, 256 individuals
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def config2(gpu):
    from tblup_amd.engine import GpuBlupEngine
    rng = np.random.default_rng(2)
    n, P = 2000, 50_000
    geno = O.synth_geno(rng, n, P)
    pheno = rng.standard_normal(n)
    perm = np.random.default_rng(3).permutation(n)
    T, V = perm[:1280], perm[1280:1600]
    keys = np.random.default_rng(4).uniform(size=(256, P))
    genomes = [O.decode_randkeys(k, 1000) for k in keys]
    eng = GpuBlupEngine(geno, pheno)
    fit, ebv = eng.evaluate(genomes, T, V, 0.4, return_ebv=True)
    yield dict(geno=geno, pheno=pheno, T=T, V=V, genomes=genomes, fit=fit, ebv=ebv, eng=eng)
    eng.close()


def test_config2_sample_vs_oracle(config2):
    c = config2
    for i in (0, 1, 77, 128, 200, 255):
        f, e = O.blup_grm_form(c["genomes"][i], c["T"], c["V"], c["geno"], c["pheno"], 0.4)
        assert abs(c["fit"][i] - f) <= FIT_ATOL
        assert _relmax(c["ebv"][i], e) <= EBV_RTOL


def test_config2_properties(config2):
    """Size-independent properties at full size: determinism, batch independence,
    invariance to index order, finite fitness in [0, 1]."""
    c = config2
    eng = c["eng"]
    assert np.all(np.isfinite(c["fit"])) and np.all((c["fit"] >= 0) & (c["fit"] <= 1))
    again = eng.evaluate(c["genomes"], c["T"], c["V"], 0.4)
    np.testing.assert_array_equal(again, c["fit"])
    alone = eng.evaluate([c["genomes"][5]], c["T"], c["V"], 0.4)
    assert alone[0] == c["fit"][5]
    rng = np.random.default_rng(9)
    shuffled = [rng.permutation(c["genomes"][i]) for i in range(8)]
    f = eng.evaluate(shuffled, c["T"], c["V"], 0.4)
    np.testing.assert_allclose(f, c["fit"][:8], rtol=0, atol=1e-12)


def test_config2_device_entry_repeats(config2):
    """tblup_eval_batch_device on a side stream, repeated and with a shorter batch, gives the
    host entry's fitness bit for bit (the workspace is reused across calls)."""
    import torch
    from tblup_amd.engine import concat_genomes
    c = config2
    eng = c["eng"]
    sid = eng.split_id(c["T"], c["V"])
    idx, off = concat_genomes(c["genomes"])
    d_idx = torch.from_numpy(idx).cuda()
    d_off = torch.from_numpy(off).cuda()
    d_fit = torch.empty(len(c["genomes"]), dtype=torch.float64, device="cuda")
    s = torch.cuda.Stream()
    for h2, want in ((0.4, c["fit"]), (0.4, c["fit"]), (0.7, None)):
        d_fit.fill_(float("nan"))
        eng.evaluate_device(sid, d_idx.data_ptr(), d_off.data_ptr(), off, h2, d_fit.data_ptr(),
                            stream_ptr=s.cuda_stream)
        s.synchronize()
        got = d_fit.cpu().numpy()
        if want is None:
            want = eng.evaluate(c["genomes"], c["T"], c["V"], h2)
        np.testing.assert_array_equal(got, want)
    d_fit.fill_(float("nan"))
    eng.evaluate_device(sid, d_idx.data_ptr(), d_off.data_ptr(), off[:9], 0.4, d_fit.data_ptr(),
                        stream_ptr=s.cuda_stream)
    s.synchronize()
    np.testing.assert_array_equal(d_fit.cpu().numpy()[:8], c["fit"][:8])


def test_config2_folds_batched_equal_per_split(config2):
    """tblup_eval_folds (IntraGCV's k folds, evaluator.py:509-537, in one call): each row equals
    that split's own evaluation bit for bit, at config-2 size, host and device entries; an unknown
    split id is an argument error."""
    import torch
    from tblup_amd import _native
    from tblup_amd.engine import concat_genomes
    from tblup_amd.evaluator import InterGCVBlupParallelEvaluator
    c = config2
    eng = c["eng"]
    folds = InterGCVBlupParallelEvaluator.make_fold_indices(np.asarray(c["T"]), 5)
    genomes = c["genomes"][:96]
    got = eng.evaluate_folds(genomes, folds, 0.4)
    assert got.shape == (5, 96)
    for k, (t, v) in enumerate(folds):
        np.testing.assert_array_equal(got[k], eng.evaluate(genomes, t, v, 0.4))
    sids = [eng.split_id(t, v) for t, v in folds]
    idx, off = concat_genomes(genomes)
    d_idx, d_off = torch.from_numpy(idx).cuda(), torch.from_numpy(off).cuda()
    d_fit = torch.full((5, 96), float("nan"), dtype=torch.float64, device="cuda")
    s = torch.cuda.Stream()
    eng.evaluate_folds_device(sids, d_idx.data_ptr(), d_off.data_ptr(), off, 0.4, d_fit.data_ptr(),
                              stream_ptr=s.cuda_stream)
    s.synchronize()
    np.testing.assert_array_equal(d_fit.cpu().numpy(), got)
    with pytest.raises(_native.TblupError, match="unknown split"):
        eng.evaluate_folds_device([sids[0], 12345], d_idx.data_ptr(), d_off.data_ptr(), off, 0.4, d_fit.data_ptr())


def test_config2_folds_ragged_and_unfused(config2, monkeypatch):
    """Folds of unequal sizes (1277 train animals in 5 folds: 256, 256, 255, 255, 255) take the
    split-by-split path, folds of equal sizes the fold-fused one (one launch sequence of 5 x B
    systems, system tiles from the shared counts C_T - C_V_f); TBLUP_FOLD_SHARE=0 builds every
    fold's tiles from its own rows, TBLUP_FOLD_FUSE=0 runs split by split.  Every row equals that
    split's own evaluation bit for bit."""
    from tblup_amd.engine import GpuBlupEngine
    from tblup_amd.evaluator import InterGCVBlupParallelEvaluator
    c = config2
    eng = c["eng"]
    genomes = c["genomes"][:40]
    ragged = InterGCVBlupParallelEvaluator.make_fold_indices(np.asarray(c["T"])[:-3], 5)
    assert len({len(t) for t, _ in ragged}) == 2
    got = eng.evaluate_folds(genomes, ragged, 0.4)
    for k, (t, v) in enumerate(ragged):
        np.testing.assert_array_equal(got[k], eng.evaluate(genomes, t, v, 0.4))
    folds = InterGCVBlupParallelEvaluator.make_fold_indices(np.asarray(c["T"]), 5)
    fused = eng.evaluate_folds(genomes, folds, 0.4)
    for var in ("TBLUP_FOLD_SHARE", "TBLUP_FOLD_FUSE"):   # read at context creation
        monkeypatch.setenv(var, "0")
        eng2 = GpuBlupEngine(c["geno"], c["pheno"], device=0)
        try:
            np.testing.assert_array_equal(eng2.evaluate_folds(genomes, folds, 0.4), fused)
        finally:
            eng2.close()


def test_config2_gblup_branch_sample(config2):
    """k > n at config-2 size: the GBLUP branch (p over all n animals, no y centring)."""
    c = config2
    rng = np.random.default_rng(11)
    genomes = [rng.choice(50_000, 2500, replace=False) for _ in range(3)]
    fit, ebv = c["eng"].evaluate(genomes, c["T"], c["V"], 0.4, return_ebv=True)
    for i, g in enumerate(genomes):
        f, e = O.blup_grm_form(g, c["T"], c["V"], c["geno"], c["pheno"], 0.4)
        assert abs(fit[i] - f) <= FIT_ATOL
        assert _relmax(ebv[i], e) <= EBV_RTOL


# ---------------------------------------------------------------------------
# SNP-space (primal) form: sklearn's own Ridge solve when k <= n_T.  Forced with
# TBLUP_FORM=2 on the golden cases (mixed k, k = 1, duplicates, k > n_T), and
# selected automatically at config-2 shape (k = 1000 < n_T = 1280).
# ---------------------------------------------------------------------------
def _snp_cases(z):
    return [(i, name, idx) for i, (name, idx) in enumerate(_cases(z)) if str(z["branch"][i]) == "snp"]


@pytest.mark.parametrize("form", ["1", "2"])
def test_forced_form_matches_goldens(golden_dir, gpu, monkeypatch, form):
    from tblup_amd.engine import GpuBlupEngine
    z = _load(golden_dir, "blup_200x1000.npz")
    monkeypatch.setenv("TBLUP_FORM", form)
    cases = _snp_cases(z)
    assert len(cases) >= 6
    with GpuBlupEngine(z["geno"], z["pheno"]) as eng:
        fit, ebv = eng.evaluate([c[2] for c in cases], z["T"], z["V"], float(z["h2"]), return_ebv=True)
        TV = np.concatenate([z["T"], z["V"]])
        tfit, tebv = eng.evaluate([c[2] for c in cases], TV, z["X"], float(z["h2"]), return_ebv=True)
    for j, (i, name, _) in enumerate(cases):
        assert abs(fit[j] - z["fitness"][i]) <= FIT_ATOL, name
        assert _relmax(ebv[j], z["ebv"][i]) <= EBV_RTOL, name
        assert abs(tfit[j] - z["test_fitness"][i]) <= FIT_ATOL, name
        assert _relmax(tebv[j], z["test_ebv"][i]) <= EBV_RTOL, name


def test_forced_primal_degenerate_panels(golden_dir, gpu, monkeypatch):
    from tblup_amd.engine import GpuBlupEngine
    z = _load(golden_dir, "blup_edge.npz")
    monkeypatch.setenv("TBLUP_FORM", "2")
    with GpuBlupEngine(z["geno"], z["pheno"]) as eng:
        f = eng.evaluate([np.arange(10, 20), np.arange(0, 10)], z["T"], z["V"], 0.4, branch="snp")
        assert np.all(np.isnan(f)), f


def test_config2_shape_golden_primal(golden_dir, gpu):
    """The three snp genomes alone: auto-selects the primal form (k = 1000 < n_T = 1280)."""
    from tblup_amd.engine import GpuBlupEngine
    z = _load(golden_dir, "blup_2000x4000.npz")
    geno = O.synth_geno(np.random.default_rng(int(z["seed"])), int(z["n"]), int(z["p"]))
    genomes = [z["idx"][z["offsets"][i]:z["offsets"][i + 1]] for i in range(3)]
    assert all(len(g) <= len(z["T"]) - 128 for g in genomes)
    with GpuBlupEngine(geno, z["pheno"]) as eng:
        fit, ebv = eng.evaluate(genomes, z["T"], z["V"], 0.4, return_ebv=True)
    for i in range(3):
        assert abs(fit[i] - z["fitness"][i]) <= FIT_ATOL
        assert _relmax(ebv[i], z["ebv"][i]) <= EBV_RTOL


def test_config2_forms_agree(config2, monkeypatch):
    """Kernel (dual) form vs the auto-selected SNP (primal) form at full size."""
    from tblup_amd.engine import GpuBlupEngine
    c = config2
    monkeypatch.setenv("TBLUP_FORM", "1")
    sel = [c["genomes"][i] for i in range(0, 256, 32)]
    with GpuBlupEngine(c["geno"], c["pheno"]) as eng:
        fit, ebv = eng.evaluate(sel, c["T"], c["V"], 0.4, return_ebv=True)
    for j, i in enumerate(range(0, 256, 32)):
        assert abs(fit[j] - c["fit"][i]) <= FIT_ATOL
        assert _relmax(ebv[j], c["ebv"][i]) <= EBV_RTOL


# ---------------------------------------------------------------------------
# BASELINE config-4 shape (5000 animals, k = 5000 > n_T = 3200: the kernel form at 25
# tile columns), on a 50k-SNP panel (the 600k-SNP panel only adds HBM, not arithmetic)
# ---------------------------------------------------------------------------
def test_config4_shape_sample_vs_oracle(gpu):
    from tblup_amd.engine import GpuBlupEngine
    rng = np.random.default_rng(44)
    n, P = 5000, 50_000
    geno = O.synth_geno(rng, n, P)
    pheno = rng.standard_normal(n)
    perm = np.random.default_rng(45).permutation(n)
    T, V = perm[:3200], perm[3200:4000]
    genomes = [np.sort(rng.choice(P, 5000, replace=False)), rng.choice(P, 5000, replace=True),
               rng.choice(P, 5200, replace=False)]            # snp, snp with duplicates, gblup (k > n)
    with GpuBlupEngine(geno, pheno) as eng:
        fit, ebv = eng.evaluate(genomes, T, V, 0.4, return_ebv=True)
        again = eng.evaluate(genomes[:1], T, V, 0.4)
    assert again[0] == fit[0]
    for i, g in enumerate(genomes):
        f, e = O.blup_grm_form(g, T, V, geno, pheno, 0.4)
        assert abs(fit[i] - f) <= FIT_ATOL
        assert _relmax(ebv[i], e) <= EBV_RTOL


# ---------------------------------------------------------------------------
# Multi-trait (BASELINE config 5, build-defined): traits share K, one Cholesky, t RHS.
# Each trait's EBVs must equal that phenotype's single-trait evaluation (the reference's
# blup() per column); fitness = mean over traits of |r|.
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("form", ["0", "1", "2"])
def test_multitrait_equals_single_traits(golden_dir, gpu, monkeypatch, form):
    from tblup_amd.engine import GpuBlupEngine
    z = _load(golden_dir, "blup_200x1000.npz")
    monkeypatch.setenv("TBLUP_FORM", form)
    rng = np.random.default_rng(7)
    Y = np.stack([z["pheno"], rng.standard_normal(200), 0.5 * z["pheno"] + rng.standard_normal(200)], axis=1)
    genomes = [idx for _, idx in _cases(z)] if form != "2" else [c[2] for c in _snp_cases(z)]
    with GpuBlupEngine(z["geno"], Y) as eng:
        fit, ebv = eng.evaluate(genomes, z["T"], z["V"], 0.4, return_ebv=True)
    assert ebv.shape == (len(genomes), 3, len(z["V"]))
    singles = []
    for tr in range(3):
        with GpuBlupEngine(z["geno"], Y[:, tr]) as eng:
            singles.append(eng.evaluate(genomes, z["T"], z["V"], 0.4, return_ebv=True))
    for i, g in enumerate(genomes):
        fs = []
        for tr in range(3):
            np.testing.assert_array_equal(ebv[i, tr], singles[tr][1][i])
            fs.append(singles[tr][0][i])
            f, e = O.blup_grm_form(g, z["T"], z["V"], z["geno"], Y[:, tr], 0.4)
            assert _relmax(ebv[i, tr], e) <= EBV_RTOL
        assert abs(fit[i] - np.mean(fs)) <= 1e-15


def test_multitrait_config5_sample(config2):
    """Config 5 shape: 2000 x 50k, k = 1000 (SNP-space form), 3 traits."""
    from tblup_amd.engine import GpuBlupEngine
    c = config2
    rng = np.random.default_rng(55)
    Y = np.stack([c["pheno"], rng.standard_normal(2000), rng.standard_normal(2000)], axis=1)
    sel = [c["genomes"][i] for i in (0, 100, 255)]
    with GpuBlupEngine(c["geno"], Y) as eng:
        fit, ebv = eng.evaluate(sel, c["T"], c["V"], 0.4, return_ebv=True)
    for j, g in enumerate(sel):
        fs = []
        for tr in range(3):
            f, e = O.blup_grm_form(g, c["T"], c["V"], c["geno"], Y[:, tr], 0.4)
            assert _relmax(ebv[j, tr], e) <= EBV_RTOL
            fs.append(f)
        assert abs(fit[j] - np.mean(fs)) <= FIT_ATOL
    # trait 0 is the single-trait phenotype of the fixture
    np.testing.assert_array_equal(ebv[:, 0], c["ebv"][[0, 100, 255]])


# ---------------------------------------------------------------------------
# GPU genome decode: RandomKeyIndividual.genome =
# np.argsort(keys)[-k:] (individual.py:154-156) -- bit-exact indices, order included
# ---------------------------------------------------------------------------
def _stable_topk(keys, k):
    return np.argsort(keys, kind="stable")[-k:]


def test_decode_randkey_matches_numpy(small):
    _, eng = small
    rng = np.random.default_rng(21)
    d = 50_000
    keys = rng.uniform(size=(12, d))
    keys[3] = -keys[3]                                      # negative keys
    keys[4] *= 1e-300                                       # subnormal / tiny range
    lens = np.array([1000, 1000, 1, 2, 1000, 8192, 4097, 999, 1000, 1000, 50, 1000])
    idx, off = eng.decode_randkey(keys, lens)
    for i in range(12):
        got = idx[off[i]:off[i + 1]]
        np.testing.assert_array_equal(got, _stable_topk(keys[i], lens[i]))
        np.testing.assert_array_equal(got, np.argsort(keys[i])[-lens[i]:])   # continuous keys: numpy default too


def test_decode_randkey_ties(small):
    """Ties straddling the k-th key: stable-argsort semantics (largest indices win); numpy's
    default kind agrees on everything outside the straddling tie."""
    _, eng = small
    rng = np.random.default_rng(22)
    d = 20_000
    keys = np.round(rng.uniform(size=(6, d)), 2)            # ~100 distinct values: heavy ties
    keys[1] = 0.5                                           # all equal
    keys[2, :] = np.clip(rng.normal(size=d) * 3e4, 0, d - 1)   # DE-style clipping: ties at 0 and d-1
    lens = [1000, 777, 8192, 1, 8000, 20]
    idx, off = eng.decode_randkey(keys, lens)
    for i in range(6):
        got = idx[off[i]:off[i + 1]]
        np.testing.assert_array_equal(got, _stable_topk(keys[i], lens[i]))
        # against numpy's default kind (what individual.py:156 calls): its order inside a tie is
        # implementation-defined (introsort, or x86-simd-sort on AVX-512 hosts), so which of the
        # indices tied at the k-th key the reference selects depends on its host.  Pinned against
        # it: the selected key values in order, and every index whose key is above the k-th key.
        ref = np.argsort(keys[i])[-lens[i]:]
        np.testing.assert_array_equal(keys[i][got], keys[i][ref])
        kth = keys[i][ref[0]]
        np.testing.assert_array_equal(np.sort(got[keys[i][got] > kth]), np.sort(ref[keys[i][ref] > kth]))


def test_evaluator_gpu_decode_path(golden_dir, gpu, tmp_path):
    """BlupParallelEvaluator decodes RandomKey individuals on the GPU; fitness equals the
    host-decoded path and the reference flow golden."""
    import random
    from tblup_amd import evaluator as E
    from tests.helpers import KeyIndividual
    z = _load(golden_dir, "blup_200x1000.npz")
    flow = _load(golden_dir, "evaluator_flow.npz")
    gp, pp = str(tmp_path / "g.npy"), str(tmp_path / "p.npy")
    np.save(gp, z["geno"].astype(np.float64))
    np.save(pp, z["pheno"])

    class RandomKeyIndividual(KeyIndividual):   # the reference's class name triggers the GPU decode
        pass

    random.seed(3)
    np.random.seed(3)
    rem = E.SNPRemovalHandler(100, 0.0, 0.4, False)
    with E.BlupParallelEvaluator(gp, pp, 0.4, n_procs=2, snp_remover=rem) as ev:
        pop = [RandomKeyIndividual(k, 100) for k in flow["flow_keys"]]
        todo, where, _ = ev.genomes_to_evaluate(pop)
        for g, indv in zip(todo, pop):
            np.testing.assert_array_equal(g, indv.genome)
        ev.evaluate(pop, pop, 0)
        np.testing.assert_allclose([p.fitness for p in pop], flow["flow_fitness"], rtol=0, atol=FIT_ATOL)


def test_knockout_local_search_gpu(golden_dir, gpu, tmp_path):
    """KnockoutLocalSearch (local.py:50-76) with speculative GPU batches = the sequential
    oracle walk."""
    import random
    from tblup_amd import evaluator as E
    from tblup_amd.local import KnockoutLocalSearch
    from tests.helpers import IdxIndividual
    z = _load(golden_dir, "blup_200x1000.npz")
    gp, pp = str(tmp_path / "g.npy"), str(tmp_path / "p.npy")
    np.save(gp, z["geno"].astype(np.float64))
    np.save(pp, z["pheno"])
    random.seed(8)
    np.random.seed(8)
    rem = E.SNPRemovalHandler(100, 0.0, 0.4, False)
    with E.BlupParallelEvaluator(gp, pp, 0.4, snp_remover=rem) as ev:
        rng = np.random.default_rng(8)
        pop = [IdxIndividual(np.sort(rng.choice(1000, 60, replace=False)), 60) for _ in range(4)]
        ev.evaluate(pop, pop, 0)

        class _Pop(list):
            evaluator = ev

        best = max(pop, key=lambda i: i.fitness)
        genome, fit = KnockoutLocalSearch(_Pop(pop), window=16).search()
    g, y, T, V = z["geno"].astype(np.float64), z["pheno"], ev.training_indices, ev.validation_indices
    full = np.union1d(best.genome, np.array([])).astype(int)
    mask = np.ones(len(full), dtype=bool)
    bf = best.fitness
    for i in range(len(full)):
        mask[i] = False
        f = O.blup(full[mask], T, V, g, y, 0.4)
        if f > bf:
            bf = f
        else:
            mask[i] = True
    np.testing.assert_array_equal(genome, full[mask])
    assert abs(fit - bf) <= FIT_ATOL


def test_primal_counts_near_int16_limit(gpu):
    """SNP-space form at n_T = 8000 (the system-tile counts reach ~3.5 n_T = 28k, just under the
    int16 `kc` store and far inside fp32's exact integers on the FP4 MFMA path): fitness and
    EBVs vs the oracle's restatement of snp_blup (evaluator.py:288-314) on the same panel."""
    from tblup_amd.engine import GpuBlupEngine
    rng = np.random.default_rng(33)
    n, p, k = 9000, 1200, 400
    geno = O.synth_geno(rng, n, p, maf_lo=0.6, maf_hi=0.95)
    pheno = rng.standard_normal(n)
    perm = rng.permutation(n)
    T, V = np.sort(perm[:8000]), np.sort(perm[8000:])
    genomes = [rng.choice(p, size=k, replace=False) for _ in range(3)]
    with GpuBlupEngine(geno, pheno) as eng:
        fit, ebv = eng.evaluate(genomes, T, V, 0.4, return_ebv=True)
    for i, g in enumerate(genomes):
        f_ref, e_ref = O.snp_blup(g, T, V, geno, pheno, 0.4, return_ebv=True)
        assert abs(fit[i] - f_ref) <= FIT_ATOL
        assert _relmax(ebv[i], e_ref) <= EBV_RTOL
