"""numpy index semantics and float32 panels against the reference (tests/golden/blup_extra.npz).

The reference gathers `data[:, indices]` (evaluator.py:275/298) from an IndexIndividual's
`_genome.astype(int)` (individual.py:93-95); DE without --clip (the default, config.py:104)
leaves such genomes with negative entries, which numpy wraps to i + P, and an index >= P
(or < -P) raises IndexError.  The drop-in applies the same rule: negatives wrap (on the
device), out-of-bounds indices raise IndexError on the host entry and give a NaN fitness
plus the context's index-error flag on the device entry.

float32 panels: the reference's snp_blup / make_grm then compute in float32 (fitness within
~1e-7, EBVs within ~5e-7 relative of the float64 result, recorded in the golden); the GPU
path is exact-integer + fp64 for {0,1,2} data of any dtype, so it matches the float64
result to 1e-9 and the float32 reference within the north star's 1e-5 relative.
"""
import os

import numpy as np
import pytest

from oracle import blup_oracle as O


@pytest.fixture(scope="module")
def extra(golden_dir):
    return np.load(os.path.join(golden_dir, "blup_extra.npz"))


@pytest.fixture(scope="module")
def panel(golden_dir):
    z = np.load(os.path.join(golden_dir, "blup_200x1000.npz"))
    return z["geno"], z["pheno"], z["T"], z["V"]


def test_golden_records_numpy_rules(extra):
    for name in extra["neg_names"]:
        idx = extra[name + "_idx"]
        assert (idx < 0).any()
        np.testing.assert_array_equal(idx, extra[name + "_internal"].astype(int))   # individual.py:93-95
    assert str(extra["oob_hi_raises"]) == "IndexError" and str(extra["oob_lo_raises"]) == "IndexError"


def test_oracle_negative_indices(extra, panel):
    geno, pheno, T, V = panel
    data = geno.astype(np.float64)
    for name in extra["neg_names"]:
        f, e = O.blup(extra[name + "_idx"], T, V, data, pheno, 0.4, return_ebv=True)
        assert abs(f - float(extra[name + "_fitness"])) < 1e-12
        np.testing.assert_allclose(e, extra[name + "_ebv"], rtol=0, atol=1e-12 * np.max(np.abs(e)))


def test_oracle_vs_float32_reference(extra, panel):
    """The oracle (float64) against the reference's float32 arithmetic: the recorded gap."""
    geno, pheno, T, V = panel
    for name in extra["f32_names"]:
        f, e = O.blup(extra[name + "_idx"], T, V, geno.astype(np.float64), pheno, 0.4, return_ebv=True)
        assert abs(f - float(extra[name + "_fitness64"])) < 1e-12
        scale = np.max(np.abs(e))
        assert np.max(np.abs(e - extra[name + "_ebv"])) <= 1e-5 * scale
        assert abs(f - float(extra[name + "_fitness"])) <= 1e-6


@pytest.mark.gpu
def test_gpu_negative_indices_wrap(gpu, extra, panel):
    from tblup_amd.engine import GpuBlupEngine
    geno, pheno, T, V = panel
    names = list(extra["neg_names"])
    genomes = [extra[n + "_idx"] for n in names]
    with GpuBlupEngine(geno, pheno, device=0) as eng:
        fit, ebv = eng.evaluate(genomes, T, V, 0.4, return_ebv=True)
        # the same columns addressed with non-negative ids give bit-identical results
        pos = [np.where(g < 0, g + geno.shape[1], g) for g in genomes]
        fit_pos = eng.evaluate(pos, T, V, 0.4)
    np.testing.assert_array_equal(fit, fit_pos)
    for i, n in enumerate(names):
        assert abs(fit[i] - float(extra[n + "_fitness"])) < 1e-9, n
        e = extra[n + "_ebv"]
        assert np.max(np.abs(ebv[i] - e)) <= 1e-9 * np.max(np.abs(e)), n


@pytest.mark.gpu
def test_gpu_out_of_bounds_raise_index_error(gpu, extra, panel):
    from tblup_amd.engine import GpuBlupEngine
    geno, pheno, T, V = panel
    with GpuBlupEngine(geno, pheno, device=0) as eng:
        for name in ("oob_hi", "oob_lo"):
            with pytest.raises(IndexError, match="out of bounds for axis 1 with size 1000"):
                eng.evaluate([np.arange(5), extra[name + "_idx"]], T, V, 0.4)
        # the context stays usable after the rejected batch
        assert np.isfinite(eng.evaluate([np.arange(50)], T, V, 0.4)[0])


@pytest.mark.gpu
def test_gpu_device_entry_flags_out_of_bounds(gpu, extra, panel):
    """tblup_eval_batch_device: negatives wrap, an out-of-bounds individual gets NaN and
    raises the index-error flag; the other individuals of the batch are unaffected."""
    import torch
    from tblup_amd.engine import GpuBlupEngine, concat_genomes
    geno, pheno, T, V = panel
    good = extra["neg_snp_idx"]
    genomes = [good, extra["oob_hi_idx"], good[::-1].copy()]
    idx, off = concat_genomes(genomes)
    with GpuBlupEngine(geno, pheno, device=0) as eng:
        sid = eng.split_id(T, V)
        d_idx = torch.from_numpy(idx).cuda()
        d_off = torch.from_numpy(off).cuda()
        d_fit = torch.empty(3, dtype=torch.float64, device="cuda")
        s = torch.cuda.current_stream()
        assert not eng.index_error(s.cuda_stream)
        eng.evaluate_device(sid, d_idx.data_ptr(), d_off.data_ptr(), off, 0.4, d_fit.data_ptr(), stream_ptr=s.cuda_stream)
        assert eng.index_error(s.cuda_stream)
        assert not eng.index_error(s.cuda_stream)            # cleared by the read
        fit = d_fit.cpu().numpy()
        host = eng.evaluate([good, good[::-1].copy()], T, V, 0.4)
    assert np.isnan(fit[1])
    assert abs(fit[0] - float(extra["neg_snp_fitness"])) < 1e-9
    np.testing.assert_allclose(fit[[0, 2]], host, rtol=0, atol=1e-12)


@pytest.mark.gpu
def test_gpu_float32_panel(gpu, extra, panel):
    """A float32 panel file: exact {0,1,2} values, so the GPU result is the float64 one
    (1e-9) and within the north star's 1e-5 relative of the reference's float32 EBVs."""
    from tblup_amd.engine import GpuBlupEngine
    geno, pheno, T, V = panel
    names = list(extra["f32_names"])
    with GpuBlupEngine(geno.astype(np.float32), pheno, device=0) as eng:
        fit, ebv = eng.evaluate([extra[n + "_idx"] for n in names], T, V, 0.4, return_ebv=True)
    for i, n in enumerate(names):
        e32, e64 = extra[n + "_ebv"], extra[n + "_ebv64"]
        assert abs(fit[i] - float(extra[n + "_fitness64"])) < 1e-9, n
        assert np.max(np.abs(ebv[i] - e64)) <= 1e-9 * np.max(np.abs(e64)), n
        assert np.max(np.abs(ebv[i] - e32)) <= 1e-5 * np.max(np.abs(e32)), n
        assert abs(fit[i] - float(extra[n + "_fitness"])) <= 1e-6, n
