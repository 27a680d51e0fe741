"""The CPU oracle (oracle/blup_oracle.py) pinned against the reference's golden vectors.

The goldens were produced by running the reference (ianwhale/tblup) itself in the
build container: tests/golden/make_golden.py.
"""
import hashlib
import os

import numpy as np
import pytest

from oracle import blup_oracle as O


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def test_make_grm_matches_reference(golden_dir):
    z = _load(golden_dir, "grm_64x200.npz")
    G = O.make_grm(z["geno"])
    np.testing.assert_allclose(G, z["G"], rtol=0, atol=1e-13)
    np.testing.assert_allclose(G, z["G_int"], rtol=0, atol=1e-13)


def _cases(z):
    for i, name in enumerate(z["names"]):
        yield i, str(name), z["idx"][z["offsets"][i]:z["offsets"][i + 1]]


@pytest.mark.parametrize("form", ["reference", "grm_form"])
def test_blup_fitness_and_ebv(golden_dir, form):
    z = _load(golden_dir, "blup_200x1000.npz")
    g, y, T, V = z["geno"], z["pheno"], z["T"], z["V"]
    for i, name, idx in _cases(z):
        if form == "reference":
            f, e = O.blup(idx, T, V, g.astype(np.float64), y, float(z["h2"]), return_ebv=True)
        else:
            f, e = O.blup_grm_form(idx, T, V, g, y, float(z["h2"]))
        ref_e = z["ebv"][i]
        assert abs(f - z["fitness"][i]) < 1e-12, name
        assert np.max(np.abs(e - ref_e)) <= 1e-12 * np.max(np.abs(ref_e)) + 1e-15, name


def test_branch_dispatch_rule(golden_dir):
    """evaluator.py:257: GBLUP iff len(indices) > n (strict)."""
    z = _load(golden_dir, "blup_200x1000.npz")
    n = z["geno"].shape[0]
    for i, name, idx in _cases(z):
        expect = "gblup" if len(idx) > n else "snp"
        assert str(z["branch"][i]) == expect, name


def test_testing_split_and_h2_sweep(golden_dir):
    z = _load(golden_dir, "blup_200x1000.npz")
    g, y = z["geno"], z["pheno"]
    TV = np.concatenate([z["T"], z["V"]])
    for i, name, idx in _cases(z):
        f, e = O.blup_grm_form(idx, TV, z["X"], g, y, float(z["h2"]))
        assert abs(f - z["test_fitness"][i]) < 1e-12, name
    idx_snp = z["idx"][z["offsets"][0]:z["offsets"][1]]
    idx_gb = z["idx"][z["offsets"][8]:z["offsets"][9]]
    for h, (fs, fg) in zip(z["h2_sweep"], z["h2_sweep_fitness"]):
        assert abs(O.blup_grm_form(idx_snp, z["T"], z["V"], g, y, h)[0] - fs) < 1e-12
        assert abs(O.blup_grm_form(idx_gb, z["T"], z["V"], g, y, h)[0] - fg) < 1e-12


def test_degenerate_panels_are_nan(golden_dir):
    z = _load(golden_dir, "blup_edge.npz")
    g, y, T, V = z["geno"], z["pheno"], z["T"], z["V"]
    sel = {"mono0_snp": np.arange(10, 20), "mono0_gblup": np.tile(np.arange(10, 20), 21),
           "het_snp": np.arange(0, 10)}
    for name, kind, value in zip(z["names"], z["kind"], z["value"]):
        assert kind == "value" and value == "nan", (name, kind, value)
        f, _ = O.blup_grm_form(sel[str(name)], T, V, g, y, 0.4)
        assert np.isnan(f), name


def test_config2_shape_golden(golden_dir):
    z = _load(golden_dir, "blup_2000x4000.npz")
    rng = np.random.default_rng(int(z["seed"]))
    geno = O.synth_geno(rng, int(z["n"]), int(z["p"]))
    assert hashlib.sha256(geno.tobytes()).hexdigest() == str(z["geno_sha256"])
    y, T, V = z["pheno"], z["T"], z["V"]
    for i in range(len(z["offsets"]) - 1):
        idx = z["idx"][z["offsets"][i]:z["offsets"][i + 1]]
        f, e = O.blup_grm_form(idx, T, V, geno, y, 0.4)
        assert abs(f - z["fitness"][i]) < 1e-10
        ref = z["ebv"][i] if i < 3 else z["ebv_gblup"]
        assert np.max(np.abs(e - ref)) <= 1e-10 * np.max(np.abs(ref))


def test_decode_matches_reference(golden_dir):
    z = _load(golden_dir, "decode.npz")
    for keys, genome in zip(z["rk_keys"], z["rk_genome"]):
        np.testing.assert_array_equal(O.decode_randkeys(keys, int(z["rk_length"])), genome)
    np.testing.assert_array_equal(O.decode_randkeys(z["coev_keys"], float(z["coev_length"])), z["coev_genome"])
    np.testing.assert_array_equal(O.decode_index(z["index_internal"]), z["index_genome"])
    np.testing.assert_array_equal(O.decode_nullable(z["index_internal"], 500), z["nullable_genome"])
    assert O.coevolution_fitness(0.5, 1.0, float(z["coev_length"]), 500) == pytest.approx(float(z["coev_fitness"]),
                                                                                        abs=0)


def test_pearson_restatement_edge_cases():
    from scipy.stats import pearsonr
    rng = np.random.default_rng(0)
    for n in (2, 3, 17, 320):
        x, y = rng.standard_normal(n), rng.standard_normal(n)
        assert O.pearson_r(x, y) == pytest.approx(float(pearsonr(x, y)[0]), abs=1e-15)
    assert np.isnan(O.pearson_r(np.ones(5), np.arange(5.0)))
    with pytest.raises(ValueError):
        O.pearson_r(np.ones(1), np.ones(1))


def test_grm_block_identity():
    """K_{R,T} of the exact-integer form equals make_grm's blocks for gblup (p over all rows)."""
    rng = np.random.default_rng(3)
    g = O.synth_geno(rng, 90, 150)
    perm = rng.permutation(90)
    T, V = perm[:50], perm[50:70]
    idx = rng.integers(0, 150, 120)
    K = O.grm_block(idx, T, V, g, branch="gblup")
    G = O.make_grm(g[:, idx])
    np.testing.assert_allclose(K, G[np.ix_(np.concatenate([T, V]), T)], rtol=0, atol=1e-12)
