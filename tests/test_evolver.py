"""DE step host side (no GPU): the oracle against the reference's goldens, the MT19937
jump-ahead of libtblup_gpu.so against numpy, and the evolver factory."""
import ctypes
import os
import random
from types import SimpleNamespace

import numpy as np
import pytest

from oracle import de_oracle as D
from tblup_amd import _native

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "de.npz")
CASES = ["rk_rand1", "rk_rand1_f5", "rk_rand1_clip", "rk_ctb", "coev_rand1", "index_rand1_int", "index_ctb"]
# name -> (strategy, d, generation, cr, F, clip, pre_draws, case index): tests/golden/make_golden.py DE_CASES
META = {
    "rk_rand1": ("de_rand_1", 1000, 1, 0.8, 0.5, False, 0, 0),
    "rk_rand1_f5": ("de_rand_1", 700, 5, 0.8, 0.5, False, 3, 1),
    "rk_rand1_clip": ("de_rand_1", 333, 10, 0.9, 0.5, True, 1, 2),
    "rk_ctb": ("de_currenttobest_1", 300, 3, 0.8, 0.5, False, 7, 3),
    "coev_rand1": ("de_rand_1", 200, 2, 0.7, 0.6, False, 2, 4),
    "index_rand1_int": ("de_rand_1", 500, 5, 0.8, 0.5, True, 5, 5),
    "index_ctb": ("de_currenttobest_1", 500, 4, 0.5, 0.5, True, 0, 6),
}


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def seed_rngs(ci, pre):
    random.seed(1000 + ci)
    np.random.seed(2000 + ci)
    np.random.rand(pre)


def coev_post(child, d):
    """CoevolutionIndividual.set_internal_genome then get_internal_genome (individual.py:184-208)."""
    L = child[-1]
    L = 1 if L < 1 else (d if L > d else L)
    return np.append(child[:-1], L)


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_de_goldens(gold, name):
    strat, d, gen, cr, F, clip, pre, ci = META[name]
    p = "de_%s_" % name
    parents = [np.array(r) for r in gold[p + "parents"]]
    seed_rngs(ci, pre)
    kids = D.de_generation(parents, list(gold[p + "fitness"]), gen, strat, d, cr, F, clip)
    if name.startswith("coev"):
        kids = [coev_post(k, d) for k in kids]
    want = gold[p + "children"]
    got = np.stack(kids)
    assert str(got.dtype) == str(gold[p + "children_dtype"])
    assert np.array_equal(got, want)
    st = np.random.get_state()
    assert np.array_equal(np.asarray(st[1], np.uint32), gold[p + "mt_key"]) and st[2] == int(gold[p + "mt_pos"])
    assert random.random() == float(gold[p + "py_next"])


def _jump(key, pos, n):
    lib = _native.load()
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.empty(624, dtype=np.uint32)
    po = ctypes.c_int32(0)
    U32 = ctypes.POINTER(ctypes.c_uint32)
    _native.check("tblup_mt19937_jump", lib.tblup_mt19937_jump(k.ctypes.data_as(U32), int(pos), int(n),
                                                               out.ctypes.data_as(U32), ctypes.byref(po)))
    return out, po.value


@pytest.mark.parametrize("pre", [0, 1, 311, 623, 624, 1000])
@pytest.mark.parametrize("n", [0, 1, 2, 623, 624, 625, 1247, 1248, 99999, 2 * 50000 * 3 + 5])
def test_mt19937_jump_equals_numpy_stream(pre, n):
    """Host GF(2) jump (mt_jump.cpp) == drawing n 32-bit words, in numpy's own (key, pos)."""
    bg = np.random.MT19937(12345)
    rs = np.random.RandomState(bg)
    rs.bytes(4 * pre) if pre else None
    st = bg.state["state"]
    key, pos = st["key"].copy(), st["pos"]
    got_key, got_pos = _jump(key, pos, n)
    if n:
        bg.random_raw(n)
    st2 = bg.state["state"]
    assert got_pos == st2["pos"]
    assert np.array_equal(got_key, st2["key"])


def test_jump_drives_legacy_rand_like_the_reference():
    """numpy's legacy rand(L) uses two words per double: a state jumped by 2L matches."""
    np.random.seed(5)
    np.random.rand(3)
    st = np.random.get_state()
    key, pos = _jump(st[1], st[2], 2 * 4321)
    np.random.rand(4321)
    want = np.random.rand(50)
    np.random.set_state(("MT19937", key, pos, 0, 0.0))
    assert np.array_equal(np.random.rand(50), want)


def test_get_evolver_factory():
    from tblup_amd import evolver as E
    args = SimpleNamespace(de_strategy="de_rand_1", dimensionality=100, crossover_rate=0.8,
                           mutation_intensity=0.5, clip=False)
    ev = E.get_evolver(args)
    assert isinstance(ev, E.DERandOneEvolver) and ev.clip is False
    args.de_strategy = "de_currenttobest_1"
    assert isinstance(E.get_evolver(args), E.DECurrentToBestOneEvolver)
    for bad in ("nope",):
        args.de_strategy = bad
        with pytest.raises(NotImplementedError):
            E.get_evolver(args)


def test_exclusive_randrange_consumes_like_reference():
    from tblup_amd.evolver import exclusive_randrange
    random.seed(3)
    a = [exclusive_randrange(0, 5, [0, 1, 2]) for _ in range(20)]
    random.seed(3)
    b = [D.exclusive_randrange(0, 5, [0, 1, 2]) for _ in range(20)]
    assert a == b and all(x in (3, 4) for x in a)


def _python_donors(strategy, n, L, best):
    """The reference's per-individual draws in order (evolver.py:118-121 / :199-203 through
    utils.py:21-36, then evolver.py:76's fixed position), via the oracle's exclusive_randrange."""
    donors, fixed = [], []
    for i in range(n):
        if strategy == "de_rand_1":
            a = D.exclusive_randrange(0, n, [i])
            b = D.exclusive_randrange(0, n, [i, a])
            c = D.exclusive_randrange(0, n, [i, a, b])
            donors.append((a, b, c))
        else:
            excl = [i, best]
            a = D.exclusive_randrange(0, n, excl)
            excl.append(a)
            b = D.exclusive_randrange(0, n, excl)
            donors.append((best, a, b))
        fixed.append(random.randrange(0, L))
    return np.array(donors, dtype=np.int32), np.array(fixed, dtype=np.int64)


@pytest.mark.parametrize("strategy", ["de_rand_1", "de_currenttobest_1"])
@pytest.mark.parametrize("n,L,pre", [(4, 1, 0), (5, 2, 3), (7, 3, 623), (64, 1000, 624), (256, 50000, 17),
                                     (1000, 3_000_000_000, 5), (300, 1 << 31, 400)])
def test_native_donors_equal_python_random(strategy, n, L, pre):
    """tblup_de_donors (CPython's MT19937 restated in C) draws the same donors and fixed
    positions as the python loops and leaves `random` in the same state."""
    from tblup_amd.evolver import _native_donors
    code = _native.DE_STRATEGY[strategy]
    for rep in range(3):
        random.seed(7 * n + rep)
        for _ in range(pre):
            random.random()
        best = -1 if strategy == "de_rand_1" else (rep * 37) % n
        st = random.getstate()
        got = _native_donors(code, n, L, best)
        after_native = random.getstate()
        random.setstate(st)
        want = _python_donors(strategy, n, L, best)
        assert got is not None
        np.testing.assert_array_equal(got[0], want[0])
        np.testing.assert_array_equal(got[1], want[1])
        assert after_native == random.getstate()


def test_native_donors_small_population_stays_in_python():
    from tblup_amd.evolver import _native_donors
    assert _native_donors(_native.DE_STRATEGY["de_rand_1"], 3, 10) is None
    lib = _native.load()
    d = np.zeros((3, 3), np.int32)
    f = np.zeros(3, np.int64)
    mt = np.zeros(624, np.uint32)
    idx = np.array([624], np.int32)
    rc = lib.tblup_de_donors(0, 3, 10, -1, mt.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                             idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                             d.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                             f.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
    assert rc != 0 and b"pop" in lib.tblup_last_error()


# ---- adaptive evolvers (evolver.py:297-687) against whole reference runs (tests/golden/make_golden.py
# gen_sade / gen_mde): every generation's children, the adaptive state, the parameter CSV, the RNGs ----
ADAPT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# name -> (kind, d, length, pop, generations, clip, case index): make_golden.py SADE_CASES / MDE_CASES
SADE_META = {"sade_rk": ("rk", 150, 15, 8, 56, False, 0), "sade_rk_clip": ("rk", 120, 10, 6, 12, True, 1),
             "sade_index": ("index", 200, 20, 6, 12, True, 2)}
MDE_META = {"mde_rk": ("rk", 150, 15, 12, 8, False, 0), "mde_index": ("index", 200, 20, 8, 6, True, 1)}


def _adaptive_run(z, name, meta, make_evolver, seeds, tmp_path, state_of):
    """Drive `make_evolver()` through the recorded run: individuals with the reference's semantics
    (tests/ga_driver.py), fitness from the run's own generator, greedy selection."""
    import hashlib
    from tests import ga_driver as GD
    from tests.helpers import Pop
    kind, d, length, pop, gens, clip, ci = meta
    parents = z[name + "_parents"]
    cls = GD.IndexIndividual if kind == "index" else GD.RandomKeyIndividual
    inds = [cls(length, d, genome=parents[i].copy()) for i in range(pop)]
    for ind, f in zip(inds, z[name + "_fitness"]):
        ind.fitness = float(f)
    frng = np.random.default_rng(seeds[2] + ci)
    random.seed(seeds[0] + ci)
    np.random.seed(seeds[1] + ci)
    if name.startswith("sade"):
        np.random.rand(3 * ci + 1)
    ev = make_evolver(d, gens, clip)
    popn = Pop(inds, 1)
    popn.monitor = SimpleNamespace(results_file=str(tmp_path / "results.csv"))
    for g in range(1, gens + 1):
        popn.generation = g
        kids = ev.evolve(popn)
        kg = np.stack([np.asarray(k.get_internal_genome()) for k in kids])
        if name + "_children_g%d" % g in z.files:
            np.testing.assert_array_equal(kg, z[name + "_children_g%d" % g])
        assert hashlib.sha256(np.ascontiguousarray(kg).tobytes()).hexdigest() == str(z[name + "_children_sha256"][g - 1]), g
        np.testing.assert_array_equal(np.array(state_of(ev), dtype=np.float64), z[name + "_state"][g - 1])
        for k, f in zip(kids, frng.uniform(size=pop)):
            k.fitness = float(f)
        popn.population = [k if k.fitness > q.fitness else q for q, k in zip(popn.population, kids)]
    assert open(tmp_path / "results_params.csv").read() == str(z[name + "_params_csv"])
    st = np.random.get_state()
    np.testing.assert_array_equal(np.asarray(st[1], dtype=np.uint32), z[name + "_mt_key"])
    assert st[2] == int(z[name + "_mt_pos"])
    if name + "_gauss" in z.files:
        assert [st[3], st[4]] == list(z[name + "_gauss"])
    assert random.random() == float(z[name + "_py_next"])


def _sade_state(ev):
    return [ev.cr_m, ev.p, ev.ns_1, ev.ns_2, ev.nf_1, ev.nf_2, len(ev.successful_crs)]


@pytest.mark.parametrize("name", sorted(SADE_META))
def test_sade_host_side_matches_reference(name, tmp_path, monkeypatch):
    """tblup_amd.evolver.SaDE (its adaptation, draws and report) over a whole reference run, with the
    GPU DE step swapped for the oracle's children from the same draws (the GPU step itself:
    tests/test_gpu_evolver.py)."""
    from copy import deepcopy
    from tblup_amd import evolver as EV

    def host_generation(self, population, t, donors, fixed, strategy, mi, cr, clip, members=None):
        genomes = [population[i].get_internal_genome() for i in range(len(population))]
        kids = D.de_children(genomes, strategy, donors, fixed, mi, cr, clip, self.dimensionality - 1)
        out = []
        for i, c in enumerate(kids):
            k = deepcopy(population[i])
            k.set_internal_genome(c)
            out.append(k)
        return out
    monkeypatch.setattr(EV.SaDE, "_gpu_generation", host_generation)
    z = np.load(os.path.join(ADAPT, "sade.npz"))
    _adaptive_run(z, name, SADE_META[name], lambda d, g, clip: EV.SaDE(d, clip), (500, 600, 400), tmp_path,
                  _sade_state)


@pytest.mark.parametrize("name", sorted(MDE_META))
def test_mde_pbx_matches_reference(name, tmp_path):
    """tblup_amd.evolver.MDE_pBX (host DE step) reproduces whole reference runs: children, the adapted
    cr_m / f_m / p, the parameter CSV and both RNG states."""
    from tblup_amd import evolver as EV
    z = np.load(os.path.join(ADAPT, "mde.npz"))
    _adaptive_run(z, name, MDE_META[name], lambda d, g, clip: EV.MDE_pBX(d, g, clip), (900, 1000, 800), tmp_path,
                  lambda ev: [ev.cr_m, ev.f_m, ev.p, len(ev.successful_crs), len(ev.successful_fs)])


def test_get_evolver_adaptive():
    from tblup_amd import evolver as EV
    a = SimpleNamespace(de_strategy="sade", dimensionality=10, clip=True, generations=5)
    assert isinstance(EV.get_evolver(a), EV.SaDE)
    a.de_strategy = "mde_pbx"
    e = EV.get_evolver(a)
    assert isinstance(e, EV.MDE_pBX) and e.g_max == 5
