"""GPU DE step (k_de.hip through tblup_de_step): children and RNG states bit-exact to the
reference's evolvers (goldens) and to the numpy oracle at config-2 size."""
import hashlib
import os
from copy import deepcopy
import random

import numpy as np
import pytest

from oracle import de_oracle as D
from tests.helpers import CoevoIndividual, IdxIndividual, KeyIndividual, Pop, RandomKeyIndividual
from tests.test_evolver import CASES, META, coev_post, seed_rngs  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gold(golden_dir, gpu):
    import os
    return np.load(os.path.join(golden_dir, "de.npz"))


def _evolver(strat, d, cr, F, clip):
    from tblup_amd import evolver as E
    cls = E.DERandOneEvolver if strat == "de_rand_1" else E.DECurrentToBestOneEvolver
    return cls(d, cr, F, clip)


def _individuals(name, parents, fitness, d):
    inds = []
    for g, f in zip(parents, fitness):
        if name.startswith("coev"):
            ind = CoevoIndividual(np.array(g[:-1]), float(g[-1]), d)
        elif name.startswith("index"):
            ind = IdxIndividual(np.array(g), len(g))
        else:
            ind = KeyIndividual(np.array(g), 10)
        ind.fitness = float(f)
        inds.append(ind)
    return inds


@pytest.mark.parametrize("name", CASES)
def test_gpu_de_matches_reference_goldens(gold, name):
    strat, d, gen, cr, F, clip, pre, ci = META[name]
    p = "de_%s_" % name
    inds = _individuals(name, gold[p + "parents"], gold[p + "fitness"], d)
    seed_rngs(ci, pre)
    kids = _evolver(strat, d, cr, F, clip).evolve(Pop(inds, gen))
    got = np.stack([np.asarray(k.get_internal_genome()) for k in kids])
    assert str(got.dtype) == str(gold[p + "children_dtype"])
    assert np.array_equal(got, gold[p + "children"])
    assert len({k.uid for k in kids} | {i.uid for i in inds}) == 2 * len(inds)   # fresh uids (deepcopy)
    st = np.random.get_state()
    assert np.array_equal(np.asarray(st[1], np.uint32), gold[p + "mt_key"]) and st[2] == int(gold[p + "mt_pos"])
    assert random.random() == float(gold[p + "py_next"])


@pytest.mark.parametrize("strat", ["de_rand_1", "de_currenttobest_1"])
def test_gpu_de_big_goldens(gold, strat):
    d, pop = int(gold["big_d"]), int(gold["big_pop"])
    rng = np.random.default_rng(7)
    keys = rng.uniform(size=(pop, d))
    fit = rng.uniform(size=pop)
    inds = [KeyIndividual(keys[i].copy(), 1000) for i in range(pop)]
    for ind, f in zip(inds, fit):
        ind.fitness = float(f)
    random.seed(31)
    np.random.seed(32)
    np.random.rand(11)
    kids = _evolver(strat, d, 0.8, 0.5, False).evolve(Pop(inds, 1))
    p = "big_%s_" % strat
    got = np.stack([k.get_internal_genome() for k in kids])
    assert np.array_equal(got[0, :64], gold[p + "children_row0"])
    assert hashlib.sha256(np.ascontiguousarray(got).tobytes()).hexdigest() == str(gold[p + "children_sha256"])
    st = np.random.get_state()
    assert np.array_equal(np.asarray(st[1], np.uint32), gold[p + "mt_key"]) and st[2] == int(gold[p + "mt_pos"])
    assert random.random() == float(gold[p + "py_next"])


@pytest.mark.parametrize("gen,pre,pop", [(1, 0, 256), (5, 623, 256), (7, 624, 256), (2, 17, 512)])
def test_gpu_de_config2_vs_oracle(gpu, gen, pre, pop):
    """pop 256 x d 50000 (BASELINE config 2), three generations in a row against the oracle; pop 512:
    the three-launch form (sequence, jumps, mask and stream: more individuals than CUs)."""
    d = 50000
    rng = np.random.default_rng(gen)
    keys = rng.uniform(size=(pop, d))
    fit = list(rng.uniform(size=pop))
    inds = [KeyIndividual(keys[i].copy(), 1000) for i in range(pop)]
    for ind, f in zip(inds, fit):
        ind.fitness = f
    ev = _evolver("de_rand_1", d, 0.8, 0.5, False)
    genomes = [keys[i] for i in range(pop)]
    random.seed(gen)
    np.random.seed(gen)
    np.random.bytes(4 * pre)
    for g in range(gen, gen + 3):
        py, npst = random.getstate(), np.random.get_state()
        kids = ev.evolve(Pop(inds, g))
        py_after, np_after = random.getstate(), np.random.get_state()
        random.setstate(py)
        np.random.set_state(npst)
        want = D.de_generation(genomes, fit, g, "de_rand_1", d, 0.8, 0.5, False)
        assert random.getstate() == py_after
        st = np.random.get_state()
        assert np.array_equal(st[1], np_after[1]) and st[2] == np_after[2]
        for k, w in zip(kids, want):
            assert np.array_equal(k.get_internal_genome(), w)
        inds, genomes = kids, want


def test_gpu_de_bad_arguments_raise(gpu):
    from tblup_amd import _native
    from tblup_amd.evolver import GpuDEStep
    step = GpuDEStep.get(0)
    par = np.zeros((4, 10))
    with pytest.raises(_native.TblupError):
        step.step(0, par, np.array([[1, 2, 4]] * 4), np.zeros(4), 0.5, 0.8, False, 9)   # donor 4 of pop 4
    with pytest.raises(_native.TblupError):
        step.step(0, par, np.array([[1, 2, 3]] * 4), np.full(4, 10), 0.5, 0.8, False, 9)   # fixed >= L


def test_gpu_de_deferred_state(gpu):
    """step_device(defer=True): children and numpy's state equal the synchronous step's; a
    second step before the state is fetched, or a fetch with nothing pending, is refused."""
    import torch
    from tblup_amd import _native
    from tblup_amd.evolver import GpuDEStep
    step = GpuDEStep.get(0)
    rng = np.random.default_rng(4)
    par = torch.from_numpy(rng.uniform(size=(16, 301))).cuda()
    donors = np.array([[(i + 1) % 16, (i + 2) % 16, (i + 3) % 16] for i in range(16)])
    fixed = rng.integers(0, 301, 16)
    np.random.seed(5)
    want = step.step_device(0, par, donors, fixed, 0.5, 0.8, True, 1.0).cpu().numpy()
    want_state = np.random.get_state()
    np.random.seed(5)
    kids, finish = step.step_device(0, par, donors, fixed, 0.5, 0.8, True, 1.0, defer=True)
    with pytest.raises(_native.TblupError, match="not fetched") as ei:
        step.step_device(0, par, donors, fixed, 0.5, 0.8, True, 1.0)
    assert ei.value.code == _native.ERR_STATE
    finish()
    assert np.array_equal(kids.cpu().numpy(), want)
    got_state = np.random.get_state()
    assert np.array_equal(got_state[1], want_state[1]) and got_state[2] == want_state[2]
    key = np.zeros(624, np.uint32)
    pos = np.zeros(1, np.int32)
    import ctypes
    rc = step._lib.tblup_de_state_wait(step._ctx, key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                       pos.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    assert rc == _native.ERR_STATE and b"no DE step pending" in step._lib.tblup_last_error()


def test_gpu_generations_with_device_keystore(gpu, tmp_path):
    """evolve -> evaluate -> select for 3 generations with the GPU evolver and evaluator (keys
    stay on the device between them) equals the same loop with the host oracle DE and a
    fresh store every generation (host-stacked decode)."""
    from oracle import blup_oracle as O
    from tblup_amd.evaluator import BlupParallelEvaluator
    from tblup_amd.keystore import DeviceKeyStore
    rng = np.random.default_rng(11)
    n, p, k, pop = 400, 3000, 150, 24
    geno = O.synth_geno(rng, n, p)
    pheno = rng.standard_normal(n)
    np.save(tmp_path / "g.npy", geno)
    np.save(tmp_path / "y.npy", pheno)
    keys0 = rng.uniform(size=(pop, p))

    class P(Pop):
        pass

    def run(use_gpu_de):
        random.seed(5)
        np.random.seed(5)
        ev = BlupParallelEvaluator(str(tmp_path / "g.npy"), str(tmp_path / "y.npy"), 0.4)
        inds = [RandomKeyIndividual(keys0[i].copy(), k) for i in range(pop)]
        fits = []
        with ev:
            popn = P(inds, 0)
            ev.evaluate(popn, popn, 0)
            evo = _evolver("de_rand_1", p, 0.8, 0.5, False)
            for g in range(1, 4):
                popn.generation = g
                if use_gpu_de:
                    kids = evo.evolve(popn)
                    hits = DeviceKeyStore.get(0).rows(kids)
                    assert all(h is not None for h in hits)
                else:
                    DeviceKeyStore.get(0).clear()
                    want = D.de_generation([x.get_internal_genome() for x in popn.population],
                                           [x.fitness for x in popn.population], g, "de_rand_1", p, 0.8, 0.5, False)
                    kids = [RandomKeyIndividual(w, k) for w in want]
                ev.evaluate(popn, kids, g)
                popn.population = [c if c.fitness > q.fitness else q for q, c in zip(popn.population, kids)]
                fits.append([x.fitness for x in kids])
                genomes = [x.get_internal_genome().copy() for x in popn.population]
        return fits, genomes

    from tblup_amd.engine import GpuBlupEngine
    calls = []
    orig = GpuBlupEngine.decode_randkey_tensor

    def spy(self, *a, **kw):
        calls.append(1)
        return orig(self, *a, **kw)
    GpuBlupEngine.decode_randkey_tensor = spy
    try:
        f_gpu, g_gpu = run(True)
    finally:
        GpuBlupEngine.decode_randkey_tensor = orig
    assert len(calls) == 3   # the children were decoded in place from the device key store
    f_ref, g_ref = run(False)
    assert f_gpu == f_ref
    for a, b in zip(g_gpu, g_ref):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("L,pop,pre", [(1, 4, 0), (10, 4, 3), (100, 5, 624), (311, 4, 1), (312, 7, 0),
                                       (313, 6, 622), (1000, 33, 100), (1, 400, 0), (313, 384, 622),
                                       (70000, 384, 5)])
def test_gpu_de_small_shapes_vs_oracle(gpu, L, pop, pre):
    """Tiny generations (< 625 stream words: the end state is rebuilt from the base window
    without a jump), block-boundary lengths and every numpy position class; pop >= 384: the
    three-launch form (more individuals than the 256 CUs), L = 70000 across two of its
    65536-element mask segments."""
    rng = np.random.default_rng(L * 7 + pop)
    keys = rng.uniform(size=(pop, L))
    fit = list(rng.uniform(size=pop))
    for strat in ("de_rand_1", "de_currenttobest_1"):
        inds = [KeyIndividual(keys[i].copy(), 1) for i in range(pop)]
        for ind, f in zip(inds, fit):
            ind.fitness = f
        random.seed(L)
        np.random.seed(pop)
        np.random.bytes(4 * pre)
        py, npst = random.getstate(), np.random.get_state()
        kids = _evolver(strat, L, 0.6, 0.7, strat == "de_rand_1").evolve(Pop(inds, 2))
        py_after, np_after = random.getstate(), np.random.get_state()
        random.setstate(py)
        np.random.set_state(npst)
        want = D.de_generation([keys[i] for i in range(pop)], fit, 2, strat, L, 0.6, 0.7, strat == "de_rand_1")
        assert random.getstate() == py_after
        st = np.random.get_state()
        assert np.array_equal(st[1], np_after[1]) and st[2] == np_after[2], (strat, L, pop, pre)
        for k, w in zip(kids, want):
            assert np.array_equal(k.get_internal_genome(), w), (strat, L, pop, pre)



@pytest.mark.parametrize("kind", ["helpers", "reference"])
def test_gpu_block_rows_many_generations(gpu, tmp_path, kind):
    """14 generations of evolve -> evaluate -> select with the children's genomes as rows of
    page-locked per-generation blocks: equal to the host-oracle loop generation by generation,
    the blocks still in use stay bounded (compaction, its copies on worker threads), compacted
    genomes keep their device rows, and rows are independent arrays (an in-place write touches
    one child only).  kind "reference": individuals with the reference's set_internal_genome
    (tests/ga_driver.py, individual.py:100-101), whose children are bound to their rows while
    the rows are still in flight."""
    from tests import ga_driver as GD
    from oracle import blup_oracle as O
    from tblup_amd import evolver as EVM
    from tblup_amd.evaluator import BlupParallelEvaluator
    from tblup_amd.keystore import DeviceKeyStore
    rng = np.random.default_rng(12)
    n, p, k, pop, gens = 300, 2000, 100, 48, 14
    geno = O.synth_geno(rng, n, p)
    pheno = rng.standard_normal(n)
    np.save(tmp_path / "g.npy", geno)
    np.save(tmp_path / "y.npy", pheno)
    keys0 = rng.uniform(size=(pop, p))

    def run(use_gpu_de):
        random.seed(9)
        np.random.seed(9)
        ev = BlupParallelEvaluator(str(tmp_path / "g.npy"), str(tmp_path / "y.npy"), 0.4)
        if kind == "reference":
            inds = [GD.RandomKeyIndividual(k, p, genome=keys0[i].copy()) for i in range(pop)]
        else:
            inds = [RandomKeyIndividual(keys0[i].copy(), k) for i in range(pop)]
        fits, alive = [], []
        with ev:
            popn = Pop(inds, 0)
            ev.evaluate(popn, popn, 0)
            evo = _evolver("de_rand_1", p, 0.8, 0.5, False)
            for g in range(1, gens + 1):
                popn.generation = g
                if use_gpu_de:
                    kids = evo.evolve(popn)
                    assert all(h is not None for h in DeviceKeyStore.get(0).rows(popn.population))
                    alive.append(sum(r() is not None for r in EVM._BLOCKS._reg.values()))
                else:
                    DeviceKeyStore.get(0).clear()
                    want = D.de_generation([x.get_internal_genome() for x in popn.population],
                                           [x.fitness for x in popn.population], g, "de_rand_1", p, 0.8, 0.5, False)
                    if kind == "reference":   # as the reference's evolver makes them (no RNG draw)
                        kids = [deepcopy(q) for q in popn.population]
                        for c, w in zip(kids, want):
                            c.set_internal_genome(w)
                    else:
                        kids = [RandomKeyIndividual(w, k) for w in want]
                ev.evaluate(popn, kids, g)
                popn.population = [c if c.fitness > q.fitness else q for q, c in zip(popn.population, kids)]
                fits.append([x.fitness for x in kids])
            genomes = [x.get_internal_genome().copy() for x in popn.population]
            if use_gpu_de:
                a, b = popn.population[0], popn.population[1]
                before = b.get_internal_genome().copy()
                a.get_internal_genome()[0] = 0.123   # an in-place write, as Individual.__setitem__ does
                assert np.array_equal(b.get_internal_genome(), before)
        return fits, genomes, alive

    f_gpu, g_gpu, alive = run(True)
    f_ref, g_ref, _ = run(False)
    assert f_gpu == f_ref
    for x, y in zip(g_gpu, g_ref):
        assert np.array_equal(x, y)
    assert max(alive) <= EVM._BLOCKS.keep + 2, alive


@pytest.mark.parametrize("n,L,shift", [(1, 1, 0), (5, 7, 1), (130, 1000, 0), (300, 50_000, 0), (129, 33, 1)])
def test_gather_rows(gpu, n, L, shift):
    """tblup_gather_rows: rows scattered over several device tensors (odd L, rows starting
    8 B off 16-B alignment, > 128 rows in several launches) gathered exactly."""
    import torch
    from tblup_amd.evolver import GpuDEStep
    step = GpuDEStep.get(0)
    srcs = [torch.rand(n, L + shift, dtype=torch.float64, device="cuda") for _ in range(3)]
    rng = np.random.default_rng(n + L)
    pick = [(int(rng.integers(3)), int(rng.integers(n))) for _ in range(n)]
    ptrs = [srcs[s].data_ptr() + 8 * (r * (L + shift) + shift) for s, r in pick]
    out = torch.full((n, L), -1.0, dtype=torch.float64, device="cuda")
    step.gather_rows(out, ptrs)
    want = torch.stack([srcs[s][r, shift:] for s, r in pick])
    assert torch.equal(out, want)


@pytest.mark.parametrize("name", ["sade_rk", "sade_rk_clip", "sade_index"])
def test_gpu_sade_matches_reference(gpu, name, tmp_path):
    """SaDE (evolver.py:407-547) with its generation on the GPU (per-individual strategy and
    crossover rate, tblup_de_step_device_async_mix) reproduces whole reference runs
    (tests/golden/sade.npz): every generation's children, the adaptive state, the parameter CSV,
    numpy's and python's RNG states."""
    from tblup_amd import evolver as EV
    from tests.test_evolver import ADAPT, SADE_META, _adaptive_run, _sade_state
    z = np.load(os.path.join(ADAPT, "sade.npz"))
    _adaptive_run(z, name, SADE_META[name], lambda d, g, clip: EV.SaDE(d, clip), (500, 600, 400), tmp_path,
                  _sade_state)
