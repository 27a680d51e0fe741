"""Device key store validity: recorded genomes stay writable (Individual.__setitem__,
individual.py:119-120) and any in-place write drops the device copy."""
import copy
import pickle

import numpy as np
import pytest

from tblup_amd.keystore import DeviceKeyStore, TrackedGenome, track


def test_tracked_genome_notices_writes():
    a = track(np.arange(10, dtype=np.float64))
    assert isinstance(a, TrackedGenome) and not a._stale
    assert np.argsort(a)[-3:].tolist() == [7, 8, 9]      # reads behave like the ndarray
    b = a + 1.0
    assert type(b) is np.ndarray                         # computations give plain arrays
    a[3] = 5.0                                           # Individual.__setitem__
    assert a._stale and a[3] == 5.0
    c = track(np.zeros(6))
    v = c[2:4]
    v[0] = 1.0                                           # write through a view
    assert c._stale and c[2] == 1.0
    d = track(np.zeros(4))
    d += 1.0                                             # in-place ufunc
    assert d._stale and np.all(d == 1.0)
    e = track(np.zeros(4))
    np.multiply(np.ones(4), 3.0, out=e)                  # out= argument
    assert e._stale and np.all(e == 3.0)
    f = track(np.ones(3))
    assert type(copy.deepcopy(f)) is np.ndarray and type(pickle.loads(pickle.dumps(f))) is np.ndarray
    assert not f._stale


class _Ind:
    def __init__(self, uid, g):
        self.uid, self._genome, self.length = uid, g, 5


def test_store_drops_written_and_replaced_genomes():
    import torch
    store = DeviceKeyStore(0)
    t = torch.zeros((3, 4), dtype=torch.float64)        # a CPU stand-in for the device block
    arrays = [track(np.full(4, float(i))) for i in range(3)]
    inds = [_Ind(100 + i, arrays[i]) for i in range(3)]
    store.record(t, inds, arrays)
    assert all(store.lookup(i) is not None for i in inds)
    inds[0]._genome[1] = 7.0                             # in-place write -> host path
    assert store.lookup(inds[0]) is None
    inds[1]._genome = np.zeros(4)                        # set_internal_genome -> host path
    assert store.lookup(inds[1]) is None
    inds[2].length = 6                                   # fill() -> host path
    assert store.lookup(inds[2]) is None
    # plain arrays are adopted as tracked views of the same buffer only when asked
    plain = [np.full(4, 9.0)]
    ind = _Ind(200, plain[0])
    store.record(t, [ind], plain)
    assert store.lookup(ind) is None and ind._genome is plain[0]
    store.record(t, [ind], plain, adopt=True)
    assert isinstance(ind._genome, TrackedGenome) and np.shares_memory(ind._genome, plain[0])
    assert store.lookup(ind) is not None


@pytest.mark.gpu
def test_gpu_write_after_evolve_is_seen(gpu, tmp_path):
    """A child's keys written in place after the GPU DE step are evaluated from the host,
    with the written values (the stale device row is not used)."""
    import random
    from oracle import blup_oracle as O
    from tblup_amd.evaluator import BlupParallelEvaluator
    from tblup_amd.evolver import DERandOneEvolver
    from tests.helpers import Pop, RandomKeyIndividual
    rng = np.random.default_rng(3)
    n, p, k, pop = 300, 2000, 100, 8
    geno = O.synth_geno(rng, n, p)
    pheno = rng.standard_normal(n)
    np.save(tmp_path / "g.npy", geno)
    np.save(tmp_path / "y.npy", pheno)
    random.seed(1)
    np.random.seed(1)
    ev = BlupParallelEvaluator(str(tmp_path / "g.npy"), str(tmp_path / "y.npy"), 0.4)
    inds = [RandomKeyIndividual(rng.uniform(size=p), k) for _ in range(pop)]
    with ev:
        popn = Pop(inds, 1)
        ev.evaluate(popn, popn, 0)
        kids = DERandOneEvolver(p, 0.8, 0.5, False).evolve(popn)
        g = kids[2].get_internal_genome()
        top = np.argsort(g)[-k:]
        g[top[:10]] = -1.0                                # knock 10 selected SNPs out in place
        assert DeviceKeyStore.get(0).lookup(kids[2]) is None
        assert DeviceKeyStore.get(0).lookup(kids[3]) is not None
        ev.evaluate(popn, kids, 1)
        T, V = ev.training_indices, ev.validation_indices
        for j in (2, 3):
            want = O.blup(O.decode_randkeys(kids[j].get_internal_genome(), k), T, V, geno.astype(np.float64),
                          pheno, 0.4)
            assert abs(kids[j].fitness - want) < 1e-9
