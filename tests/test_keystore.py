"""Device key store validity: recorded genomes stay writable through numpy's write paths
(Individual.__setitem__, individual.py:119-120, and the rest) and any in-place write drops the
device copy; a write the store cannot see raises instead of leaving a stale device row."""
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


@pytest.mark.parametrize("write", [
    lambda g: np.copyto(g, np.arange(g.size, dtype=np.float64)[::-1]),
    lambda g: g.sort(),
    lambda g: g.fill(0.5),
    lambda g: g.put([0, 1], [2.0, 3.0]),
    lambda g: g.partition(2),
    lambda g: np.put(g, [2], [9.0]),
    lambda g: np.place(g, g > 0.5, [0.25]),
    lambda g: np.putmask(g, g > 0.5, 0.75),
    lambda g: np.add.at(g, [0, 0, 3], 1.0),
    lambda g: np.clip(g, 0.2, 0.6, out=g),
    lambda g: np.negative(g[::-2], out=g[::-2]),
    lambda g: g[1:4].__setitem__(slice(None), -1.0),
    lambda g: g.byteswap(inplace=True),
], ids=["copyto", "sort", "fill", "put", "partition", "np.put", "np.place", "np.putmask", "ufunc.at",
        "clip-out", "reversed-view-out", "view-setitem", "byteswap"])
def test_every_numpy_write_path_marks_stale(write):
    """Each in-place write numpy offers either marks the recorded array stale (and writes, with
    numpy's own result) or raises; none leaves it looking unchanged."""
    rng = np.random.default_rng(2)
    vals = rng.uniform(size=8)
    g = track(vals.copy())
    want = vals.copy()
    write(want)                                          # numpy's result on a plain array
    write(g)
    assert g._stale
    np.testing.assert_array_equal(g.view(np.ndarray), want)


def test_unseen_write_paths_raise():
    """Writes the store cannot intercept meet a read-only array: the recorded memory has no
    other writable numpy alias (the owner / block is locked too)."""
    owner = np.random.default_rng(1).uniform(size=6)
    g = track(owner)
    for write in (lambda: np.random.shuffle(g), lambda: np.asarray(g).__setitem__(0, 1.0),
                  lambda: g.view(np.ndarray).__setitem__(0, 1.0), lambda: owner.__setitem__(0, 1.0),
                  lambda: g.base.__setitem__(0, 1.0)):
        with pytest.raises(ValueError):
            write()
    assert not g._stale
    cp = g.copy()                                        # copies are plain, writable, untracked
    cp[0] = 5.0
    assert not g._stale and cp[0] == 5.0


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
    with pytest.raises(ValueError):                      # an old plain reference cannot write behind
        plain[0][0] = 1.0                                # the store's back (adopt=True)
    ind._genome[0] = 1.0                                 # the individual's own writes still work
    assert store.lookup(ind) is None and plain[0][0] == 1.0


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
        # writes that are neither item assignment nor ufuncs
        np.copyto(kids[4].get_internal_genome(), rng.uniform(size=p))
        kids[5].get_internal_genome().sort()
        store = DeviceKeyStore.get(0)
        assert store.lookup(kids[2]) is None and store.lookup(kids[4]) is None and store.lookup(kids[5]) is None
        assert store.lookup(kids[3]) is not None
        ev.evaluate(popn, kids, 1)
        T, V = ev.training_indices, ev.validation_indices
        for j in (2, 3, 4, 5):
            want = O.blup(O.decode_randkeys(kids[j].get_internal_genome(), k), T, V, geno.astype(np.float64),
                          pheno, 0.4)
            assert abs(kids[j].fitness - want) < 1e-9


def test_track_rows_matches_track():
    """track_rows (round 6: a block's rows tracked in one pass) gives every row the semantics of
    track(row): its own owner, staleness per row, writes land in the block, the block is found
    from the row (the evolver's compaction), views stay tracked and copies are plain."""
    from tblup_amd.keystore import track_rows
    block = np.arange(24, dtype=np.float64).reshape(4, 6)
    rows = track_rows(block)
    block.flags.writeable = False
    assert len(rows) == 4 and all(type(r) is TrackedGenome for r in rows)
    assert all(r._blk is block and not r.flags.writeable for r in rows)
    rows[2][1] = -1.0                          # the private writable alias
    assert rows[2]._stale and not rows[1]._stale and not rows[3]._stale
    assert block[2, 1] == -1.0
    with pytest.raises(ValueError):
        np.asarray(rows[0])[0] = 5.0           # no other writable alias
    v = rows[3][1:4]
    assert v._tracked() and v._root() is rows[3]
    np.copyto(v, 7.0)
    assert rows[3]._stale and np.all(block[3, 1:4] == 7.0)
    c = rows[1].copy()
    assert not c._tracked() and np.array_equal(c, block[1])
    assert np.array_equal(copy.deepcopy(rows[0]), block[0])
