"""Knockout local search (tblup/local.py:50-76): the speculative batched walk makes the
same decisions as the reference's sequential loop (host logic; fitness from the oracle)."""
import os

import numpy as np
import pytest

from oracle import blup_oracle as O
from tblup_amd.local import knockout_walk


def _sequential(genome, best_fitness, fitness):
    """The reference loop, restated (local.py:65-76)."""
    mask = np.ones(len(genome), dtype=bool)
    for i in range(len(genome)):
        mask[i] = False
        f = fitness(genome[mask])
        if f > best_fitness:
            best_fitness = f
        else:
            mask[i] = True
    return mask, best_fitness


@pytest.mark.parametrize("tree", [False, True])
@pytest.mark.parametrize("window", [1, 3, 8, 256])
def test_batched_knockout_matches_sequential(golden_dir, window, tree):
    z = np.load(os.path.join(golden_dir, "blup_200x1000.npz"))
    g, y, T, V = z["geno"].astype(np.float64), z["pheno"], z["T"], z["V"]
    genome = np.sort(np.random.default_rng(5).choice(1000, 40, replace=False))

    def fitness(sel):
        return O.blup(sel, T, V, g, y, 0.4)

    start = fitness(genome)
    ref_mask, ref_best = _sequential(genome, start, fitness)
    calls = []

    def batch(subsets):
        calls.append(len(subsets))
        return [fitness(s) for s in subsets]

    mask, best, n_batches = knockout_walk(genome, start, batch, window, tree=tree)
    np.testing.assert_array_equal(mask, ref_mask)
    assert best == ref_best
    assert (~ref_mask).sum() >= 1            # the case exercises at least one acceptance
    assert n_batches == len(calls)
    assert max(calls) <= window
    if window >= len(genome) and not tree:
        assert n_batches <= 1 + (~ref_mask).sum()


@pytest.mark.parametrize("rate", [0.02, 0.3, 0.5, 0.9])
def test_tree_walk_matches_sequential_synthetic(rate):
    """Decision-tree speculation on a synthetic fitness (a deterministic function of the
    subset, accepting about `rate` of the knock-outs early on): identical masks and best
    fitness, and fewer batches than the linear windows whenever acceptances are frequent."""
    genome = np.arange(300)

    def fitness(sel):
        h = np.random.default_rng([int(x) for x in np.setdiff1d(genome, sel)] + [7]).random()
        return (len(genome) - len(sel)) * 1e-3 + (h < rate) * 1.0 + h * 1e-6

    def batch(subsets):
        return [fitness(s) for s in subsets]

    start = 0.5
    ref_mask, ref_best = _sequential(genome, start, fitness)
    m1, b1, n1 = knockout_walk(genome, start, batch, 64, tree=False)
    m2, b2, n2 = knockout_walk(genome, start, batch, 64, tree=True)
    for m, b in ((m1, b1), (m2, b2)):
        np.testing.assert_array_equal(m, ref_mask)
        assert b == ref_best
    if (~ref_mask).sum() > 20:
        assert n2 < n1
