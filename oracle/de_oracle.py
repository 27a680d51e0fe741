"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

Numpy restatement of one generation of the reference's differential-evolution
step (ianwhale/tblup `tblup/evolver.py`), the checker of the GPU DE step
(tblup_amd/csrc/k_de.hip).  Only `tests/` and `bench.py`'s host-timing leg use
it; the product path never imports it.

It consumes python's `random` and numpy's global RandomState exactly like the
reference's sequential loop, so a seeded call reproduces the reference's
children and leaves both generators in the reference's state.  Pinned by
`tests/golden/de.npz` (generated from the reference's own evolvers by
`tests/golden/make_golden.py::gen_de`, test `tests/test_evolver.py`).
"""
import random

import numpy as np


def exclusive_randrange(begin, end, exclude):
    """tblup/utils.py:21-36."""
    r = random.randrange(begin, end)
    exclude = set(exclude)
    assert len(exclude) < (end - begin), "Exclusion range larger than random range."
    while r in exclude:
        r = random.randrange(begin, end)
    return r


def binary_crossover(target, mutant, cr):
    """BinaryCrossoverMixin.crossover (evolver.py:63-82) on raw genomes."""
    genome_len = len(target)
    fixed = random.randrange(0, genome_len)
    crossover = np.random.rand(genome_len) < cr
    crossover[fixed] = True
    return np.where(crossover, mutant, target)


def de_generation(genomes, fitness, generation, strategy, dimensionality, cr, F, clip=True):
    """Children internal genomes of one `evolve` call (evolver.py:140-157 / 223-244).

    genomes: list of internal genomes (population order); fitness: list of floats.
    strategy 'de_rand_1' (evolver.py:103-138) or 'de_currenttobest_1' (evolver.py:179-221,
    always clipped: evolve() does not pass clip)."""
    mi = 5 if generation % 5 == 0 else F
    n = len(genomes)
    out = []
    if strategy == "de_rand_1":
        for i in range(n):
            a = exclusive_randrange(0, n, [i])
            b = exclusive_randrange(0, n, [i, a])
            c = exclusive_randrange(0, n, [i, a, b])
            mutant = genomes[a] + mi * (genomes[b] - genomes[c])
            child = binary_crossover(genomes[i], mutant, cr)
            if clip:
                child = np.clip(child, 0, dimensionality - 1)
            out.append(child)
        return out
    if strategy == "de_currenttobest_1":
        best_index = max(range(n), key=lambda j: fitness[j])   # first maximum, like max(population)
        best = genomes[best_index]
        for i in range(n):
            excl = [i, best_index]
            a = exclusive_randrange(0, n, excl)
            excl.append(a)
            b = exclusive_randrange(0, n, excl)
            x = genomes[i]
            mutant = x + mi * (best - x) + mi * (genomes[a] - genomes[b])
            child = binary_crossover(x, mutant, cr)
            out.append(np.clip(child, 0, dimensionality - 1))
        return out
    raise NotImplementedError(strategy)


def de_children(genomes, strategies, donors, fixed, F, crs, clip, hi):
    """Children of one SaDE generation (evolver.py:523-545) from the host's draws: per individual
    DE/rand/1 (strategy 0, donors a, b, c: evolver.py:118-132) or DE/current-to-best/1 (strategy 1,
    donors best, a, b: evolver.py:199-214) with its own crossover rate and the caller's forced
    position, one np.random.rand(L) per individual in order (evolver.py:74-82), optional clip."""
    out = []
    for i, x in enumerate(genomes):
        a, b, c = (genomes[j] for j in donors[i])
        mutant = a + F * (b - c) if strategies[i] == 0 else x + F * (a - x) + F * (b - c)
        take = np.random.rand(len(x)) < crs[i]
        take[fixed[i]] = True
        child = np.where(take, mutant, x)
        out.append(np.clip(child, 0, hi) if clip else child)
    return out
