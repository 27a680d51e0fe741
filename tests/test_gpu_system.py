"""The reference's DE system tests (tblup/test/system.py) on the GPU evolver: DE/rand/1
(tblup/evolver.py:86-157, clip off as `--clip false`) on the Ackley and Rastrigin
functions with Storn & Price's settings must reach the reference's values to reach within
its evaluation budgets, and the trajectory must equal the numpy oracle's."""
import math
import random

import numpy as np
import pytest

from oracle import de_oracle as D
from tests.helpers import IdxIndividual, Pop

pytestmark = pytest.mark.gpu


def ackley(genome):
    """tblup/test/system.py:9-20 (maximised: negated)."""
    g = np.clip(genome, -32, 32)
    n = float(len(g))
    s1 = float(np.sum(g ** 2.0))
    s2 = float(np.sum(np.cos(2.0 * math.pi * g)))
    return -1 * (-20.0 * math.exp(-0.2 * math.sqrt(s1 / n)) - math.exp(s2 / n) + 20 + math.e)


def rastrigin(genome):
    """tblup/test/system.py:23-32 (maximised: negated)."""
    g = np.clip(genome, -5.12, 5.12)
    return -1 * (len(g) * 10 + float(np.sum(g ** 2 - 10 * np.cos(2 * math.pi * g))))


class FnIndividual(IdxIndividual):
    """TestIndividual (system.py:35-46): real genome, genome property = the raw vector."""

    @property
    def genome(self):
        return self._genome


def run_de(func, dimension, pop_size, cr, f, eval_limit, ipr, seed, oracle=False, max_gen=None):
    from tblup_amd.evolver import DERandOneEvolver
    random.seed(seed)
    np.random.seed(seed)
    inds = [FnIndividual(np.random.rand(dimension) * (ipr[1] - ipr[0]) + ipr[0], dimension)
            for _ in range(pop_size)]
    evals = 0
    for ind in inds:
        ind.fitness = func(ind.genome)
        evals += 1
    popn = Pop(inds, 1)
    evo = DERandOneEvolver(dimension, cr, f, clip=False)
    traj = []
    while evals < eval_limit and (max_gen is None or popn.generation <= max_gen):
        if oracle:
            kids = [FnIndividual(c, dimension) for c in D.de_generation(
                [x.get_internal_genome() for x in popn.population], [x.fitness for x in popn.population],
                popn.generation, "de_rand_1", dimension, cr, f, False)]
        else:
            kids = evo.evolve(popn)
        for k in kids:
            k.fitness = func(k.genome)
            evals += 1
        popn.population = [c if c.fitness > p.fitness else p for p, c in zip(popn.population, kids)]
        traj.append(max(x.fitness for x in popn.population))
        popn.generation += 1
    return max(x.fitness for x in popn.population), traj


def test_ackley_full_run_equals_reference_algorithm(gpu):
    """system.py:151-159 settings (dimension 100, pop 50, cr 0.1, F 0.5, 37000 evaluations).
    The reference's own algorithm does not reach that test's value to reach (-e^-3): its
    evolve() uses F = 5 on every 5th generation (evolver.py:147-151) and the numpy oracle,
    which reproduces it, stalls at -19.96 (the reference's system test never ran: SURVEY.md
    section 4).  The GPU run must end exactly where the reference algorithm ends."""
    best, traj = run_de(ackley, 100, 50, 0.1, 0.5, 37000, (-32, 32), seed=0)
    ref_best, ref_traj = run_de(ackley, 100, 50, 0.1, 0.5, 37000, (-32, 32), seed=0, oracle=True)
    assert best == ref_best and traj == ref_traj


def test_rastrigin_reaches_value_to_reach(gpu):
    """system.py:161-169: dimension 100, pop 20, cr 0 (one gene per child), F 0.5, 75000 evaluations, VTR -0.9."""
    best, _ = run_de(rastrigin, 100, 20, 0.0, 0.5, 75000, (-5.12, 5.12), seed=0)
    assert best >= -0.9


def test_trajectory_equals_oracle(gpu):
    """40 generations of the Ackley run: the GPU evolver's best-fitness trajectory is the
    numpy oracle's, value for value (same RNG streams, same arithmetic)."""
    _, gpu_traj = run_de(ackley, 100, 50, 0.1, 0.5, 10 ** 9, (-32, 32), seed=3, max_gen=40)
    _, ref_traj = run_de(ackley, 100, 50, 0.1, 0.5, 10 ** 9, (-32, 32), seed=3, oracle=True, max_gen=40)
    assert gpu_traj == ref_traj
