"""Knockout local search (tblup/local.py) with speculative batched evaluation.

The reference's KnockoutLocalSearch.search (local.py:50-76) walks the best
genome once, knocking index i out and keeping it out iff the fitness of the
smaller genome beats the best so far -- k sequential single-individual blup()
calls.  Here the next `window` candidates are evaluated in ONE batched GPU call,
all relative to the current mask: every candidate before the first accepted one
was evaluated against exactly the mask the sequential walk would have used, so
those decisions stand; the first acceptance changes the mask, and the walk
resumes after it with a fresh batch.  Decisions are therefore identical to the
sequential walk on the same fitness values (acceptances are rare, so a k = 1000
walk costs ~k/window + #accepted batched calls instead of k).
"""
import numpy as np
from copy import deepcopy

from .evaluator import BlupParallelEvaluator


def get_local_search(args, population):
    """local.py:7-18."""
    if args.local_search == args.LOCAL_SEARCH_KNOCKOUT:
        return KnockoutLocalSearch(population)
    raise NotImplementedError("Local search method {} not implemented.".format(args.local_search))


class LocalSearch:
    def __init__(self, population):
        self.population = population

    def search(self):
        raise NotImplementedError()


def knockout_walk(genome, best_fitness, evaluate_batch, window=256):
    """The greedy knockout walk of local.py:62-76 with speculative batches.

    evaluate_batch(list of index arrays) -> fitness array.  Returns (mask, best_fitness,
    n_batches)."""
    genome = np.asarray(genome)
    mask = np.ones(len(genome), dtype=bool)
    i, n_batches = 0, 0
    while i < len(genome):
        cand = list(range(i, min(len(genome), i + window)))
        subsets = []
        for j in cand:
            m = mask.copy()
            m[j] = False
            subsets.append(genome[m])
        fits = np.asarray(evaluate_batch(subsets), dtype=np.float64)
        n_batches += 1
        nxt = cand[-1] + 1
        for j, f in zip(cand, fits):
            if f > best_fitness:        # local.py:69-71: keep the index masked
                best_fitness = f
                mask[j] = False
                nxt = j + 1             # later candidates assumed the old mask: re-evaluate them
                break
        i = nxt
    return mask, best_fitness, n_batches


class KnockoutLocalSearch(LocalSearch):
    """local.py:37-76, batched on the population evaluator's GPU engine."""

    def __init__(self, population, window=256):
        super().__init__(population)
        assert issubclass(population.evaluator.__class__, BlupParallelEvaluator), \
            "Knockout only implemented for BLUP regressors."
        self.window = window

    def search(self):
        """main.py:42-45 runs the search after `with evaluator:` has closed, so the
        evaluator's context is gone; like the reference's search, which np.loads the data
        itself (local.py:59), a short-lived GPU context is opened for the walk then."""
        evaluator = self.population.evaluator
        best = deepcopy(max(self.population, key=lambda individual: individual.fitness))
        genome = evaluator.snp_remover.combine_with_removed(best.genome)
        train, valid = evaluator.training_indices, evaluator.validation_indices
        engine, own = evaluator.engine, evaluator.engine is None
        if own:
            engine = evaluator._open_engine()
        try:
            def evaluate_batch(subsets):
                return engine.evaluate(subsets, train, valid, evaluator.h2)

            mask, best_fitness, _ = knockout_walk(genome, best.fitness, evaluate_batch, self.window)
        finally:
            if own:
                engine.close()
        return genome[mask], best_fitness
