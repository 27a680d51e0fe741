"""Knockout local search (tblup/local.py) with speculative batched evaluation.

The reference's KnockoutLocalSearch.search (local.py:50-76) walks the best
genome once, knocking index i out and keeping it out iff the fitness of the
smaller genome beats the best so far -- k sequential single-individual blup()
calls.  Here the next `window` candidates are evaluated in ONE batched GPU call,
all relative to the current mask: every candidate before the first accepted one
was evaluated against exactly the mask the sequential walk would have used, so
those decisions stand; the first acceptance changes the mask, and the walk
resumes after it with a fresh batch.  Decisions are therefore identical to the
sequential walk on the same fitness values.  Acceptances are NOT rare (about half of
the knock-outs from a config-2 population's best, `profiles/r03a_knockout.json`), so
the default speculates over a decision tree instead of a line (knockout_walk).
"""
import heapq
from copy import deepcopy

import numpy as np

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


def knockout_walk(genome, best_fitness, evaluate_batch, window=256, tree=True, latency=130.0):
    """The greedy knockout walk of local.py:62-76 with speculative batches.

    evaluate_batch(list of index arrays) -> fitness array.  Returns (mask, best_fitness,
    n_batches).

    tree=False: linear windows -- the next `window` knock-outs against the current mask; the
    walk resumes after the first acceptance.
    tree=True (default): decision-tree speculation.  A node is a path of decisions for the next
    positions (each knock-out accepted or rejected) plus the candidate after it; the batch holds
    the most probable nodes (acceptance rate p estimated from the walk so far, node probability
    p^accepted (1-p)^rejected along its path), and the walk then follows the actual decisions
    through the evaluated tree -- every node on the followed path was evaluated against exactly
    the mask and best fitness the sequential walk has there, so the decisions are the
    sequential walk's.  The batch size B <= window maximises the expected decisions resolved
    (the sum of the selected nodes' probabilities) per batch cost `latency + B` (a batch costs a
    fixed latency of about `latency` individuals' throughput: config 2 on one MI355X, B = 1
    0.86 ms, B = 256 2.5 ms).  With p = 0.5 a batch of 32-64 resolves 5-6 decisions where a
    linear window resolves 2."""
    genome = np.asarray(genome)
    n = len(genome)
    mask = np.ones(n, dtype=bool)
    i, n_batches = 0, 0
    if not tree:
        while i < n:
            cand = list(range(i, min(n, i + window)))
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
    accepted = decided = 0
    while i < n:
        p = (accepted + 1.0) / (decided + 2.0)
        # best-first expansion of the decision tree rooted at position i
        heap, order, tick = [(-1.0, 0, ())], [], 1
        while heap and len(order) < window:
            negp, _, path = heapq.heappop(heap)
            order.append((path, -negp))
            if i + len(path) + 1 < n:
                heapq.heappush(heap, (negp * p, tick, path + (True,)))
                heapq.heappush(heap, (negp * (1.0 - p), tick + 1, path + (False,)))
                tick += 2
        gain = np.cumsum([q for _, q in order])
        B = int(np.argmax(gain / (latency + np.arange(1, len(order) + 1)))) + 1
        nodes = {}
        subsets = []
        for path, _ in order[:B]:
            m = mask.copy()
            for d, acc in enumerate(path):
                if acc:
                    m[i + d] = False
            m[i + len(path)] = False
            nodes[path] = len(subsets)
            subsets.append(genome[m])
        fits = np.asarray(evaluate_batch(subsets), dtype=np.float64)
        n_batches += 1
        path = ()
        while i < n and path in nodes:
            f = fits[nodes[path]]
            acc = bool(f > best_fitness)    # local.py:69-71
            if acc:
                best_fitness = f
                mask[i] = False
                accepted += 1
            decided += 1
            path += (acc,)
            i += 1
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
