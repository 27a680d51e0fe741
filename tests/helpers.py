"""Test-side stand-ins for the reference's individuals and an oracle-backed engine.

The oracle engine is TEST INFRASTRUCTURE: it lets the CPU suite exercise the
evaluator's host logic (splits, archive, SNP removal, CV folds, sharding)
without a GPU.  The product evaluator never constructs it.
"""
import itertools

import numpy as np

from oracle import blup_oracle as O

_uid = itertools.count(10_000)


class KeyIndividual:
    """RandomKeyIndividual stand-in (tblup/individual.py:132-167)."""

    def __init__(self, keys, length):
        self.uid = next(_uid)
        self._genome = np.asarray(keys)
        self.length = length
        self.fitness = float("-inf")

    @property
    def genome(self):
        return O.decode_randkeys(self._genome, self.length)

    def __len__(self):
        return int(self.length)

    def set_fitness(self, f):
        self.fitness = f


    def get_internal_genome(self):
        return self._genome

    def set_internal_genome(self, genome):
        self._genome = genome

    def __deepcopy__(self, memo):
        """individual.py:43-59 / 110-118: same class and attributes, a new uid."""
        cp = self.__class__.__new__(self.__class__)
        cp.__dict__.update(self.__dict__)
        cp.uid = next(_uid)
        return cp


class CoevoIndividual(KeyIndividual):
    """CoevolutionIndividual stand-in (tblup/individual.py:170-222): the length rides along
    as the last element of the internal genome."""

    def __init__(self, keys, length, dimensionality):
        super().__init__(keys, length)
        self.dimensionality = dimensionality

    def get_internal_genome(self):
        return np.append(self._genome, self.length)

    def set_internal_genome(self, genome):
        if len(genome) == self.dimensionality + 1:
            if genome[-1] < 1:
                self.length = 1
            elif genome[-1] > self.dimensionality:
                self.length = self.dimensionality
            else:
                self.length = genome[-1]
            self._genome = np.delete(genome, -1)
        elif len(genome) == self.dimensionality:
            self._genome = genome
        else:
            raise RuntimeError("Genome of invalid length, must be dimensionality d or d + 1.")


class Pop:
    """The slice of tblup.Population the evolvers read (.population, .generation, [], len)."""

    def __init__(self, individuals, generation):
        self.population = individuals
        self.generation = generation

    def __getitem__(self, i):
        return self.population[i]

    def __len__(self):
        return len(self.population)


class RandomKeyIndividual(KeyIndividual):
    """Same stand-in under the reference's class name: the evaluator batch-decodes
    RandomKeyIndividual / CoevolutionIndividual genomes on the GPU (by class name)."""


class IdxIndividual(KeyIndividual):
    """IndexIndividual stand-in (tblup/individual.py:73-130)."""

    @property
    def genome(self):
        return O.decode_index(self._genome)

    def __len__(self):
        return len(self._genome)


class OracleEngine:
    """Same evaluate() contract as tblup_amd.engine.GpuBlupEngine, computed by the oracle."""

    def __init__(self, data, labels):
        self.data = np.asarray(data, dtype=np.float64)
        self.labels = np.asarray(labels, dtype=np.float64)
        self.calls = 0

    def evaluate(self, genomes, train, valid, h2, branch="auto", return_ebv=False):
        self.calls += 1
        out = []
        for g in genomes:
            if branch == "auto":
                out.append(O.blup(g, train, valid, self.data, self.labels, h2))
            elif branch == "gblup":
                out.append(O.gblup(g, train, valid, self.data, self.labels, h2))
            else:
                out.append(O.snp_blup(g, train, valid, self.data, self.labels, h2))
        return np.array(out, dtype=np.float64)

    def evaluate_folds(self, genomes, splits, h2, branch="auto"):
        """GpuBlupEngine.evaluate_folds: (n_splits, B), row f = evaluate(genomes, *splits[f])."""
        return np.array([self.evaluate(genomes, t, v, h2, branch) for t, v in splits]).reshape(len(splits), -1)

    def close(self):
        pass


def shard_population(pop, n_snps, k, seed=11):
    """A population of `pop` selected-index sets where individual i comes from its own seed:
    the same individuals in every process, whatever the sharding (tests/test_gpu_shards.py)."""
    return [np.random.default_rng((seed, i)).choice(n_snps, k, replace=False) for i in range(pop)]
