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

    def close(self):
        pass
