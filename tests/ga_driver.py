"""TEST INFRASTRUCTURE: a restatement of the reference's `main()` control loop.

The reference's control plane (main.py, Population, Monitor, selector, stop
condition, individuals) is out of this build's scope and the reference itself never
travels to the GPU box, so the end-to-end drop-in test drives the product's
evaluator / evolver / local search through this restatement of it:

  main.py:10-45            main(): seeds, build_kwargs, `with evaluator:`, generations,
                           evaluate_testing "Testing" row, archive, local search AFTER the
                           `with` block
  tblup/utils.py:39-76     build_kwargs (order of the factory calls = RNG order)
  tblup/population.py      __init__ (initial population, evaluate, report, archive,
                           report_testing) and do_generation
  tblup/selector.py        DifferentialEvolutionSelector
  tblup/monitor.py         gather_stats / get_row_summary (median quirk, rounding),
                           save_archive (str/int key quirk), report_testing, removals log,
                           report_local
  tblup/stop_condition.py  StopCondition / HeritabilityStopCondition
  tblup/individual.py      IndexIndividual, RandomKeyIndividual, CoevolutionIndividual
                           (constructor RNG draws, genome decode, deepcopy with new uid,
                           Coevolution's set_fitness penalty)

It covers the options `tests/golden/make_golden.py::MAIN_CASES` uses (no seeder, no
feature scheduler, no splitter) and is pinned by `tests/golden/main_runs.npz`, which the
reference's own main() produced: tests/test_main_flow.py runs it with the oracle engine
and evolver on the CPU (pinning this restatement) and with the tblup_amd drop-ins on the
GPU.  Files are not written: the CSV / JSON contents are returned as text.
"""
import argparse
import csv
import io
import itertools
import json
import random
from copy import deepcopy
from math import sqrt

import numpy as np

_uid = itertools.count()


# --------------------------------------------------------------------------- config.py
def parse_args(argv):
    """The flags of tblup/config.py the MAIN_CASES use, with the reference's defaults."""
    def boollike(v):
        return v.lower() in ("yes", "true", "t", "y", "1")
    p = argparse.ArgumentParser()
    p.add_argument("-s", "--seed", type=int, default=0)
    p.add_argument("-p", "--processes", type=int, default=4)
    p.add_argument("-o", "--output", default=None)
    p.add_argument("--geno")
    p.add_argument("--pheno")
    p.add_argument("--splitter", default=None)
    p.add_argument("--pca_outliers", type=boollike, default=False)
    p.add_argument("--regressor", default="blup")
    p.add_argument("--remove_snps", type=boollike, default=False)
    p.add_argument("--removal_r", type=int, default=None)
    p.add_argument("--heritability", type=float, default=0.4)
    p.add_argument("--cv_folds", type=int, default=5)
    p.add_argument("--generations", type=int, default=100)
    p.add_argument("--population_size", type=int, default=50)
    p.add_argument("--features", type=int, default=100)
    p.add_argument("--de_strategy", default="de_rand_1")
    p.add_argument("--crossover_rate", type=float, default=0.8)
    p.add_argument("--mutation_intensity", type=float, default=0.5)
    p.add_argument("--individual", default="randkeys")
    p.add_argument("--coevolve_gamma", type=float, default=1.0)
    p.add_argument("--clip", type=boollike, default=False)
    p.add_argument("--record_testing", type=boollike, default=False)
    p.add_argument("--local_search", default=None)
    p.add_argument("--stop_condition", default=None)
    p.add_argument("--h2_alpha", type=float, default=0.0)
    a = p.parse_args(argv)
    a.REGRESSOR_TYPE_BLUP = "blup"
    a.REGRESSOR_TYPE_INTRACV_BLUP = "intracv_blup"
    a.REGRESSOR_TYPE_INTERCV_BLUP = "intercv_blup"
    a.REGRESSOR_TYPE_MONTECV_BLUP = "montecv_blup"
    a.LOCAL_SEARCH_KNOCKOUT = "knockout"
    a.dimensionality = int(np.load(a.geno, mmap_mode="r").shape[1])
    return a


# --------------------------------------------------------------------------- individuals
class IndexIndividual:
    def __init__(self, length, dimensionality, genome=None, gamma=1.0):
        self.uid = next(_uid)
        self.length = length
        self.dimensionality = dimensionality
        self.fitness = float("-inf")
        self._genome = genome if genome is not None else np.random.randint(0, dimensionality, length)

    def __deepcopy__(self, memo):
        cp = self.__class__.__new__(self.__class__)
        cp.__dict__.update(self.__dict__)
        cp.uid = next(_uid)
        cp._genome = deepcopy(self._genome)
        return cp

    def set_fitness(self, fitness):
        self.fitness = fitness

    @property
    def genome(self):
        return self._genome.astype(int)

    def get_internal_genome(self):
        return self._genome

    def set_internal_genome(self, genome):
        self._genome = genome

    def __len__(self):
        return len(self._genome)

    def __getitem__(self, item):
        return self._genome[item]

    def __setitem__(self, key, value):
        self._genome[key] = value


class RandomKeyIndividual(IndexIndividual):
    def __init__(self, length, dimensionality, genome=None, gamma=1.0):
        # individual.py:138-151: the IndexIndividual constructor runs first without the
        # genome, so numpy's randint draw happens before the keys are drawn
        super().__init__(length, dimensionality)
        self._genome = genome if genome is not None else np.random.uniform(size=dimensionality)

    @property
    def genome(self):
        return np.argsort(self._genome)[-int(self.length):]

    def __len__(self):
        return int(self.length)


class CoevolutionIndividual(RandomKeyIndividual):
    def __init__(self, length, dimensionality, genome=None, gamma=1.0):
        super().__init__(length, dimensionality, genome=genome)
        self.length = random.randint(int(length * 0.9), int(length * 1.1))
        self.gamma = gamma

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

    def set_fitness(self, fitness):
        self.fitness = fitness - self.gamma * (self.length / self.dimensionality)


INDIVIDUALS = {"index": IndexIndividual, "randkeys": RandomKeyIndividual, "coevolve": CoevolutionIndividual}


# --------------------------------------------------------------------------- monitor.py
class Monitor:
    ROUND_DECIMALS = 4
    MAX_FITNESS_INDEX, MIN_FITNESS_INDEX, MEDIAN_FITNESS_INDEX, MEAN_FITNESS_INDEX = 1, 2, 3, 4
    HEADER = ["generation", "max_fitness", "min_fitness", "median_fitness", "mean_fitness", "stdev_fitness", "len"]

    def __init__(self, args):
        self.results = [self.HEADER]
        self.testing = [self.HEADER] if args.record_testing else None
        self.archive = {}
        self.local = None
        self.removals = []
        self.gen_fitness = []
        self.gen_len = []

    def write(self, row):
        self.results.append(row)
        return row

    def report(self, population):
        return self.write(self.gather_stats(population))

    def report_testing(self, population):
        res = population.evaluator.evaluate_testing(population)
        self.testing.append([population.generation] + self.get_row_summary(list(res)))

    def save_archive(self, population):
        # monitor.py:183-201: the JSON round trip turns keys into str, so the int
        # comparison never matches and a run ends with the final generation's entry too
        if len(self.archive) == 0 or population.generation != max(self.archive.keys()):
            best = max(population, key=lambda individual: individual.fitness)
            self.archive[str(population.generation)] = {
                "fitness": best.fitness,
                "genome": [int(i) for i in best.genome],
                "combined_genome": [int(i) for i in population.evaluator.snp_remover.combine_with_removed(best.genome)],
            }

    def report_local(self, genome, fitness):
        self.local = {"fitness": fitness, "length": len(genome), "genome": [int(i) for i in genome]}

    def gather_stats(self, population):
        fits, lens = [], 0
        for indv in population:
            fits.append(indv.fitness)
            lens += len(indv)
        self.gen_fitness.append([float(f) for f in fits])
        self.gen_len.append([float(len(i)) for i in population])
        return [population.generation] + self.get_row_summary(fits) + [lens / len(population)]

    def get_row_summary(self, fitnesses):
        fitnesses.sort()
        median_idx = len(fitnesses) / 2.0
        if int(median_idx) == median_idx:
            median = fitnesses[int(median_idx)]
        else:
            median = (fitnesses[int(median_idx)] + fitnesses[int(median_idx) + 1]) / 2
        r = self.ROUND_DECIMALS
        return [round(fitnesses[-1], r), round(fitnesses[0], r), round(median, r),
                round(np.mean(fitnesses).item(), r), round(np.std(fitnesses, ddof=1).item(), r)]

    def log_snp_removal_event(self, generation):
        self.removals.append(generation)

    @staticmethod
    def csv_text(rows):
        f = io.StringIO()
        w = csv.writer(f, lineterminator="\n")   # the reference reads its files back in text mode
        for r in rows:
            w.writerow(r)
        return f.getvalue()


# --------------------------------------------------------------------------- stop_condition.py
class StopCondition:
    def should_stop(self, population, stats):
        return False


class HeritabilityStopCondition(StopCondition):
    def __init__(self, h2, alpha, kind):
        self.threshold = sqrt(h2) * (1 + alpha)
        self.index = {"h2_max": Monitor.MAX_FITNESS_INDEX, "h2_min": Monitor.MIN_FITNESS_INDEX,
                      "h2_mean": Monitor.MEAN_FITNESS_INDEX, "h2_median": Monitor.MEDIAN_FITNESS_INDEX}[kind]

    def should_stop(self, population, stats):
        return stats[self.index] > self.threshold


# --------------------------------------------------------------------------- population.py
class Population:
    ARCHIVE_INTERVAL = 100

    def __init__(self, evolver, evaluator, individual, length, dimensionality, num_individuals, monitor,
                 stop_condition, record_testing=False, coevolve_gamma=1.0):
        self.evolver, self.evaluator, self.monitor = evolver, evaluator, monitor
        self.population = [individual(length, dimensionality, gamma=coevolve_gamma) for _ in range(num_individuals)]
        self.record_testing = record_testing
        self.dimensionality = dimensionality
        self.stop_condition = stop_condition
        self.generation = 0
        self.evaluator.evaluate(self, self, self.generation)
        self.monitor.report(self)
        self.monitor.save_archive(self)
        if self.record_testing:
            self.monitor.report_testing(self)
        self.generation += 1

    def __getitem__(self, index):
        return self.population[index]

    def __len__(self):
        return len(self.population)

    def do_generation(self):
        next_pop = self.evolver.evolve(self)
        self.evaluator.evaluate(self, next_pop, self.generation)
        # DifferentialEvolutionSelector.select (selector.py:20-38)
        self.population = [c if c.fitness > p.fitness else p for p, c in zip(self.population, next_pop)]
        stats = self.monitor.report(self)
        if self.generation % self.ARCHIVE_INTERVAL == 0:
            self.monitor.save_archive(self)
        if self.record_testing:
            self.monitor.report_testing(self)
        self.generation += 1
        return not self.stop_condition.should_stop(self, stats)


# --------------------------------------------------------------------------- main.py
def run_main(argv, get_evaluator, get_evolver, get_local_search):
    """main() of main.py:10-45 with the given factories; returns what the reference's run
    leaves in its results directory (as text / arrays) plus the per-generation fitness."""
    args = parse_args(argv)
    random.seed(args.seed)
    np.random.seed(args.seed)
    evolver = get_evolver(args)
    evaluator = get_evaluator(args)
    individual = INDIVIDUALS[args.individual]
    monitor = Monitor(args)
    stop = (HeritabilityStopCondition(args.heritability, args.h2_alpha, args.stop_condition)
            if args.stop_condition is not None else StopCondition())
    final_genomes = None
    with evaluator:
        population = Population(evolver, evaluator, individual, args.features, args.dimensionality,
                                args.population_size, monitor, stop, args.record_testing, args.coevolve_gamma)
        splits = {"train": np.asarray(evaluator.training_indices), "validation": np.asarray(evaluator.validation_indices),
                  "testing": np.asarray(evaluator.testing_indices)}
        for _ in range(1, args.generations + 1):
            if not population.do_generation():
                break
        final_genomes = [np.asarray(i.genome, dtype=np.int64) for i in population]
        results = evaluator.evaluate_testing(population)
        monitor.write(["Testing"] + monitor.get_row_summary(list(results)) + ["Final"])
        monitor.save_archive(population)
    if args.local_search is not None:
        genome, fitness = get_local_search(args, population).search()
        monitor.report_local(genome, fitness)
    return {
        "results_csv": Monitor.csv_text(monitor.results),
        "testing_csv": Monitor.csv_text(monitor.testing) if monitor.testing is not None else "",
        "archive": monitor.archive,
        "local": monitor.local,
        "removals": "".join("%d\n" % g for g in monitor.removals),
        "splits": splits,
        "gen_fitness": np.array(monitor.gen_fitness),
        "gen_len": np.array(monitor.gen_len),
        "final_genomes": final_genomes,
    }


# --------------------------------------------------------------------------- CPU stand-ins
class OracleEvolver:
    """The reference's DE evolvers (evolver.py:86-244) through oracle/de_oracle.py: children
    are deep copies of the parents with the oracle's child genomes (CPU checker only)."""

    def __init__(self, args):
        self.args = args

    def evolve(self, population):
        from oracle import de_oracle
        a = self.args
        genomes = [population[i].get_internal_genome() for i in range(len(population))]
        fits = [population[i].fitness for i in range(len(population))]
        kids = de_oracle.de_generation(genomes, fits, population.generation, a.de_strategy, a.dimensionality,
                                       a.crossover_rate, a.mutation_intensity, a.clip)
        out = []
        for i, g in enumerate(kids):
            c = deepcopy(population[i])
            c.set_internal_genome(g)
            out.append(c)
        return out


def compare(run, z, name, fit_atol=1e-9):
    """Assert a run_main() result equals the reference's main_runs.npz entry `name`."""
    pre = name + "_"
    gf = z[pre + "gen_fitness"]
    assert run["gen_fitness"].shape == gf.shape, (run["gen_fitness"].shape, gf.shape)
    np.testing.assert_allclose(run["gen_fitness"], gf, rtol=0, atol=fit_atol)
    np.testing.assert_array_equal(run["gen_len"], z[pre + "gen_len"])
    for part in ("train", "validation", "testing"):
        np.testing.assert_array_equal(run["splits"][part], z[pre + part])
    off = z[pre + "final_off"]
    idx = z[pre + "final_idx"]
    assert len(run["final_genomes"]) == len(off) - 1
    for j, g in enumerate(run["final_genomes"]):
        np.testing.assert_array_equal(g, idx[off[j]:off[j + 1]])
    assert run["results_csv"] == str(z[pre + "results_csv"])
    assert run["testing_csv"] == str(z[pre + "testing_csv"])
    assert run["removals"] == str(z[pre + "removals"])
    ref_arch = json.loads(str(z[pre + "archive_json"]))
    assert sorted(run["archive"]) == sorted(ref_arch)
    for g, e in ref_arch.items():
        assert abs(run["archive"][g]["fitness"] - e["fitness"]) <= fit_atol
        assert run["archive"][g]["genome"] == e["genome"]
        assert run["archive"][g]["combined_genome"] == e["combined_genome"]
    loc = str(z[pre + "local_json"])
    if loc:
        ref_loc = json.loads(loc)
        assert run["local"]["genome"] == ref_loc["genome"] and run["local"]["length"] == ref_loc["length"]
        assert abs(run["local"]["fitness"] - ref_loc["fitness"]) <= fit_atol
    else:
        assert run["local"] is None
