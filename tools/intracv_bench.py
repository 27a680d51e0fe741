"""IntraGCV (k = 5 folds inside every fitness evaluation, evaluator.py:494-537) against one
fold's evaluation, through the drop-in classes on the GPU: config 1 (200 x 1000, k = 100,
pop 32) and config 2 (2000 x 50k, k = 1000, pop 256).  Prints one JSON line per config with
the median time of a fresh population's evaluate() for the plain evaluator (one split) and
for IntraGCV (its k folds one after another on the evaluator's context).  A variant with the
folds on k contexts driven from k host threads measured slower (config 1: 1.54 vs 0.91 ms,
config 2: 35.8 vs 32.3 ms) and was dropped."""
import json
import os
import random
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed_evals(ev, make_pop, reps):
    ts = []
    with ev:
        for r in range(reps + 1):
            pop = make_pop()
            t0 = time.perf_counter()
            ev.evaluate(pop, pop, 0)
            if r:
                ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3


def main():
    import torch  # noqa: F401
    from oracle import blup_oracle as O
    from tests.ga_driver import RandomKeyIndividual
    from tblup_amd import evaluator as E
    for name, n, p, k, pop in (("config1", 200, 1000, 100, 32), ("config2", 2000, 50000, 1000, 256)):
        rng = np.random.default_rng(3)
        geno = O.synth_geno(rng, n, p)
        tmp = tempfile.mkdtemp()
        gp, pp = os.path.join(tmp, "g.npy"), os.path.join(tmp, "y.npy")
        np.save(gp, geno)
        np.save(pp, rng.standard_normal(n))

        def make_pop():
            return [RandomKeyIndividual(k, p, genome=rng.uniform(size=p)) for _ in range(pop)]
        random.seed(1)
        np.random.seed(1)
        one = timed_evals(E.BlupParallelEvaluator(gp, pp, 0.4), make_pop, 5)
        random.seed(1)
        np.random.seed(1)
        intra = timed_evals(E.IntraGCVBlupParallelEvaluator(gp, pp, 0.4, n_folds=5), make_pop, 5)
        print(json.dumps({"config": name, "pop": pop, "one_split_ms": round(one, 3), "intragcv_ms": round(intra, 3),
                          "ratio": round(intra / one, 2)}), flush=True)


if __name__ == "__main__":
    main()
