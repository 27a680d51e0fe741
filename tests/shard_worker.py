"""Rank process of tests/test_gpu_shards.py: a torchrun-style rank that drives the REAL HIP
engine (no OracleEngine) on its shard of a population through the drop-in evaluator's sharded
path (BlupParallelEvaluator._fitness: shard_range -> engine.evaluate -> allgather_fitness).
Every rank uses GPU 0 of a one-GPU box and the gloo backend (RCCL needs one device per rank)."""
import json
import os
import sys


def run(rank, world, port, gp, pp, pop, k, out_dir):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", TBLUP_DIST_BACKEND="gloo")
    import random

    import numpy as np
    import torch.distributed as dist

    from tblup_amd import evaluator as E
    from tests.helpers import shard_population

    random.seed(7)                       # the reference's split draws (evaluator.py:196-203) on every rank
    np.random.seed(7)
    ev = E.BlupParallelEvaluator(gp, pp, 0.4, device=0)
    n_snps = ev.n_columns
    genomes = shard_population(pop, n_snps, k)
    seen = []
    with ev:                             # creates the gloo group (init_from_env) and the GPU context
        assert dist.is_initialized() and dist.get_world_size() == world
        orig = ev.engine.evaluate

        def spy(g, *a, **kw):
            seen.append(len(g))
            return orig(g, *a, **kw)
        ev.engine.evaluate = spy
        fit = ev._fitness(genomes, ev.training_indices, ev.validation_indices)
        testing = ev._fitness(genomes[: 2 * world + 1], np.concatenate((ev.training_indices, ev.validation_indices)),
                              ev.testing_indices)
    np.save(os.path.join(out_dir, f"fit{rank}.npy"), np.asarray(fit))
    np.save(os.path.join(out_dir, f"test{rank}.npy"), np.asarray(testing))
    json.dump({"seen": seen, "group_after": dist.is_initialized(),
               "T": [int(x) for x in ev.training_indices], "V": [int(x) for x in ev.validation_indices]},
              open(os.path.join(out_dir, f"rank{rank}.json"), "w"))
