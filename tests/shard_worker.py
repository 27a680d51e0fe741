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


def run_main_gpu(rank, world, port, case, out_dir):
    """main.py (tests/ga_driver.py) on a tests/golden/main_runs.npz case with the GPU drop-ins --
    HIP evaluator, GPU DE evolver, speculative evaluation of the children -- as one of `world`
    torchrun-style ranks on GPU 0 (gloo): the children's shard of this rank is evaluated on the
    device while their genomes cross to the host, and evaluate() all-gathers the shards."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    # LOCAL_WORLD_SIZE: the ranks share one node, so the children's rows go through the node-shared
    # ring (tblup_amd/shmrows.py: each rank copies its shard, page-locked /dev/shm segments)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", LOCAL_WORLD_SIZE=str(world), TBLUP_DIST_BACKEND="gloo")
    import numpy as np

    from tblup_amd import evaluator as E
    from tblup_amd import evolver as EV
    from tblup_amd import local as LS
    from tests import ga_driver as D

    z = np.load(os.path.join(root, "tests", "golden", "main_runs.npz"))
    gp, pp = os.path.join(out_dir, "geno.npy"), os.path.join(out_dir, "pheno.npy")
    taken = []

    def get_evaluator(args):
        ev = E.get_evaluator(args)
        orig = ev._take_spec

        def spy(*a, **k):
            r = orig(*a, **k)
            taken.append(r is not None)
            return r
        ev._take_spec = spy
        return ev

    argv = list(z["base_argv"]) + ["--geno", gp, "--pheno", pp] + list(z[case + "_argv"])
    from tblup_amd.shmrows import RING
    acquired = []
    orig_acq = RING.acquire

    def acq(*a, **k):
        blk = orig_acq(*a, **k)
        acquired.append(blk is not None)
        return blk
    RING.acquire = acq
    run = D.run_main(argv, get_evaluator, EV.get_evolver, LS.get_local_search)
    D.compare(run, z, case)
    json.dump({"taken": taken, "shared": acquired}, open(os.path.join(out_dir, f"main_gpu_rank{rank}.json"), "w"))
