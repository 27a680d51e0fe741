"""Worker for tests/test_distributed.py (world_size 2, gloo, CPU)."""
import json
import os
import sys


def run(rank, world, port, gp, pp, keys_path, out_dir):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import random

    import numpy as np
    import torch.distributed as dist

    from tblup_amd import evaluator as E
    from tblup_amd.distributed import shard_range
    from tests.helpers import KeyIndividual, OracleEngine

    dist.init_process_group("gloo", rank=rank, world_size=world)
    random.seed(3)
    np.random.seed(3)
    ev = E.BlupParallelEvaluator(gp, pp, 0.4, snp_remover=E.SNPRemovalHandler(100, 0.0, 0.4, False))
    eng = OracleEngine(np.load(gp), np.load(pp))
    seen = []
    orig = eng.evaluate

    def spy(genomes, *a, **k):
        seen.append(len(genomes))
        return orig(genomes, *a, **k)

    eng.evaluate = spy
    ev.engine = eng
    keys = np.load(keys_path)
    pop = [KeyIndividual(k, 100) for k in keys]
    ev.evaluate(pop, pop, 0)
    testing = ev.evaluate_testing(pop)
    lo, hi = shard_range(len(pop), rank, world)
    json.dump({"fitness": [float(p.fitness) for p in pop], "testing": [float(x) for x in testing],
               "evaluated": seen, "shard": [lo, hi]}, open(os.path.join(out_dir, f"rank{rank}.json"), "w"))
    dist.barrier()
    dist.destroy_process_group()


def run_main_flow(rank, world, port, case, out_dir):
    """main.py-style run (tests/ga_driver.py) of a tests/golden/main_runs.npz case under a
    torchrun-like environment with NO process group created by the caller: the evaluator's
    __enter__ must create it (gloo here), shard every batch and destroy it on exit."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), TBLUP_DIST_BACKEND="gloo")
    import numpy as np
    import torch.distributed as dist

    from tblup_amd import evaluator as E
    from tblup_amd import local as LS
    from tests import ga_driver as D
    from tests.helpers import OracleEngine

    z = np.load(os.path.join(root, "tests", "golden", "main_runs.npz"))
    gp, pp = os.path.join(out_dir, "geno.npy"), os.path.join(out_dir, "pheno.npy")
    seen, inside = [], []

    def get_evaluator(args):
        ev = E.get_evaluator(args)

        def open_engine():
            inside.append(dist.is_initialized())
            eng = OracleEngine(np.load(ev.data_path), np.load(ev.labels_path))
            orig = eng.evaluate

            def spy(genomes, *a, **k):
                seen.append(len(genomes))
                return orig(genomes, *a, **k)
            eng.evaluate = spy
            return eng
        ev._open_engine = open_engine
        return ev

    argv = list(z["base_argv"]) + ["--geno", gp, "--pheno", pp] + list(z[case + "_argv"])
    assert not dist.is_initialized()
    run = D.run_main(argv, get_evaluator, D.OracleEvolver, LS.get_local_search)
    after = dist.is_initialized()
    D.compare(run, z, case)
    json.dump({"seen": seen, "group_inside": inside, "group_after": after},
              open(os.path.join(out_dir, f"main_rank{rank}.json"), "w"))


def run_rank_error(rank, world, port, out_dir):
    """One rank's shard fails (an out-of-bounds index, numpy's IndexError) while the other's
    succeeds: both ranks must raise the same error type instead of rank 0 waiting in the fitness
    all-gather; the status words travel in that all-gather."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import numpy as np
    import torch.distributed as dist

    from tblup_amd import _native
    from tblup_amd.distributed import allgather_fitness
    from tblup_amd.evaluator import _gather_or_raise

    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    full, st = allgather_fitness(np.full(4 - rank, float(rank)), 7, status=(rank, 5 * (1 - rank)))
    out["status_max"] = [int(x) for x in st]
    out["full"] = [float(x) for x in full]

    def shard():
        if rank == 1:
            raise _native.TblupIndexError("tblup_eval_batch", _native.ERR_INDEX, "index 9 is out of bounds")
        return np.ones(4)
    try:
        _gather_or_raise(shard, (4,), 8, None)
        out["raised"] = None
    except _native.TblupIndexError as e:
        out["raised"] = type(e).__name__
    # any other exception on one rank (a torch / ValueError / ctypes failure): the
    # failing rank re-raises its own error, the other raises TblupError, nobody hangs
    def shard_other():
        if rank == 0:
            raise ValueError("genome of the wrong shape")
        return np.ones(4)
    try:
        _gather_or_raise(shard_other, (4,), 8, None)
        out["raised_other"] = None
    except Exception as e:   # noqa: BLE001
        out["raised_other"] = type(e).__name__
    full = _gather_or_raise(lambda: np.full(4, rank + 0.5), (4,), 8, None)   # and a clean call after it
    out["clean"] = [float(x) for x in full]
    json.dump(out, open(os.path.join(out_dir, f"err_rank{rank}.json"), "w"))
    dist.barrier()
    dist.destroy_process_group()


def run_panel_load(rank, world, port, path, out_dir):
    """Node-shared panel start-up (tblup_amd.panel.load_panel): both ranks get
    the int8 panel while their peak RSS grows by far less than the float64 file."""
    import resource
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    import numpy as np
    import torch.distributed as dist

    from tblup_amd.panel import load_panel

    dist.init_process_group("gloo", rank=rank, world_size=world)
    before = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024
    arr = load_panel(path)
    # every row read (as the GPU context's copy reads them), summed in blocks of rows
    checksum = sum(int(arr[i:i + 50].sum(dtype=np.int64)) for i in range(0, arr.shape[0], 50))
    rows = arr.shape[0]
    peak = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024
    shared = not isinstance(arr, np.ndarray) or isinstance(arr, np.memmap)
    json.dump({"grow": peak - before, "dtype": str(arr.dtype), "shape": list(arr.shape), "rows": rows,
               "shared": bool(shared), "checksum": checksum,
               "leftover": sorted(f for f in os.listdir("/dev/shm") if f.startswith("tblup_panel_"))},
              open(os.path.join(out_dir, f"panel_rank{rank}.json"), "w"))
    dist.barrier()
    dist.destroy_process_group()
