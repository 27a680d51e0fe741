"""End-to-end DE generation time through the drop-in Python classes at BASELINE config 2
(2000 x 50k, k = 1000, pop 256): GPU evolve (tblup_amd.evolver) -> GPU evaluate
(tblup_amd.evaluator, keys decoded in place from the device key store) -> selection,
against the same generation with the host numpy evolve (oracle) and host argsort decode."""
import json
import os
import random
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(n=2000, p=50000, k=1000, pop=256, gens=4):
    # under torch.distributed.run (WORLD_SIZE > 1): one rank per process; more ranks than GPUs share
    # them (gloo: RCCL needs one device per rank), each rank evaluating its shard of the children
    world = int(os.environ.get("WORLD_SIZE", "1"))
    import torch
    if world > 1:
        ndev = max(1, torch.cuda.device_count())
        os.environ["LOCAL_RANK"] = str(int(os.environ.get("LOCAL_RANK", "0")) % ndev)
        if ndev < world:
            os.environ.setdefault("TBLUP_DIST_BACKEND", "gloo")
        torch.cuda.set_device(int(os.environ["LOCAL_RANK"]))
    from oracle import blup_oracle as O
    from oracle import de_oracle as D
    from tests.helpers import Pop
    # the reference's RandomKeyIndividual semantics (deepcopy copies the genome, individual.py:110-118)
    from tests.ga_driver import RandomKeyIndividual
    from tblup_amd.evaluator import BlupParallelEvaluator
    from tblup_amd.evolver import DERandOneEvolver
    rng = np.random.default_rng(0)
    geno = O.synth_geno(rng, n, p)
    pheno = rng.standard_normal(n)
    tmp = tempfile.mkdtemp()
    np.save(os.path.join(tmp, "g.npy"), geno)
    np.save(os.path.join(tmp, "y.npy"), pheno)
    random.seed(0)
    np.random.seed(0)
    ev = BlupParallelEvaluator(os.path.join(tmp, "g.npy"), os.path.join(tmp, "y.npy"), 0.4)
    inds = [RandomKeyIndividual(k, p, genome=rng.uniform(size=p)) for _ in range(pop)]
    evo = DERandOneEvolver(p, 0.8, 0.5, False)
    out = {"n": n, "p": p, "k": k, "pop": pop, "world": world}
    phase = {}
    # time spent in python's cyclic garbage collector, per generation (gc.callbacks)
    import gc
    gc_t = {"start": 0.0, "ms": 0.0, "n2": 0}

    def gc_cb(ph, info):
        if ph == "start":
            gc_t["start"] = time.perf_counter()
        else:
            gc_t["ms"] += 1e3 * (time.perf_counter() - gc_t["start"])
            gc_t["n2"] += info.get("generation", 0) == 2
    gc.callbacks.append(gc_cb)
    seg_all, gc_all = [], []

    def timed(obj, name):
        fn = getattr(obj, name)

        def wrap(*a, **kw):
            t = time.perf_counter()
            r = fn(*a, **kw)
            phase[name] = phase.get(name, 0.0) + time.perf_counter() - t
            return r
        setattr(obj, name, wrap)
    with ev:
        for nm in ("genomes_to_evaluate", "_fitness", "_batch_genomes"):
            timed(ev, nm)
        import tblup_amd.evolver as EVM
        for nm in ("_copy_rows", "_child_dtypes"):
            fn = getattr(EVM, nm)

            def wrap(*a, _fn=fn, _nm=nm, **kw):
                t = time.perf_counter()
                r = _fn(*a, **kw)
                phase[_nm] = phase.get(_nm, 0.0) + time.perf_counter() - t
                return r
            setattr(EVM, nm, wrap)
        timed(evo, "_donors")
        timed(EVM.GpuDEStep.get(0), "step_device")
        timed(ev.engine, "evaluate")
        timed(ev.engine, "decode_randkey_tensor")
        EVM.PROFILE = {}
        popn = Pop(inds, 0)
        popn.evaluator = ev   # as tblup.Population holds it (population.py:28): lets the evolver hand over
        ev.evaluate(popn, popn, 0)
        ts = []
        for g in range(1, gens + 1):
            popn.generation = g
            t0 = time.perf_counter()
            kids = evo.evolve(popn)
            t1 = time.perf_counter()
            ev.evaluate(popn, kids, g)
            t2 = time.perf_counter()
            popn.population = [c if c.fitness > q.fitness else q for q, c in zip(popn.population, kids)]
            ts.append((t1 - t0, t2 - t1, time.perf_counter() - t0))
            seg_all.append({k: round(1e3 * v, 2) for k, v in EVM.PROFILE.items()})
            gc_all.append((round(gc_t["ms"], 2), gc_t["n2"]))
            gc_t["ms"], gc_t["n2"] = 0.0, 0
            if g == gens:
                out["phases_last_gen_ms"] = {k: round(1e3 * v, 2) for k, v in phase.items()}
                out["evolve_segments_last_gen_ms"] = {k: round(1e3 * v, 2) for k, v in EVM.PROFILE.items()}
            phase.clear()
            EVM.PROFILE.clear()
        best = min(ts, key=lambda t: t[2])
        allg = [1e3 * t[2] for t in ts]
        out.update({"gpu_evolve_ms": 1e3 * best[0], "gpu_evaluate_ms": 1e3 * best[1], "gpu_generation_ms": 1e3 * best[2],
                    "gpu_generation_ms_median": float(np.median(allg)),
                    "gpu_generation_ms_mean_all": float(np.mean(allg)),
                    "gpu_generation_ms_mean_after_first": float(np.mean(allg[1:])) if len(allg) > 1 else None,
                    "gpu_generation_ms_all": [round(x, 2) for x in allg],
                    "gc_ms_and_full_collections_all": gc_all,
                    "evolve_segments_all_ms": seg_all})
        if world > 1:
            from tblup_amd.shmrows import RING
            out["shared_rows"] = any(r is not None for r in RING._rings.values())
            out["gpu_generation_ms_max_over_ranks"] = _max_over_ranks(out["gpu_generation_ms_median"])
            if int(os.environ.get("RANK", "0")) == 0:
                print(json.dumps(out))
            return
        # host evolve (numpy restatement of the reference loop) + host decode, same population
        genomes = [x.get_internal_genome() for x in popn.population]
        t0 = time.perf_counter()
        kids = D.de_generation(genomes, [x.fitness for x in popn.population], gens + 1, "de_rand_1", p, 0.8, 0.5,
                               False)
        t1 = time.perf_counter()
        [np.argsort(c)[-k:] for c in kids]
        t2 = time.perf_counter()
        out.update({"host_evolve_ms": 1e3 * (t1 - t0), "host_decode_ms": 1e3 * (t2 - t1)})
    print(json.dumps(out))


def _max_over_ranks(x):
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


if __name__ == "__main__":
    # usage: python tools/generation_bench.py [GENS] [POP]   (torch.distributed.run for N > 1 ranks)
    main(gens=int(sys.argv[1]) if len(sys.argv) > 1 else 4, pop=int(sys.argv[2]) if len(sys.argv) > 2 else 256)
