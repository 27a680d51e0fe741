"""Knockout local search (local.py:50-76) at config 2 on one GPU, and the setup cost of the
eigendecomposition / Schur-complement downdate route it could be replaced by.

The walk starts from the best of a pop-256 population (bench.py's synthetic workload) and runs
`tblup_amd.local.knockout_walk` with decision-tree speculation (the default) and with linear
windows of 64 / 256 candidates (the decisions are identical for every mode).  Printed as one JSON line:
  * per window: wall ms of the whole walk, batches, accepted knock-outs;
  * one B = 1 evaluation (the sequential walk's per-candidate cost: k of them);
  * the downdate route's fixed costs for ONE base system (k x k, fp64): the eigendecomposition
    G = Q L Q^T (numpy LAPACK on the host's threads, and torch.linalg.eigh on the GPU) -- paid
    again whenever the removed set grows past what a Schur-complement correction handles."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from tblup_amd.engine import GpuBlupEngine
    from tblup_amd.local import knockout_walk
    cfg = bench.CONFIGS["config2"]
    geno, pheno, T, V, genomes, _ = bench.make_workload(cfg, 1234, 0, 256)
    h2 = 0.4
    out = {"config": "config2", "k": int(genomes.shape[1])}
    with GpuBlupEngine(geno, pheno, device=0) as eng:
        fit = eng.evaluate(list(genomes), T, V, h2)
        b = int(np.argmax(fit))
        best, best_fit = genomes[b], float(fit[b])
        for _ in range(3):
            eng.evaluate([best], T, V, h2)
        ts = []
        for _ in range(10):
            t0 = time.perf_counter()
            eng.evaluate([best], T, V, h2)
            ts.append(time.perf_counter() - t0)
        out["one_eval_b1_ms"] = round(float(np.median(ts)) * 1e3, 3)
        out["sequential_walk_est_ms"] = round(out["one_eval_b1_ms"] * len(best), 1)
        ref = None
        for name, w, tree in (("tree_w256", 256, True), ("linear_w64", 64, False), ("linear_w256", 256, False)):
            sizes = []

            def batch(s):
                sizes.append(len(s))
                return eng.evaluate(s, T, V, h2)
            t0 = time.perf_counter()
            mask, bf, nb = knockout_walk(best, best_fit, batch, w, tree=tree)
            dt = time.perf_counter() - t0
            if ref is None:
                ref = (mask, bf)
            assert np.array_equal(mask, ref[0]) and bf == ref[1]
            out[f"walk_{name}"] = {"ms": round(dt * 1e3, 1), "batches": nb, "accepted": int((~mask).sum()),
                                   "mean_batch": round(float(np.mean(sizes)), 1)}
        out["fitness_before_after"] = [best_fit, float(ref[1])]
    # downdate route: one eigendecomposition of the k x k system (SNP form, train-centred)
    Xc = geno[np.ix_(T, best)].astype(np.float64)
    Xc -= Xc.mean(axis=0)
    G = Xc.T @ Xc
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        np.linalg.eigh(G)
        ts.append(time.perf_counter() - t0)
    out["eigh_host_ms"] = round(min(ts) * 1e3, 1)
    out["host_threads"] = os.cpu_count()
    Gd = torch.from_numpy(G).cuda()
    torch.linalg.eigh(Gd)
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        torch.linalg.eigh(Gd)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    out["eigh_gpu_torch_ms"] = round(min(ts) * 1e3, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
