"""Probe: one config-2 evaluation step (18 dependent launches on one stream) replayed as a
captured hipGraph vs launched directly.  Prints ms per step for both and checks the
fitness vectors are identical.   usage: python tools/graph_probe.py [steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import bench
from tblup_amd.engine import GpuBlupEngine, concat_genomes


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    cfg = bench.CONFIGS["config2"]
    n, P, k, pop, nT, nV = cfg
    geno, pheno, T, V, genomes, _ = bench.make_workload(cfg, 0, 0, pop, 1)
    torch.cuda.set_device(0)
    eng = GpuBlupEngine(geno, pheno, device=0)
    sid = eng.split_id(T, V)
    idx, off = concat_genomes(list(genomes))
    d_idx = torch.from_numpy(idx).cuda()
    d_off = torch.from_numpy(off).cuda()
    d_fit = torch.empty(pop, dtype=torch.float64, device="cuda")
    s = torch.cuda.Stream()

    def step():
        eng.evaluate_device(sid, d_idx.data_ptr(), d_off.data_ptr(), off, 0.4, d_fit.data_ptr(),
                            stream_ptr=s.cuda_stream)

    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.synchronize()
    ref = d_fit.cpu().numpy().copy()

    def direct():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        step()
    torch.cuda.synchronize()
    d_fit.zero_()
    g.replay()
    torch.cuda.synchronize()
    same = bool(np.array_equal(d_fit.cpu().numpy(), ref))

    def replay():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            g.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    res = {"direct_ms": [], "graph_ms": [], "lib_graph_ms": []}
    for _ in range(3):
        res["direct_ms"].append(round(direct(), 4))
        res["graph_ms"].append(round(replay(), 4))
        if hasattr(eng, "set_graph"):
            eng.set_graph(True)
            res["lib_graph_ms"].append(round(direct(), 4))
            eng.set_graph(False)
    res["identical_fitness"] = same
    if hasattr(eng, "set_graph"):
        eng.set_graph(True)
        d_fit.zero_()
        step()
        torch.cuda.synchronize()
        res["lib_graph_identical"] = bool(np.array_equal(d_fit.cpu().numpy(), ref))
        res["lib_graph_stats"] = eng.graph_stats()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
