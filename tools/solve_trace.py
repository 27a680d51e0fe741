"""Timeline of the chained solve (k_solve_chain) of one config-2 evaluation (TBLUP_WG_TRACE=1):
per block row J (one unit each per individual) the start / wait-done / end spread and the mean
unit time, and the overall span.   usage: python tools/solve_trace.py [--pop N]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["TBLUP_WG_TRACE"] = "1"

import bench  # noqa: E402


def main():
    pop = int(sys.argv[sys.argv.index("--pop") + 1]) if "--pop" in sys.argv else 256
    import torch
    from tblup_amd.engine import GpuBlupEngine, concat_genomes
    geno, pheno, T, V, genomes, _ = bench.make_workload(bench.CONFIGS["config2"], 1234, 0, pop)
    eng = GpuBlupEngine(geno, pheno, device=0)
    sid = eng.split_id(T, V)
    idx, off = concat_genomes(list(genomes))
    d_idx, d_off = torch.from_numpy(idx).cuda(), torch.from_numpy(off).cuda()
    d_fit = torch.empty(pop, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    for _ in range(4):
        eng.evaluate_device(sid, d_idx.data_ptr(), d_off.data_ptr(), off, 0.4, d_fit.data_ptr(), stream_ptr=s.cuda_stream)
    torch.cuda.synchronize()
    rec = eng.wg_trace()
    r = rec[rec["kind"] == 7]
    if not len(r):
        print("no chained-solve records")
        return
    t0 = r["start"].min()
    us = lambda x: (x - t0) * 1e6
    print(f"pop {pop}: {len(r)} units, span {us(r['end'].max()):.1f} us")
    for J in sorted(set(r["J"].tolist()), reverse=True):
        for kind, name in ((7, "U"),):
            m = r[(r["J"] == J) & (r["kind"] == kind)]
            if not len(m):
                continue
            wt = m["start"] + m["wait"]
            print(f"J={J} {name} n={len(m):5d} start {us(m['start'].min()):7.1f}..{us(m['start'].max()):7.1f}  "
                  f"waited {us(wt.min()):7.1f}..{us(wt.max()):7.1f}  end {us(m['end'].min()):7.1f}..{us(m['end'].max()):7.1f}  "
                  f"mean {1e6 * (m['end'] - m['start']).mean():6.1f} us (wait {1e6 * m['wait'].mean():6.1f})")
    fin = r[(r["kind"] == 7) & (r["I"] == 1)]
    print(f"final units: end {us(fin['end'].min()):.1f}..{us(fin['end'].max()):.1f}, mean {1e6 * (fin['end'] - fin['start']).mean():.1f} us")


if __name__ == "__main__":
    main()
