"""Per-workgroup timeline of one evaluation step (config 2 unless --config) (TBLUP_WG_TRACE=1).

For every Cholesky launch: makespan, workgroups by kind with their mean / max duration,
slot utilisation (sum of workgroup time / (resident slots x makespan); the off-diagonal
kernel fits 2 workgroups per CU, the diagonal 1), the time the first / last workgroup
starts, and the gap to the previous launch.  Writes the raw records to an .npy for later
analysis.   usage: python tools/wg_trace.py [out.npy] [--pop N] [--config configN]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["TBLUP_WG_TRACE"] = "1"

import bench  # noqa: E402

KIND = {1: "diag", 2: "tile", 3: "prep", 4: "kjj", 5: "sys", 6: "part", 9: "dprep", 10: "epart"}   # (7 / 8: chained solve, tools/solve_trace.py)


def main():
    out = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "gpurun_out/wg_trace.npy"
    pop = int(sys.argv[sys.argv.index("--pop") + 1]) if "--pop" in sys.argv else 256
    config = sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "config2"
    import torch
    from tblup_amd.engine import GpuBlupEngine, concat_genomes
    cfg = bench.CONFIGS[config]
    geno, pheno, T, V, genomes, _ = bench.make_workload(cfg, 1234, 0, pop)
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
    raw = eng.wg_trace(raw=True)
    rec = rec[(rec["kind"] <= 6) | (rec["kind"] >= 9)]
    np.save(out, rec)
    np.save(out.replace(".npy", "_raw.npy"), raw)
    props = torch.cuda.get_device_properties(0)
    cus = props.multi_processor_count
    t0 = rec["start"].min()
    prev_end = None
    tot = 0.0
    print(f"{len(rec)} workgroups, {cus} CUs")
    launches = []
    sysm = rec["kind"] == 5
    if sysm.any():
        launches.append((rec[sysm]["start"].min(), -1, False, sysm))
    for J in sorted(set(rec["J"].tolist())):
        for is_diag in (True, False):
            m = (rec["J"] == J) & (np.isin(rec["kind"], (1, 9, 10)) == is_diag) & ~sysm
            if not m.any():
                continue
            launches.append((rec[m]["start"].min(), J, is_diag, m))
    launches.sort(key=lambda x: x[0])
    for st, J, is_diag, m in launches:
        r = rec[m]
        en = r["end"].max()
        span = en - st
        slots = cus * (1 if is_diag else 2)
        util = float(np.sum(r["end"] - r["start"]) / (slots * span))
        gap = 0.0 if prev_end is None else st - prev_end
        prev_end = en
        tot += span
        parts = []
        for k in sorted(set(r["kind"].tolist())):
            rk = r[r["kind"] == k]
            d = (rk["end"] - rk["start"]) * 1e6
            parts.append(f"{KIND[k]} n={len(rk)} mean={d.mean():.1f} max={d.max():.1f} us "
                         f"last-start=+{(rk['start'].max() - st) * 1e6:.1f}")
        first_tile = ""
        if not is_diag:
            nxt = r[(r["kind"] == 2) & (r["I"] == J + 1)]
            if len(nxt):
                first_tile = f" tile(J+1,J) done by +{(nxt['end'].max() - st) * 1e6:.1f}"
        print(f"{'diag' if is_diag else 'off '} J={J}: start +{(st - t0) * 1e6:8.1f} span {span * 1e6:7.1f} us "
              f"gap {gap * 1e6:5.1f} util {util:.2f}{first_tile} | " + "; ".join(parts))
    print(f"sum of launch spans {tot * 1e6:.1f} us, first start to last end {(prev_end - t0) * 1e6:.1f} us")
    # T-unit phases (wave 0's marks, k_chol.hip tile_unit): K / partial in registers, GEMM1 done,
    # X staged (after the barrier that waits for every wave's GEMM1), end (GEMM2, stores, w update)
    rk2 = (raw[:, 2] >> np.uint64(56)).astype(np.int64)
    tiles = raw[rk2 == 2]
    if len(tiles):
        ph = tiles[:, 3] >> np.uint64(16)
        p = np.stack([(ph >> np.uint64(16 * k)) & np.uint64(0xFFFF) for k in range(3)], 1).astype(np.float64) / 100.0
        tot_us = (tiles[:, 1].astype(np.int64) - tiles[:, 0].astype(np.int64)) / 100.0
        tJ = (tiles[:, 3] & np.uint64(0xFFFF)).astype(np.int64)
        print("T-unit phases (us, means over the launch's tiles): K-ready, GEMM1 (wave 0), wait for the waves + X staged, GEMM2 + stores")
        for J in sorted(set(tJ.tolist())):
            m = tJ == J
            k0, g1, xs, en = p[m, 0], p[m, 1], p[m, 2], tot_us[m]
            print(f"  J={J}: n={int(m.sum()):5d}  K {k0.mean():6.1f}  GEMM1 {(g1 - k0).mean():6.1f}  "
                  f"X {(xs - g1).mean():5.1f}  GEMM2+ {(en - xs).mean():5.1f}  total {en.mean():6.1f}")
    # phase stamps of diagonal workgroup 0 (tblup_internal.h DTR_RECS): per wave, 30 slots.  They
    # follow the diagonal launch's own records (B x (1 + D-units beside it) + E-units), so locate them from
    # the last diagonal record of launch J (the units per launch depend on the schedule policy)
    NT = 8
    names = ["start", "pre-barrier", "post-barrier"] + [f"{x}{p}" for p in range(8) for x in ("a", "b", "w")] + [
        "xinv7", "post-xinv7", "dinv", "z", "syrk-issued", "-"] + [f"{x}{t}" for t in range(8) for x in
                                                                   ("stg-ready", "stg-go")] + ["syrk-done"] + [
        "f4-upd-done", "f4-x-init", "f4-steps", "f4-stored", "f4-branch"]
    rkind = (raw[:, 2] >> np.uint64(56)).astype(np.int64)
    rJ = (raw[:, 3] & np.uint64(0xFFFF)).astype(np.int64)
    for J in range(NT):
        diag_rows = np.nonzero(np.isin(rkind, (1, 9, 10)) & (rJ == J))[0]
        if not len(diag_rows):
            continue
        pos = int(diag_rows.max()) + 1
        st = raw[pos:pos + 128].reshape(-1).reshape(8, 64).astype(np.int64)
        if J in (0, 3):
            base = st[0, 0]
            print(f"diag J={J} wg0 phase stamps (us from start), waves 0 / 1 / 4:")
            for k in [0, 30] + list(range(32, 49)) + list(range(1, 30)) + [54, 50, 51, 52, 53]:
                if st[0, k] == 0 and st[1, k] == 0:
                    continue
                vals = " ".join(f"{(st[w, k] - base) / 100.0:7.2f}" if st[w, k] else "      -" for w in (0, 1, 4))
                print(f"  {names[k]:>12s} {vals}")


if __name__ == "__main__":
    main()
