"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes per kernel class.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in KiB;
FETCH_SIZE reports half of the bytes of a wide coalesced streaming read, so it is doubled.

    python tools/pmc_traffic.py FETCH_CSV WRITE_CSV --config config2 --out profiles/pmc_traffic.json
"""
import argparse
import csv
import json
from collections import defaultdict

CLASSES = {"k_indiv_stats": "stats", "k_gather": "gather", "k_grm": "grm", "k_diag_grm": "grm", "k_diag_grm8": "grm",
           "k_sys_tiles": "grm", "k_sys_tiles_st": "grm", "k_sys_diag_counts": "grm",
           "k_chol_diag": "chol_diag", "k_chol_offdiag": "chol_offdiag", "k_solve": "solve",
           "k_de_step": "de_step", "k_decode_topk": "decode", "k_snp_scan": "snp_scan"}


def per_class(path, counter):
    """{class: {kernel: [bytes per launch]}}"""
    acc = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"]
            for key, cls in CLASSES.items():
                if "::" + key + "(" in name or "::" + key + "<" in name:
                    acc[cls][key].append(float(row["Counter_Value"]) * 1024.0)
    return acc


def class_mean(kernels):
    """a class's bytes per launch: the sum over its kernels of each one's mean per launch (the
    system tiles are two kernels per step: k_sys_tiles_st + k_sys_diag_counts)"""
    return sum(sum(v) / len(v) for v in kernels.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--config", default="config2")
    ap.add_argument("--pop", type=int, default=256, help="per-GPU population the profiled bench ran")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch = per_class(a.fetch_csv, "FETCH_SIZE")
    write = per_class(a.write_csv, "WRITE_SIZE")
    out = {"config": a.config, "pop_per_gpu": a.pop, "source": [a.fetch_csv, a.write_csv],
           "note": "bytes per launch = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024, averaged over launches",
           "per_launch_bytes": {}, "per_launch_fetch_bytes": {}, "per_launch_write_bytes": {}, "launches": {}}
    for cls in CLASSES.values():
        if cls not in fetch or cls not in write:
            continue
        f = 2.0 * class_mean(fetch[cls])
        w = class_mean(write[cls])
        out["per_launch_bytes"][cls] = round(f + w)
        out["per_launch_fetch_bytes"][cls] = round(f)
        out["per_launch_write_bytes"][cls] = round(w)
        out["launches"][cls] = max(len(v) for v in fetch[cls].values())
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out["per_launch_bytes"]))


if __name__ == "__main__":
    main()
