"""Summarise a rocprofv3 --pmc pass of SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE into the MFMA
utilisation of each kernel class (tools/pmc_mfma.sh collects it).

Units (MI355X_MICROARCH.md): SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-busy SIMD cycles summed over
the 1024 SIMDs; GRBM_GUI_ACTIVE is the dispatch's cycles summed over the 8 XCDs.  So
    mfma_busy = MFMA_BUSY / (1024 * GRBM_GUI_ACTIVE / 8)
is the fraction of SIMD cycles with an MFMA in flight, and GRBM_GUI_ACTIVE / 8 / wall the
effective clock the chip held.

    python tools/pmc_mfma.py gpurun_out/pmc_mfma/pmc_counter_collection.csv --out profiles/pmc_mfma.json
"""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import CLASSES  # noqa: E402

SIMDS, XCDS = 1024, 8
LONG_S = 0.2e-3   # mean dispatch length from which the GRBM quotient is trusted as the clock ...
MAX_CLK = 2.4e9   # ... when it is physically possible (MI355X peak engine clock)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--config", default="config2")
    ap.add_argument("--pop", type=int, default=256, help="per-GPU population the profiled bench ran")
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    per = defaultdict(lambda: defaultdict(dict))   # class -> dispatch -> counter -> value
    wall = defaultdict(dict)
    with open(args.csv) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            for key, cls in CLASSES.items():
                if "::" + key + "(" in name or "::" + key + "<" in name:
                    d = row["Dispatch_Id"]
                    per[cls][d][row["Counter_Name"]] = float(row["Counter_Value"])
                    wall[cls][d] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
    # GRBM_GUI_ACTIVE / 8 / wall is the clock the chip held only for dispatches of >= ~0.3 ms (the
    # guide: the quotient reads high on shorter ones -- 2.5-3.9 GHz here, above the 2.4 GHz maximum).
    # Those classes are normalised by their wall time at the reference clock of the long ones.
    raw = {}
    for cls, disp in per.items():
        busy = sum(v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for v in disp.values())
        grbm = sum(v.get("GRBM_GUI_ACTIVE", 0.0) for v in disp.values())
        secs = sum(wall[cls].values())
        if grbm > 0 and secs > 0:
            raw[cls] = (busy, grbm, secs, len(disp))
    long_ = {c: r for c, r in raw.items() if r[2] / r[3] >= LONG_S and r[1] / XCDS / r[2] <= MAX_CLK}
    ref = (sum(r[1] for r in long_.values()) / XCDS / sum(r[2] for r in long_.values())) if long_ else None
    out = {}
    for cls, (busy, grbm, secs, nd) in raw.items():
        clk = grbm / XCDS / secs
        if cls in long_ or ref is None:
            out[cls] = {"mfma_busy": round(busy / (SIMDS * grbm / XCDS), 4), "clock_ghz": round(clk / 1e9, 3),
                        "normalised_by": "GRBM_GUI_ACTIVE", "dispatches": nd}
        else:
            out[cls] = {"mfma_busy": round(busy / (SIMDS * secs * ref), 4), "clock_ghz": None,
                        "grbm_quotient_ghz": round(clk / 1e9, 3),
                        "normalised_by": "wall time x the long dispatches' clock %.3f GHz" % (ref / 1e9),
                        "dispatches": nd}
    json.dump({"config": args.config, "pop_per_gpu": args.pop, "source": args.csv,
               "note": "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x the dispatch's cycles): cycles = "
                       "GRBM_GUI_ACTIVE / 8 XCDs for dispatches >= 0.2 ms whose quotient is <= 2.4 GHz, else wall time x the clock those held",
               "per_class": out}, open(args.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
