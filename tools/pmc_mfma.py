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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--config", default="config2")
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
    out = {}
    for cls, disp in per.items():
        busy = sum(v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for v in disp.values())
        grbm = sum(v.get("GRBM_GUI_ACTIVE", 0.0) for v in disp.values())
        secs = sum(wall[cls].values())
        if grbm <= 0:
            continue
        out[cls] = {"mfma_busy": round(busy / (SIMDS * grbm / XCDS), 4),
                    "clock_ghz": round(grbm / XCDS / secs / 1e9, 3) if secs > 0 else None,
                    "dispatches": len(disp)}
    json.dump({"config": args.config, "source": args.csv,
               "note": "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)",
               "per_class": out}, open(args.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
