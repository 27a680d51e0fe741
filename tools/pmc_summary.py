"""Per-kernel means (per dispatch) of every counter in rocprofv3 --pmc CSVs.

    python tools/pmc_summary.py OUT.json a/pmc_counter_collection.csv [b/...csv ...]
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import CLASSES  # noqa: E402


def main():
    out_path, paths = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))   # class -> counter -> dispatch -> value
    wall = defaultdict(dict)
    for p in paths:
        with open(p) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                for cls in CLASSES:
                    if "::" + cls + "(" in name or "::" + cls + "<" in name:
                        d = (p, row["Dispatch_Id"])
                        acc[cls][row["Counter_Name"]][d] += float(row["Counter_Value"])
                        wall[cls][d] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
    res = {}
    for cls, ctrs in acc.items():
        res[cls] = {c: round(sum(v.values()) / len(v), 2) for c, v in sorted(ctrs.items())}
        ws = list(wall[cls].values())
        res[cls]["wall_us_mean"] = round(1e6 * sum(ws) / len(ws), 2)
    json.dump({"sources": paths, "per_dispatch_mean": res}, open(out_path, "w"), indent=1)
    for cls, v in res.items():
        print(cls, v)


if __name__ == "__main__":
    main()
