"""Per-dispatch durations of the last pipeline step from a rocprofv3 kernel trace CSV."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
seq = [(r["Kernel_Name"].split("(")[0].replace("tblup::", ""), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
        int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
seq = [x for x in seq if x[0].startswith("k_")]
# last step = from the last k_indiv_stats on
start = max(i for i, x in enumerate(seq) if x[0] == "k_indiv_stats")
last = seq[start:]
t0 = last[0][2]
tot = {}
for name, d, st, en in last:
    print(f"{name:16s} {d:9.1f} us  start+{(st - t0) / 1e3:9.1f}")
    tot[name] = tot.get(name, 0) + d
print("step span us:", (last[-1][3] - t0) / 1e3)
for k, v in tot.items():
    print(f"  {k:16s} {v:9.1f}")
