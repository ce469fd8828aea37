"""Per-kernel medians over the last 30 steps of a rocprofv3 kernel trace (a step
starts at each preprocess_fwd launch): python tools/trace_medians.py TRACE.csv"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "preprocess_fwd" in r["Kernel_Name"]]
steps = [(idx[k], idx[k + 1]) for k in range(max(0, len(idx) - 31), len(idx) - 1)]
per, tot, busy = defaultdict(list), [], []
for a, b in steps:
    tot.append((int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3)
    busy.append(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[a:b]) / 1e3)
    for j, r in enumerate(rows[a:b]):
        per[j].append(((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["Kernel_Name"][:64]))
med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
print(sys.argv[1].split("/")[-1], "step median %.1f us, kernel time %.1f us" % (med(tot), med(busy)))
for j in sorted(per):
    print(f"  {med([d for d, _ in per[j]]):7.1f}  {per[j][0][1]}")
