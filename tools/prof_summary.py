"""Per-kernel statistics (rocprofv3 --stats layout) from a rocprofv3 kernel-trace database.

usage: python tools/prof_summary.py RUN_DIR_OR_DB OUT.csv [--top N]
Reads the rocpd SQLite database rocprofv3 writes by default, groups the kernel
dispatches by name and writes Name, Calls, TotalDurationNs, AverageNs,
Percentage, MinNs, MaxNs, StdDev (same columns as rocprofv3's kernel_stats.csv);
prints the top kernels."""
import csv
import glob
import math
import sqlite3
import sys
from pathlib import Path

src = Path(sys.argv[1])
db = src if src.suffix == ".db" else Path(sorted(glob.glob(str(src / "**" / "*.db"), recursive=True))[0])
out = Path(sys.argv[2])
top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 25
con = sqlite3.connect(db)
rows = con.execute("select name, end - start from kernels").fetchall()
by = {}
for name, d in rows:
    by.setdefault(name, []).append(float(d))
total = sum(sum(v) for v in by.values())
stats = []
for name, v in by.items():
    n = len(v)
    mean = sum(v) / n
    sd = math.sqrt(sum((x - mean) ** 2 for x in v) / n)
    stats.append((name, n, sum(v), mean, 100.0 * sum(v) / total, min(v), max(v), sd))
stats.sort(key=lambda r: -r[2])
with open(out, "w", newline="") as f:
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for r in stats:
        w.writerow([r[0], r[1], int(r[2]), round(r[3], 1), round(r[4], 2), int(r[5]), int(r[6]), round(r[7], 1)])
# one step's dispatch sequence: the kernels between the last two preprocess launches
if "--step-trace" in sys.argv:
    seq = con.execute("select name, start, end from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(seq) if "preprocess_fwd_kernel" in r[0]]
    if len(marks) >= 3:
        a, b = marks[-3], marks[-2]
        t0 = seq[a][1]
        with open(sys.argv[sys.argv.index("--step-trace") + 1], "w") as f:
            f.write("start_us,dur_us,gap_us,name\n")
            prev = t0
            for name, st, en in seq[a:b]:
                f.write(f"{(st - t0) / 1e3:.1f},{(en - st) / 1e3:.1f},{(st - prev) / 1e3:.1f},{name[:120]}\n")
                prev = en
            f.write(f"{(seq[b][1] - t0) / 1e3:.1f},0,0,<next step>\n")
for r in stats[:top]:
    print(f"{r[2] / 1e6:8.2f} ms {r[1]:5d} {r[3] / 1e3:8.1f} us  {r[0][:90]}")
