"""Gaps between gap_probe's kernel pairs (tools/gap_probe.hip) from a rocprofv3
kernel-trace database: per (variant, size) the median A duration and the median
gap from A's end to the tiny kernel's start.  usage: gap_summary.py RUN_DIR REPS"""
import glob
import sqlite3
import statistics
import sys

db = sorted(glob.glob(sys.argv[1] + "/**/*.db", recursive=True))[0]
reps = int(sys.argv[2])
rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
pairs = [(rows[i], rows[i + 1]) for i in range(0, len(rows) - 1, 2)]
sizes = (1, 8, 32, 64, 256)
for v, name in enumerate(("plain stores", "nontemporal stores", "atomics (1 per 64-B row)")):
    for k, mb in enumerate(sizes):
        sel = pairs[(v * len(sizes) + k) * reps:(v * len(sizes) + k + 1) * reps][2:]
        dur = statistics.median((a[2] - a[1]) / 1e3 for a, _ in sel)
        gap = statistics.median((b[1] - a[2]) / 1e3 for a, b in sel)
        print(f"{name:26s} {mb:4d} MB  A {dur:8.1f} us  gap {gap:6.2f} us")
