"""Print one step of a rocprofv3 kernel trace (rocpd .db): each dispatch's start
offset, duration, the idle gap before it on the device and its queue, from the
N-th launch of a marker kernel to the next.
usage: python tools/trace_step.py RESULTS.db [--marker render_fwd] [--index 40]"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="render_fwd")
    ap.add_argument("--index", type=int, default=40)
    args = ap.parse_args()
    rows = sqlite3.connect(args.db).execute(
        "select name, start, end, queue_id from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if args.marker in r[0]]
    i0, i1 = idx[args.index], idx[args.index + 1] + 1
    t0, prev = rows[i0][1], None
    for name, a, b, q in rows[i0:i1]:
        gap = (a - prev) / 1e3 if prev is not None else 0.0
        print(f"{(a - t0) / 1e3:8.1f} {(b - a) / 1e3:7.1f} gap {gap:6.1f} q{q} {name[:72]}")
        prev = b if prev is None else max(prev, b)


if __name__ == "__main__":
    main()
