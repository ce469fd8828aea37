"""Per-step gaps of the forced one-rank exchange in a rocprofv3 kernel trace (rocpd
.db): render_bwd end -> colours start, colours end -> SH rebuild start, and the
next forward's preprocess start after the later of preprocess_bwd / the rebuild.
usage: python tools/xgaps.py RESULTS.db"""
import sqlite3
import statistics
import sys

rows = sqlite3.connect(sys.argv[1]).execute("select name, start, end from kernels order by start").fetchall()
out = []
for i, (n, a, b) in enumerate(rows):
    if "colors_from_accum" not in n:
        continue
    rb = max((r for r in rows[max(0, i - 6):i] if "render_bwd" in r[0]), key=lambda r: r[1], default=None)
    sh = next((r for r in rows[i + 1:i + 8] if "sh_from_colors" in r[0]), None)
    pb = next((r for r in rows[max(0, i - 4):i + 8] if "preprocess_bwd" in r[0]), None)
    pf = next((r for r in rows[i + 1:i + 12] if "preprocess_fwd" in r[0]), None)
    if not (rb and sh and pb and pf):
        continue
    out.append(((a - rb[2]) / 1e3, (b - a) / 1e3, (sh[1] - b) / 1e3, (sh[2] - sh[1]) / 1e3,
                (pb[2] - pb[1]) / 1e3, (pf[1] - max(sh[2], pb[2])) / 1e3, (pf[1] - rb[2]) / 1e3))
names = ["rbwd->col", "col", "col->sh", "sh", "pbwd", "->pfwd", "rbwd_end->pfwd"]
for k, nm in enumerate(names):
    v = [o[k] for o in out[5:]]
    print(f"{nm:>15} median {statistics.median(v):7.1f} us  min {min(v):7.1f}  max {max(v):7.1f}  (n={len(v)})")
