"""Cost of the SH rebuild (`sh_from_colors_kernel`) against the number of views.

With N ranks every rank rebuilds f_dc.grad / f_rest.grad from the N gathered
colour records (multiview.py): it reads 12 B per Gaussian per view
plus the means and writes the 192-B SH gradient row once.  This times
`gsr_sh_grad_from_colors` on synthetic records (config C: P = 1M, SH3) for
N = 1..16 views with HIP events, on one GPU, and prints one JSON line with the
per-N time and the algorithmic bandwidth.
usage: python tools/sh_exchange_cost.py [--reps K]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "3dgs_study_amd"), str(ROOT)]

import torch  # noqa: E402

from diff_gaussian_rasterization import _C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--P", type=int, default=1_000_000)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    P, M = args.P, 16
    gen = torch.Generator(device="cpu").manual_seed(0)
    means = (torch.rand(P, 3, generator=gen) * 4 - 2).to(dev)
    F = _C.sh_record_floats(P)
    dc = torch.empty(P, 1, 3, device=dev)
    rest = torch.empty(P, M - 1, 3, device=dev)
    out = {}
    for n in (1, 2, 4, 8, 16):
        rec = torch.zeros(n, F, device=dev)
        for v in range(n):  # camera on a circle of radius 6 (the config D views), degree 3
            ang = torch.tensor(v * 2 * torch.pi / max(n, 8))
            rec[v, 0:3] = torch.stack([6 * torch.sin(ang), torch.tensor(0.0), 6 * torch.cos(ang)]).to(dev)
            rec[v, 3] = 3.0
            rec[v, 4:4 + 3 * P] = torch.randn(3 * P, generator=gen).to(dev) * 1e-3
        for _ in range(5):
            _C.sh_grad_from_colors(means, rec, n, dc, rest)
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(args.reps):
            _C.sh_grad_from_colors(means, rec, n, dc, rest)
        e1.record(s)
        torch.cuda.synchronize()
        us = 1e3 * e0.elapsed_time(e1) / args.reps
        nbytes = P * (12 + 12 * n + 4 * M * 3)  # means + n dRGB rows + the dsh row
        out[n] = {"us": round(us, 2), "GB_per_s": round(nbytes / us / 1e3, 1), "algorithmic_MB": round(nbytes / 1e6, 1)}
        print(n, out[n], flush=True)
    print(json.dumps({"kernel": "sh_from_colors_kernel", "P": P, "M": M, "views": out}), flush=True)


if __name__ == "__main__":
    main()
