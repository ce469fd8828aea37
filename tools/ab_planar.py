"""A/B of the autograd path's dsh layout at config C on one GPU: coefficient planes
(the default) vs upstream's rows (the library call patched to ignore dsh_planar),
alternating blocks of steps so clock drift hits both alike.  Prints one JSON line.
usage: python tools/ab_planar.py [--steps K] [--rounds R]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "3dgs_study_amd"), str(ROOT)]

import torch  # noqa: E402

import synthetic  # noqa: E402
import train_step  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = synthetic.CONFIGS["C"]
    cam = synthetic.make_camera(cfg["W"], cfg["H"], view=0).to(dev)
    g = synthetic.make_gaussians(cfg["P"], cfg["sh_degree"], seed=0).to(dev, requires_grad=True)
    target = synthetic.make_target(cfg["W"], cfg["H"], seed=1).to(dev)
    bg = torch.zeros(3, device=dev)
    params = g.params()
    native = _C.rasterize_gaussians_backward

    def rows(*a, dsh_planar=False, **kw):
        return native(*a, **kw)

    res = {"planes": [], "rows": []}
    for _ in range(args.rounds):
        for mode in ("planes", "rows"):
            _C.rasterize_gaussians_backward = native if mode == "planes" else rows
            for i in range(args.steps + 5):
                if i == 5:
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                for p in params:
                    p.grad = None
                train_step.train_step(cam, g, target, bg)
            torch.cuda.synchronize()
            res[mode].append(round(1e3 * (time.perf_counter() - t0) / args.steps, 4))
    _C.rasterize_gaussians_backward = native
    print(json.dumps({"config": "C", "ms_per_step": res,
                      "best": {k: min(v) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
