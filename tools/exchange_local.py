"""Local (one-GPU) cost of the view-parallel SH colour exchange at config C.

Times render -> L1 -> backward -> GradAllReduce() on one rank with the exchange
forced on (no communication: the one record is its own gather) against the plain
path, so the difference is what the exchange changes on every rank: no dsh
write and no SH cat backward, plus the HIP rebuild kernel.  Prints one JSON line.
usage: python tools/exchange_local.py [--steps K]
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
from multiview import GradAllReduce  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = synthetic.CONFIGS["C"]
    cam = synthetic.make_camera(cfg["W"], cfg["H"], view=0).to(dev)
    g = synthetic.make_gaussians(cfg["P"], cfg["sh_degree"], seed=0).to(dev, requires_grad=True)
    target = synthetic.make_target(cfg["W"], cfg["H"], seed=1).to(dev)
    bg = torch.zeros(3, device=dev)
    params = g.params()
    res = {}
    for name, force in (("plain", False), ("sh_colour_forced", True), ("plain_again", False)):
        ar = GradAllReduce(params, sh=(params[0], params[1], params[2]), sh_force=force)

        def step():
            for p in params:
                p.grad = None
            train_step.train_step(cam, g, target, bg)
            ar()

        for _ in range(10):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        res[name] = round(1e3 * (time.perf_counter() - t0) / args.steps, 4)
        ar.remove_hooks()
    print(json.dumps({"config": "C", "ms_per_step": res}), flush=True)


if __name__ == "__main__":
    main()
