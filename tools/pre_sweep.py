"""Stage times of the headline unit (config C's camera and image) across Gaussian
counts around the wave-round boundaries of the per-Gaussian kernels: a launch of
P / 64 waves fills ceil(P / 64 / slots) rounds of resident waves, so a time that
jumps just past a round boundary (and not in proportion to P) is a wave-quantization
tail.  usage (on the box): python tools/pre_sweep.py [--steps 60] [P ...]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3dgs_study_amd"), ROOT]

import torch  # noqa: E402

import synthetic  # noqa: E402
import train_step  # noqa: E402
from bench import stage_split  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("P", type=int, nargs="*",
                    default=[655_360, 819_200, 950_000, 983_040, 990_000, 1_000_000, 1_048_576, 1_100_000,
                             1_228_800, 1_250_000])
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    W, H = 1920, 1080
    cam = synthetic.make_camera(W, H, view=0).to(dev)
    target = synthetic.make_target(W, H, seed=1).to(dev)
    bg = torch.zeros(3, device=dev)
    for P in args.P:
        g = synthetic.make_gaussians(P, 3, seed=0).to(dev, requires_grad=True)
        params = g.params()

        def step():
            for p in params:
                p.grad = None
            train_step.train_step(cam, g, target, bg, glue="fused")

        for _ in range(10):
            step()
        per, _ = stage_split(step, args.steps)
        us = {k: per[k][0] * 1e3 for k in ("preprocess", "preprocess_bwd", "render_bwd", "depth_sort") if k in per}
        waves = (P + 63) // 64
        print(f"P {P:>9} waves {waves:>6} " + " ".join(f"{k} {v:7.2f} us ({v * 1e3 / P:6.2f} ns/G)"
                                                      for k, v in us.items()), flush=True)
        del g, params
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
