"""Where does the fused full training step's time go?  Runs
train_step.full_train_step (fused) at config C for K steps and prints how each
forward ran (_C.last_forward: one call / regrown / two calls), the capacity and
num_rendered, and the step rate; `--plain` runs the bench unit instead.
usage: python tools/full_step_probe.py [--steps K]"""
import argparse
import collections
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
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--lam", type=float, default=None, help="override lambda_dssim")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cam = synthetic.make_camera(1920, 1080, view=0).to(dev)
    target = synthetic.make_target(1920, 1080).to(dev)
    bg = torch.zeros(3, device=dev)
    g = synthetic.make_gaussians(1_000_000, 3, seed=0).to(dev, requires_grad=True)
    st = train_step.TrainState(g, spatial_lr_scale=6.6, fused=True)
    if args.lam is not None:
        st.opt["lambda_dssim"] = args.lam
    paths = collections.Counter()
    it = 1
    for _ in range(5):
        train_step.full_train_step(it, cam, g, st, target, bg)
        it += 1
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        train_step.full_train_step(it, cam, g, st, target, bg)
        it += 1
        lf = dict(_C.last_forward)
        paths[lf.get("path")] += 1
        if k % 10 == 0:
            print(k, lf, flush=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print({"it_per_s": round(args.steps / dt, 1), "ms": round(1e3 * dt / args.steps, 3), "paths": dict(paths)},
          flush=True)


if __name__ == "__main__":
    main()
