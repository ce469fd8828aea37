"""Where the host's time per step goes (cProfile over the bench's unit at a config):
the Python / ctypes path of render -> L1 -> backward, sorted by own time.  The
profiler inflates every call; read it for proportions.
usage (on the box): python tools/host_profile.py [--config B] [--steps 200]"""
import argparse
import cProfile
import pstats
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "3dgs_study_amd"), str(ROOT)]

import torch  # noqa: E402

import synthetic  # noqa: E402
import train_step  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="B")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--top", type=int, default=35)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = synthetic.CONFIGS[args.config]
    cam = synthetic.make_camera(cfg["W"], cfg["H"], view=0).to(dev)
    g = synthetic.make_gaussians(cfg["P"], cfg["sh_degree"], seed=0).to(dev, requires_grad=True)
    target = synthetic.make_target(cfg["W"], cfg["H"], seed=1).to(dev)
    bg = torch.zeros(3, device=dev)
    params = g.params()

    def step():
        for p in params:
            p.grad = None
        train_step.train_step(cam, g, target, bg, glue="fused")

    for _ in range(60):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    print(f"unprofiled: {1e3 * (time.perf_counter() - t0) / args.steps:.4f} ms/step", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(args.top)


if __name__ == "__main__":
    main()
