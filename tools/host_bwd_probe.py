"""Where the host's time goes in the fused bench step (config C): the forward call,
the loss, and inside loss.backward() the two Python backward bodies (the autograd
engine runs them on its device thread) against the engine's own overhead.

usage (on the box): python tools/host_bwd_probe.py [--steps 200]"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3dgs_study_amd"), ROOT]

import synthetic  # noqa: E402
import train_ops  # noqa: E402
import train_step  # noqa: E402
import diff_gaussian_rasterization as dgr  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402

acc: dict = {}


def add(name, dt):
    acc[name] = acc.get(name, 0.0) + dt


def wrap(cls, name, label):
    fn = getattr(cls, name)

    def w(*a, **k):
        t0 = time.perf_counter()
        r = fn(*a, **k)
        add(label, time.perf_counter() - t0)
        return r
    setattr(cls, name, staticmethod(w))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = synthetic.CONFIGS["C"]
    cam = synthetic.make_camera(cfg["W"], cfg["H"], 0).to(dev)
    g = synthetic.make_gaussians(cfg["P"], cfg["sh_degree"], seed=0).to(dev, requires_grad=True)
    target = synthetic.make_target(cfg["W"], cfg["H"], seed=1).to(dev)
    bg = torch.zeros(3, device=dev)
    wrap(dgr._RasterizeModel, "backward", "raster.backward (py body)")
    wrap(dgr._RasterizeModel, "forward", "raster.forward (py body)")
    wrap(train_ops._L1SSIM, "backward", "l1.backward (py body)")
    wrap(train_ops._L1SSIM, "forward", "l1.forward (py body)")
    native_bw = _C.rasterize_gaussians_backward

    def nb(*a, **k):
        t0 = time.perf_counter()
        r = native_bw(*a, **k)
        add("  _C.rasterize_gaussians_backward", time.perf_counter() - t0)
        return r
    _C.rasterize_gaussians_backward = nb

    def step():
        t0 = time.perf_counter()
        out = train_step.render_fused(cam, g, bg, l1_target=target)  # the bench's fused unit
        t1 = time.perf_counter()
        loss = out["l1"]
        t2 = time.perf_counter()
        loss.backward(train_step._unit_seed(loss))
        t3 = time.perf_counter()
        for p in g.params():
            p.grad = None
        add("render_fused (call)", t1 - t0)
        add("loss (call)", t2 - t1)
        add("loss.backward (call)", t3 - t2)

    for _ in range(20):
        step()
    torch.cuda.synchronize()
    acc.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(f"steps {args.steps}: {1e6 * wall / args.steps:.1f} us/step wall")
    for k, v in acc.items():
        print(f"{k:40s} {1e6 * v / args.steps:8.1f} us/step")


if __name__ == "__main__":
    main()
