"""Host-side timeline of the bench step (config C by default): how long the Python
thread spends in each part of render -> L1 -> backward, and how long it waits in
the forward's one host sync.  If the sync wait is ~0 the step is host-bound.

usage (on the box): python tools/host_timeline.py [--steps 30] [--config C]"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3dgs_study_amd"))

import synthetic  # noqa: E402
import train_step  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=30)
ap.add_argument("--config", default="C")
args = ap.parse_args()

dev = torch.device("cuda", 0)
cfg = synthetic.CONFIGS[args.config]
cam = synthetic.make_camera(cfg["W"], cfg["H"], 0).to(dev)
g = synthetic.make_gaussians(cfg["P"], cfg["sh_degree"], seed=0).to(dev, requires_grad=True)
target = synthetic.make_target(cfg["W"], cfg["H"], seed=1).to(dev)
bg = torch.zeros(3, device=dev)
params = g.params()
lib = _C.load_library()

acc = {}


def tick(name, t0):
    t = time.perf_counter()
    acc[name] = acc.get(name, 0.0) + (t - t0)
    return t


orig_pre, orig_render, orig_bwd = lib.gsr_forward_preprocess, lib.gsr_forward_render, lib.gsr_backward
orig_leaves = lib.gsr_backward_leaves


class Wrap:
    def __init__(self, f, name):
        self.f, self.name = f, name

    def __call__(self, *a, **kw):
        t0 = time.perf_counter()
        r = self.f(*a, **kw)
        tick(self.name, t0)
        return r


lib.gsr_forward_preprocess = Wrap(orig_pre, "  ctypes gsr_forward_preprocess (incl. sync)")
lib.gsr_forward_render = Wrap(orig_render, "  ctypes gsr_forward_render")
lib.gsr_backward = Wrap(orig_bwd, "  ctypes gsr_backward")
lib.gsr_backward_leaves = Wrap(orig_leaves, "  ctypes gsr_backward_leaves")
import diff_gaussian_rasterization as dgr  # noqa: E402

dgr._leaf_plan = Wrap(dgr._leaf_plan, " _leaf_plan")
dgr._leaf_outputs = Wrap(dgr._leaf_outputs, " _leaf_outputs")
_C._inputs = Wrap(_C._inputs, "  _C._inputs")
orig_rg, orig_rgb = _C.rasterize_gaussians, _C.rasterize_gaussians_backward
_C.rasterize_gaussians = Wrap(orig_rg, " _C.rasterize_gaussians")
_C.rasterize_gaussians_backward = Wrap(orig_rgb, " _C.rasterize_gaussians_backward")

for it in range(10 + args.steps):
    if it == 10:
        torch.cuda.synchronize()
        acc.clear()
        T0 = time.perf_counter()
    t = time.perf_counter()
    for p in params:
        p.grad = None
    out = train_step.render(cam, g, bg)
    t = tick("render()", t)
    loss = train_step.l1_loss(out["render"], target)
    t = tick("l1_loss", t)
    loss.backward()
    t = tick("loss.backward()", t)
torch.cuda.synchronize()
T1 = time.perf_counter()
n = args.steps
print(f"wall per step {1e3 * (T1 - T0) / n:.3f} ms")
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
    print(f"{1e3 * v / n:8.3f} ms  {k}")
