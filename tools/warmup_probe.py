"""How many steps does the headline unit need to reach its steady rate in a fresh
process?  Times each of the first N steps of config C (render -> L1 -> backward,
the bench's fused glue) with HIP events on the compute stream, and prints the
per-step device times in groups.
usage: python tools/warmup_probe.py [--steps N]"""
import argparse
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
    ap.add_argument("--steps", type=int, default=120)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cam = synthetic.make_camera(1920, 1080, view=0).to(dev)
    target = synthetic.make_target(1920, 1080).to(dev)
    bg = torch.zeros(3, device=dev)
    g = synthetic.make_gaussians(1_000_000, 3, seed=0).to(dev, requires_grad=True)
    params = g.params()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    host = []
    torch.cuda.synchronize()
    ev[0].record()
    for k in range(args.steps):
        h0 = time.perf_counter()
        for p in params:
            p.grad = None
        train_step.train_step(cam, g, target, bg, glue="fused")
        ev[k + 1].record()
        host.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    ms = [ev[k].elapsed_time(ev[k + 1]) for k in range(args.steps)]
    for a in range(0, args.steps, 10):
        seg = ms[a:a + 10]
        print(f"steps {a:3d}-{a + len(seg) - 1:3d}: device {sum(seg) / len(seg):.4f} ms/step, "
              f"host {1e3 * sum(host[a:a + 10]) / len(seg):.4f} ms/step, first {seg[0]:.3f}", flush=True)


if __name__ == "__main__":
    main()
