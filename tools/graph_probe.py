"""Eager vs captured (train_step.CapturedUnit) rates of the fused training unit,
alternating rounds per config.

    python tools/graph_probe.py [--configs B C] [--steps 200] [--rounds 2]
"""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "3dgs_study_amd"), str(ROOT)]

import torch  # noqa: E402

import synthetic  # noqa: E402
import train_step  # noqa: E402


def rate(fn, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return steps / (time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["B", "C"])
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--graph-only", action="store_true", help="replays only (for a kernel trace)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for name in args.configs:
        c = synthetic.CONFIGS[name]
        cam = synthetic.make_camera(c["W"], c["H"], view=0).to(dev)
        g = synthetic.make_gaussians(c["P"], c["sh_degree"], seed=0).to(dev, requires_grad=True)
        target = synthetic.make_target(c["W"], c["H"], seed=1).to(dev)
        bg = torch.zeros(3, device=dev)
        params = g.params()

        def eager():
            for p in params:
                p.grad = None
            train_step.train_step(cam, g, target, bg, glue="fused")

        for _ in range(20):
            eager()
        unit = train_step.CapturedUnit(cam, g, target, bg)
        if args.graph_only:
            for r in range(args.rounds):
                print(f"{name} graph {rate(unit.replay, args.steps):.1f} it/s", flush=True)
            continue
        for r in range(args.rounds):
            e = rate(eager, args.steps)
            gr = rate(unit.replay, args.steps)
            n = unit.check()
            print(f"{name} round {r}: eager {e:.1f} it/s, graph {gr:.1f} it/s (x{gr / e:.3f}; num_rendered {n}, "
                  f"capacity {unit.capacities[-1]})", flush=True)
        del unit


if __name__ == "__main__":
    main()
