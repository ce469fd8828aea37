"""Where the host's time goes in one fused training unit (render -> L1 -> backward)
at a given config (default B: 100k Gaussians, 800x800, SH3).

Wraps every gsr_* entry point of the loaded libgsr.so with a timer, runs the
bench's step loop, and prints per step: the whole step's host time, the time
inside each library call (kernel launches and, for gsr_forward, the num_rendered
wait — reported apart by gsr_host_wait_us), and the rest (Python, autograd,
tensor allocation).  Optionally a cProfile of the loop (--profile N: the top N
functions by own time).

    python tools/host_probe.py [--config B] [--steps 300] [--profile 25]
"""
import argparse
import collections
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
from diff_gaussian_rasterization import _C  # noqa: E402

SIZES = {"A": (10_000, 256, 256, 0), "B": (100_000, 800, 800, 3), "C": (1_000_000, 1920, 1080, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="B", choices=sorted(SIZES))
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--profile", type=int, default=0)
    args = ap.parse_args()
    P, W, H, deg = SIZES[args.config]
    dev = torch.device("cuda:0")
    cam = synthetic.make_camera(W, H, view=0).to(dev)
    g = synthetic.make_gaussians(P, sh_degree=deg, seed=0).to(dev, requires_grad=True)
    target = synthetic.make_target(W, H, seed=1).to(dev)
    bg = torch.zeros(3, device=dev)
    params = g.params()

    def step():
        for p in params:
            p.grad = None
        train_step.train_step(cam, g, target, bg, glue="fused")

    for _ in range(30):
        step()
    torch.cuda.synchronize()

    lib = _C.load_library()
    spent = collections.Counter()
    calls = collections.Counter()
    for name in dir(lib):
        if not name.startswith("gsr_") or name in ("gsr_last_error", "gsr_host_wait_us"):
            continue
        fn = getattr(lib, name)

        def wrap(fn=fn, name=name):
            def f(*a):
                t = time.perf_counter()
                r = fn(*a)
                spent[name] += time.perf_counter() - t
                calls[name] += 1
                return r
            return f
        setattr(lib, name, wrap())
    # the wrappers' own cost, to subtract
    t = time.perf_counter()
    for _ in range(10000):
        time.perf_counter()
    tick = (time.perf_counter() - t) / 10000

    _C.host_wait_ms(reset=True)
    torch.cuda.synchronize()
    prof = cProfile.Profile() if args.profile else None
    t0 = time.perf_counter()
    host = 0.0
    if prof:
        prof.enable()
    for _ in range(args.steps):
        h0 = time.perf_counter()
        step()
        host += time.perf_counter() - h0
    if prof:
        prof.disable()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n = args.steps
    wait = _C.host_wait_ms() * 1e-3
    lib_total = sum(spent.values()) - 2 * tick * sum(calls.values())
    print(f"config {args.config}: {n} steps, {1e3 * dt / n:.4f} ms/step wall, host {1e3 * host / n:.4f} ms/step "
          f"(wait {1e3 * wait / n:.4f}, in library calls {1e3 * lib_total / n:.4f} incl. the wait, "
          f"outside them {1e3 * (host - lib_total) / n:.4f})")
    for name, s in spent.most_common():
        print(f"  {name:32s} {calls[name] / n:5.1f} calls/step  {1e3 * s / n:.4f} ms/step")
    if prof:
        pstats.Stats(prof).sort_stats("tottime").print_stats(args.profile)


if __name__ == "__main__":
    main()
