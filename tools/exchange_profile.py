"""Where the view-parallel exchange's per-rank cost goes, on one GPU (config C).

Variants, alternating, each timed over --steps steps:
  plain    — the N = 1 step (fused leaf gradients, no exchange);
  local    — the SH colour exchange forced on without a process group (the record
             is its own gather, no RCCL): the rasterizer-side and rebuild cost;
  rccl     — a one-rank RCCL group with every collective forced on (the bench's
             exchange_1rank): + the bucket all-reduce, the record all-gather.
Per variant: it/s, and the mean host time spent inside the forward's one host sync
(gsr_forward_preprocess): near zero means the step is host-bound.
usage (on the box): python tools/exchange_profile.py [--steps 60] [--rounds 2]"""
import argparse
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3dgs_study_amd"), ROOT]

import diff_gaussian_rasterization as dgr  # noqa: E402
import synthetic  # noqa: E402
import train_step  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402
from multiview import GradAllReduce  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--only", default="plain,local,rccl", help="comma-separated variants to run")
    ap.add_argument("--no-wrap", action="store_true", help="do not time the forward's host sync")
    ap.add_argument("--glue", default="fused", choices=["fused", "reference"])
    ap.add_argument("--rebuild-on-side", type=int, default=None, choices=[0, 1],
                    help="override GradAllReduce.rebuild_on_side (the SH rebuild on the exchange stream)")
    ap.add_argument("--colours-apart", type=int, default=None, choices=[0, 1],
                    help="override GradAllReduce.colours_apart (the colour kernel on the exchange stream)")
    ap.add_argument("--host", action="store_true", help="host-side time of the exchange's calls (perf_counter)")
    ap.add_argument("--pg", default="eager", choices=["eager", "lazy", "none"],
                    help="process group: RCCL with device_id (eager communicator), without (lazy), or none")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    cfg = synthetic.CONFIGS["C"]
    cam = synthetic.make_camera(cfg["W"], cfg["H"], view=0).to(dev)
    g = synthetic.make_gaussians(cfg["P"], cfg["sh_degree"], seed=0).to(dev, requires_grad=True)
    target = synthetic.make_target(cfg["W"], cfg["H"], seed=1).to(dev)
    bg = torch.zeros(3, device=dev)
    params = g.params()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    if args.pg != "none":
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=dev if args.pg == "eager" else None)

    lib = _C.load_library()
    sync = {"t": 0.0, "n": 0}

    def wrapper(orig):
        def wrapped(*a):
            t0 = time.perf_counter()
            r = orig(*a)
            sync["t"] += time.perf_counter() - t0
            sync["n"] += 1
            return r
        return wrapped

    if not args.no_wrap:  # the forward's native call: its one host wait (two-call or one-call form)
        lib.gsr_forward_preprocess = wrapper(lib.gsr_forward_preprocess)
        lib.gsr_forward = wrapper(lib.gsr_forward)
    hostt = {}
    if args.host:  # wrap the calls on the step's host path and sum their wall time
        import multiview

        def wrap(owner, name, label):
            fn = getattr(owner, name)

            def w(*a, **k):
                t0 = time.perf_counter()
                try:
                    return fn(*a, **k)
                finally:
                    hostt[label] = hostt.get(label, 0.0) + time.perf_counter() - t0
            setattr(owner, name, w)
        wrap(dist, "all_reduce", "dist.all_reduce")
        wrap(dist, "all_gather_into_tensor", "dist.all_gather")
        wrap(multiview.GradAllReduce, "_on_backward_end", "cb:_on_backward_end")
        wrap(multiview.GradAllReduce, "_sh_rebuild", "sh_rebuild")
        wrap(multiview.GradAllReduce, "__call__", "reducer()")
        wrap(multiview.GradAllReduce, "push", "push")
        wrap(multiview.GradAllReduce, "leaf_bucket", "leaf_bucket")
        wrap(_C, "rasterize_gaussians_backward", "_C.backward")
        wrap(_C, "_rasterize", "_C._rasterize")
        wrap(train_step, "train_step", "train_step")
        wrap(torch.Tensor, "backward", "loss.backward")
    if args.colours_apart is not None:
        GradAllReduce.colours_apart = bool(args.colours_apart)
    if args.rebuild_on_side is not None:
        GradAllReduce.rebuild_on_side = bool(args.rebuild_on_side)
    res = {}
    for rnd in range(args.rounds):
        for name in args.only.split(","):
            ar = None
            if name == "local":
                ar = GradAllReduce(params, sh=(params[0], params[1], params[2]), sh_force=True, timing=True)
            elif name == "rccl":
                ar = GradAllReduce(params, sh=(params[0], params[1], params[2]), comm_force=True, timing=True)

            def step():
                for p in params:
                    p.grad = None
                train_step.train_step(cam, g, target, bg, glue=args.glue)
                if ar is not None:
                    ar()

            for _ in range(10):
                step()
            torch.cuda.synchronize()
            if ar is not None:
                ar.reset_stats()
            _C.timing_enable(["exchange_wait", "sh_rebuild"])
            sync["t"], sync["n"] = 0.0, 0
            hostt.clear()
            t0 = time.perf_counter()
            host = 0.0
            for _ in range(args.steps):
                h0 = time.perf_counter()
                step()
                host += time.perf_counter() - h0
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            stages = _C.timing_read()
            _C.timing_enable(False)
            if args.host:
                print(name, rnd, "host us/step:", {k: round(1e6 * v / args.steps, 1) for k, v in sorted(hostt.items())},
                      flush=True)
                hostt.clear()
            r = {"it_s": round(args.steps / dt, 1), "ms": round(1e3 * dt / args.steps, 4),
                 "sync_wait_ms": round(1e3 * sync["t"] / max(sync["n"], 1), 4),
                 "plan": list(dgr.last_leaf_plan)}
            if ar is not None:
                n = max(ar.stats()["timed_calls"], 1)
                r.update(wait_ms=round(stages["exchange_wait"][0] / n, 4),
                         rebuild_ms=round(stages["sh_rebuild"][0] / n, 4))
                ar.remove_hooks()
            res.setdefault(name, []).append(r)
            print(name, rnd, r, flush=True)
    if args.pg != "none":
        dist.destroy_process_group()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
