#!/usr/bin/env python3
"""Headline benchmark: differentiable Gaussian rasterizer training iterations on MI355X.

Metric (BASELINE.json): train iters/sec (fwd+bwd) + Mpix/sec at 1080p with 1M
Gaussians, 1/2/4/8 GPUs.  One step = one view per GPU of the reference's training
unit (train.py:98-105): render() through diff_gaussian_rasterization
-> L1 loss against a target -> loss.backward() (all leaf gradients); with N > 1
GPUs the views shard across ranks (view = rank) over replicated Gaussians and the
leaf gradients are summed with one RCCL all-reduce per step (weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints one JSON line.  Besides the contract fields it carries
  * roofline: the dominant stage's algorithmic bytes per launch ÷ its
    average launch time, measured with HIP events on the launch stream inside the
    timed region, against the 8 TB/s HBM peak; `traffic` = PMC-measured HBM bytes
    per launch from profiles/pmc_summary.json when present (else null);
  * cpu_baseline: the CPU oracle (oracle/, C port of the upstream algorithm)
    timed on this host for one full view of the same workload (rank 0, N = 1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "3dgs_study_amd"))
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec

WORKLOADS = {
    "C": "1M Gaussians, 1920x1080, SH deg 3, render->L1->backward, one view per GPU per step",
    "B": "100k Gaussians, 800x800, SH deg 3, render->L1->backward, one view per GPU per step",
    "A": "10k Gaussians, 256x256, SH deg 0, render() forward only (no grad), one view per GPU per step",
    "E": "5M Gaussians, 3840x2160, SH deg 3, render() forward only (no grad), one view per GPU per step",
}
RENDER_METRIC = "render frames/sec (fwd-only) + Mpix/sec, 4K (3840x2160), 5M Gaussians, SH3"


def render_metric(cfg_name: str) -> str:
    """The forward-only metric of a config (E is BASELINE.json's; A is the CPU-plumbing case)."""
    if cfg_name == "E":
        return RENDER_METRIC
    import synthetic
    c = synthetic.CONFIGS[cfg_name]
    return f"render frames/sec (fwd-only) + Mpix/sec, {c['W']}x{c['H']}, {c['P']} Gaussians, SH{c['sh_degree']}"


def algorithmic_bytes(stage: str, P: int, I: int, W: int, H: int, M: int, backward: bool = True,
                      S: int = None) -> float:
    """Bytes a launch of a stage must move at minimum, for the form the library runs
    (SURVEY.md §8d's per-unit figures, with this library's own data flow where it
    differs from upstream's).  backward: the unit has a backward (preprocess then
    also stores the SH direction Jacobian, 9 floats per Gaussian, which
    preprocess_bwd reads instead of the 192-B SH row).  S: the footprint's row spans
    (the row-span binning; None = the LSD sort's upstream-shaped
    figures)."""
    T = ((W + 15) // 16) * ((H + 15) // 16)
    HW = W * H
    jac = 36 if backward and M > 1 else 0
    out = {
        # means/scale/rot/opacity/SH in; depth, means2D, 48-B splat record, clamp bits,
        # tiles_touched, 16-B rect record, radii out (+ the Jacobian)
        "preprocess": P * (44 + 12 * M) + P * (85.0 + jac),
        # preprocess's colour half when it runs apart (gsr_colour_mode 1; the
        # geometry half is then "preprocess" without the SH row, colour words and
        # Jacobian): means 12 + radii 4 + the SH row in, colour 12 + clamp 1 + Jacobian out
        "colour": P * (16 + 12 * M) + P * (13.0 + jac),
        "scan": P * 8.0,
        "depth_sort": P * 16.0,                               # depths + tiles_touched in, order + offsets out
        "duplicate": P * 20.0 + I * 8.0,                      # duplicateWithKeys: per-G read, (tile, id) out
        "tile_sort": I * 16.0 + I * 4.0 + T * 8.0,            # one read + write of 8-B pairs; ranges
        "render_fwd": I * 40.0 + T * 16.0 + HW * 20.0,
        "render_bwd": I * 40.0 + HW * 20.0 + T * 8.0 + P * 44.0,
        # reads: means3D 12, scales 12, rotations 16, opacity 4, radii 4, the accumulator's
        # 9 sums 36, the SH direction Jacobian 36 (or the 12M-B SH row without it), clamp
        # bits 1; writes: dmeans3D 12, dscales 12, drot 16, dopacity 4, dsh 12M
        "preprocess_bwd": P * (85.0 + (36 if jac else 12 * M) + 44 + 12 * M),
    }
    if S is not None:  # the row-span binning
        out["scan"] = P * 36.0                                 # order 4 + rects 16 (gathered) in, 16 out
        out["duplicate"] = P * 20.0 + S * 8.0                  # rank-ordered rects + ids in, spans out
        out["tile_sort"] = S * 12.0 + I * 4.0 + T * 8.0        # span columns (count), spans (scatter); ids, ranges
    return out.get(stage, 0.0)


def stage_model_fracs(per_stage: dict, P: int, I: int, W: int, H: int, M: int, backward: bool = True,
                      S: int = None) -> dict:
    """Each stage's model bytes / its measured mean launch time / peak (a stage whose
    model would need more than the peak has a model that over-credits it: VERDICT r5)."""
    out = {}
    for k, v in per_stage.items():
        ms = v[0] if isinstance(v, tuple) else v
        b = algorithmic_bytes(k, P, I, W, H, M, backward, S)
        if k == "preprocess" and "colour" in per_stage:
            b = P * (44 + 72.0)  # the geometry half alone: the colour half is its own stage
        if ms and b:
            out[k] = round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    return out


def model_over_peak(fracs: dict) -> list:
    """Stages whose model bytes exceed what the measured time allows at peak."""
    return sorted(k for k, f in fracs.items() if f > 1.0)


def iter_bytes(P: int, I: int, W: int, H: int, M: int, backward: bool = True) -> float:
    """SURVEY.md §8(d)'s algorithmic bytes of one unit: forward P(147 + 12M) + I·84 +
    HW·20 + T·16, backward P(283 + 24M) + I·40 + HW·20 + T·8."""
    T = ((W + 15) // 16) * ((H + 15) // 16)
    fwd = P * (147 + 12 * M) + I * 84 + W * H * 20 + T * 16
    bwd = P * (283 + 24 * M) + I * 40 + W * H * 20 + T * 8
    return float(fwd + (bwd if backward else 0))


RASTER_STAGES = ("preprocess", "depth_sort", "scan", "duplicate", "tile_sort", "render_fwd", "bwd_prepare",
                 "render_bwd", "preprocess_bwd")


def raster_ms(per_stage: dict) -> float:
    """The rasterizer's own device time per step: the sum of its stages' mean launch
    times (HIP events on the launch stream; the caller's torch kernels excluded)."""
    return round(sum(per_stage[k][0] if isinstance(per_stage[k], tuple) else per_stage[k]
                     for k in RASTER_STAGES if k in per_stage), 4)


def pmc_stage(stage: str) -> dict:
    """profiles/pmc_summary.json's record of a stage (tools/pmc.sh): HBM bytes per
    launch and the VALU issue utilisation, measured by rocprofv3 --pmc passes."""
    f = ROOT / "profiles" / "pmc_summary.json"
    if not f.exists():
        return {}
    try:
        return json.loads(f.read_text()).get("stages", {}).get(stage, {})
    except (OSError, ValueError):
        return {}


def pmc_traffic(stage: str):
    v = pmc_stage(stage).get("hbm_bytes_per_launch")
    return float(v) if v is not None else None


def pmc_key(cfg_name: str, footprint: str) -> str:
    """The suffix of a workload's PMC records (tools/round_profile.sh runs one pass per
    config and footprint): "<stage>_C_rect", "unit_C_rect", ..."""
    return f"_{cfg_name}_{footprint}"


def pmc_unit_bytes(key: str):
    """profiles/pmc_summary.json's measured HBM bytes of one benchmark unit (every gsr
    kernel's per-dispatch bytes x dispatches per unit; tools/pmc_summary.py), or None."""
    f = ROOT / "profiles" / "pmc_summary.json"
    try:
        v = json.loads(f.read_text()).get("units", {}).get(key, {}).get("hbm_bytes_per_unit")
    except (OSError, ValueError):
        return None
    return float(v) if v is not None else None


def measured_frac(key: str, units_per_s: float):
    """The iteration-level HBM roofline from the PMC-measured bytes per unit (VERDICT r4:
    beside §8(d)'s model figure), or None without a PMC record for this workload."""
    b = pmc_unit_bytes(key)
    return round(b * units_per_s / 1e9 / HBM_PEAK_GBS, 4) if b else None


def num_rendered_seen() -> int:
    """num_rendered of the last forward the binding ran (the benchmarked view, read after
    the warm-up: no extra forward, so PMC runs count whole units)."""
    from diff_gaussian_rasterization import _C

    return int(_C.last_forward.get("num_rendered", 0))


def _host_cpu() -> dict:
    """Core count (`nproc`, which honours the box's CPU share / OMP_NUM_THREADS) and
    the CPU model name (lscpu's "Model name", from /proc/cpuinfo)."""
    import subprocess

    try:
        n = int(subprocess.run(["nproc"], capture_output=True, text=True, check=True).stdout.strip())
    except (OSError, ValueError, subprocess.CalledProcessError):
        n = len(os.sched_getaffinity(0))
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"nproc": n, "model": model}


def cpu_baseline(configs=("A", "B", "C", "E"), repeats: int = 3, cap_s: float = 1800.0) -> dict:
    """SURVEY.md §8(d)'s CPU baseline: the reference's render() shape with
    convert_SHs_python and compute_cov3D_python (gaussian_renderer/__init__.py:74-90:
    SH -> RGB and the 3D covariance in torch, autograd through them), the rasterizer
    forward / backward by the C oracle's OpenMP build (oracle/, a port of the
    upstream algorithm; rasterize -> L1 -> backward for the training configs), on
    all `nproc` host cores.  Median of `repeats` after one warm-up per config."""
    ncpu = _host_cpu()
    os.environ.setdefault("OMP_NUM_THREADS", str(ncpu["nproc"]))
    import math

    import numpy as np
    import torch

    import synthetic
    import train_step
    from oracle import oracle

    oracle.build()
    torch.set_num_threads(ncpu["nproc"])
    threads = oracle.num_threads(mt=True)

    def one(cfg, cam, g, target):
        xyz, opac = g.get_xyz, g.get_opacity
        feats = g.get_features
        shs_view = feats.transpose(1, 2).view(-1, 3, (g.max_sh_degree + 1) ** 2)
        dirs = xyz - cam.camera_center.repeat(feats.shape[0], 1)
        dirs = dirs / dirs.norm(dim=1, keepdim=True)
        colors = torch.clamp_min(train_step.eval_sh(g.active_sh_degree, shs_view, dirs) + 0.5, 0.0)
        cov3D = train_step.covariance(g.get_scaling, 1.0, g.rotation)
        f = oracle.forward(xyz.detach().numpy(), opac.detach().numpy(), cam.world_view_transform.numpy(),
                           cam.full_proj_transform.numpy(), cam.camera_center.numpy(), np.zeros(3, np.float32),
                           cam.image_height, cam.image_width, math.tan(cam.FoVx * 0.5), math.tan(cam.FoVy * 0.5), 1.0,
                           g.active_sh_degree, colors_precomp=colors.detach().numpy(),
                           cov3D_precomp=cov3D.detach().numpy(), mt=True)
        if not cfg["backward"]:
            return
        dL = (np.sign(f["color"] - target) / f["color"].size).astype(np.float32)  # L1 backward
        b = oracle.backward(f, dL)
        torch.autograd.backward([xyz, colors, cov3D, opac],
                                [torch.from_numpy(b[k]) for k in ("dmeans3D", "dcolors", "dcov3D", "dopacity")])

    out = {}
    t_all = time.perf_counter()
    for name in configs:
        cfg = synthetic.CONFIGS[name]
        P, W, H, deg = cfg["P"], cfg["W"], cfg["H"], cfg["sh_degree"]
        cam = synthetic.make_camera(W, H, 0)
        g = synthetic.make_gaussians(P, deg, seed=0).to("cpu", requires_grad=True)
        target = synthetic.make_target(W, H, seed=1).numpy()
        times = []
        t_cfg = time.perf_counter()
        for k in range(repeats + 1):
            if time.perf_counter() - t_cfg > cap_s:
                break
            for p in g.params():
                p.grad = None
            t0 = time.perf_counter()
            one(cfg, cam, g, target)
            if k:  # the first run is the warm-up
                times.append(time.perf_counter() - t0)
        unit = "train-iters/s" if cfg["backward"] else "frames/s"
        if len(times) < repeats:
            out[name] = {"status": "timeout", "cap_s": cap_s, "runs": len(times)}
            continue
        med = sorted(times)[len(times) // 2]
        out[name] = {"value": round(1.0 / med, 4), "unit": unit, "s_per_iter": round(med, 3),
                     "work": "render -> L1 -> backward" if cfg["backward"] else "render (forward)",
                     "gaussians": P, "width": W, "height": H, "sh_degree": deg}
        del g
    head = out.get("C", {})
    return {"value": head.get("value"), "unit": "train-iters/s", "cores": threads, "kind": "port",
            "nproc": ncpu["nproc"], "cpu_model": ncpu["model"], "torch_threads": torch.get_num_threads(),
            "sample": f"config C (the headline workload) through the reference-shaped render() with "
                      f"convert_SHs_python / compute_cov3D_python (torch) and the C oracle's OpenMP build as the "
                      f"rasterizer, forward + L1 + backward on {threads} threads; median of {repeats} after 1 "
                      f"warm-up; the configs table has A, B, E the same way ({time.perf_counter() - t_all:.0f} s)",
            "configs": out}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="C", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--lambda-dssim", type=float, default=0.0,
                    help="0 = L1-only headline unit; 0.2 = the reference's L1+SSIM loss")
    ap.add_argument("--full-steps", type=int, default=20,
                    help="timed iterations of the full train.py step (L1+SSIM, Adam), torch vs fused; 0 = skip")
    ap.add_argument("--grad-exchange", default="sh-colour", choices=["sh-colour", "allreduce"],
                    help="N>1: 'sh-colour' all-gathers per-view colour gradients for the SH block and all-reduces "
                         "the rest (multiview.py); 'allreduce' all-reduces all 59 floats/Gaussian")
    ap.add_argument("--footprint-steps", type=int, default=100,
                    help="timed steps of the same unit with the other tile footprint (gsr.h gsr_footprint); 0 = skip")
    ap.add_argument("--stage-events", default="split", choices=["split", "all", "none"],
                    help="split: the per-stage split (stages_ms, dominant stage) from its own steady-state block of "
                         "the same K steps right before the timed region, whose steps carry events only around the "
                         "dominant stage (its live launch time = the roofline); all: events on every stage inside "
                         "the timed region (they cost ~5%% of the step); none: no events")
    ap.add_argument("--exchange-steps", type=int, default=100,
                    help="N=1: timed steps with the view-parallel exchange forced on in a one-rank RCCL group "
                         "(every collective runs; reported beside the plain step); 0 = skip")
    ap.add_argument("--render-steps", type=int, default=20,
                    help="timed forward-only renders of config E (5M, 4K) reported beside the C line; 0 = skip")
    ap.add_argument("--glue", default="fused", choices=["fused", "reference"],
                    help="the render/loss code around the rasterizer (train_step.py): 'fused' renders from "
                         "GaussianModel's stored parameters (rasterize_model: no SH cat, in-kernel activations) "
                         "with the fused loss kernel; 'reference' is the reference's render() + torch loss")
    ap.add_argument("--glue-steps", type=int, default=100,
                    help="N=1: timed steps of the same unit with the other glue, reported beside; 0 = skip")
    ap.add_argument("--binning", default="rowspan", choices=["rowspan", "lsd"],
                    help="the binning form (gsr_binning_mode): the row-span binning (default) or the LSD sort by "
                         "tile index; the same lists either way")
    ap.add_argument("--graph-steps", type=int, default=1,
                    help="N = 1: also time K replays of the unit captured as a HIP graph (train_step.CapturedUnit); "
                         "0 = off")
    ap.add_argument("--config-b-steps", type=int, default=200,
                    help="N=1: timed steps of config B (100k, 800x800, SH3, fwd+bwd) reported beside; 0 = skip")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import synthetic
    import train_step
    from diff_gaussian_rasterization import _C
    from multiview import GradAllReduce

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}; launch N>1 with torch.distributed.run")
    # GSR_DIST_BACKEND=gloo rehearses the N>1 path with ranks sharing the visible
    # GPUs (a 1-GPU box); the measured configuration is "nccl" (RCCL over xGMI),
    # one rank per GPU
    backend = os.environ.get("GSR_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local_rank %= torch.cuda.device_count()
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)

    _C.set_binning_mode(args.binning)
    if not synthetic.CONFIGS[args.config]["backward"]:
        render_main(args, dev, world, rank)
        return
    cfg = synthetic.CONFIGS[args.config]
    P, W, H, deg = cfg["P"], cfg["W"], cfg["H"], cfg["sh_degree"]
    M = (deg + 1) ** 2
    cam = synthetic.make_camera(W, H, view=rank % 8).to(dev)
    g = synthetic.make_gaussians(P, deg, seed=0).to(dev, requires_grad=True)
    target = synthetic.make_target(W, H, seed=1).to(dev)
    bg = torch.zeros(3, device=dev)
    params = g.params()
    sh = (params[0], params[1], params[2]) if args.grad_exchange == "sh-colour" else None
    # the exchange engages only when world > 1 (timing: its wait / SH rebuild per step)
    reducer = GradAllReduce(params, sh=sh, timing=world > 1)

    def one_step():
        for p in params:
            p.grad = None
        out = train_step.train_step(cam, g, target, bg, lambda_dssim=args.lambda_dssim, glue=args.glue)
        if world > 1:
            reducer()  # wait for the exchange started inside backward (+ rebuild the SH gradients)
        return out

    for _ in range(max(args.warmup, 1)):
        out = one_step()
    torch.cuda.synchronize()
    I = num_rendered_seen()  # the instances of this rank's view (the byte model)
    S = _C.last_spans(W, H)  # its row spans (the row-span binning's byte model), None with the LSD sort
    if world > 1:
        dist.barrier()
    # Stage split (HIP events on the launch stream around every rasterizer stage,
    # gsr_timing_*): a steady-state block of at least SPLIT_MIN_STEPS steps after the
    # warm-up.  Recording 14 events per step costs ~5 % of the step, so the timed
    # region below carries events only around the dominant stage.  In a fresh
    # process the device reaches its steady rate only after ~50 steps of this unit
    # (tools/warmup_probe.py: 0.729 ms/step over steps 10-19, 0.691 over 30-39,
    # 0.676 from 50 on — the clocks ramping under sustained load), so a short
    # warm-up (the driver's --warmup 5) would time the ramp, not the kernels.
    per_stage, dom = {}, "render_bwd"
    if args.stage_events == "split":
        per_stage, dom = stage_split(one_step, max(args.steps, SPLIT_MIN_STEPS))
    # Timed region: K steps; events around the dominant stage give its live
    # average launch time (the roofline).
    on = {"split": [dom], "all": True, "none": False}[args.stage_events]
    if world > 1 and on is not True:
        on = (on or []) + list(EXCHANGE_STAGES)
    _C.timing_enable(on)
    # the dominant stage's events on every DOM_EVERY-th step (each event pair's
    # marker leaves the device idle ~4 us: on every step they cost ~1.3 % at C)
    _C.timing_sample(DOM_EVERY if args.stage_events == "split" else 1)
    torch.cuda.synchronize()
    if world > 1:
        reducer.reset_stats()
        dist.barrier()
    t0 = time.perf_counter()
    host = 0.0
    for _ in range(args.steps):
        h0 = time.perf_counter()
        out = one_step()
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    stages = _C.timing_read()
    _C.timing_enable(False)
    _C.timing_sample(1)
    elapsed = t1 - t0
    exchange = None
    if world > 1:
        ex = reducer.stats()
        wait_ms, rebuild_ms = _exchange_split(stages, ex["timed_calls"])
        t = torch.tensor([elapsed, wait_ms, rebuild_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0].item())
        import diff_gaussian_rasterization as dgr
        # per rank, max over the ranks: how long the compute stream waited for the
        # bucket's all-reduce + the records' all-gather, and the SH rebuild
        exchange = {"exchange_wait_ms": round(float(t[1].item()), 4), "sh_rebuild_ms": round(float(t[2].item()), 4),
                    "bytes_per_rank": ex["bytes_per_rank"], "calls": ex["calls"],
                    "fused_leaves": list(dgr.last_leaf_plan), "stat": "max over ranks of the per-step mean"}
    if args.stage_events == "all":
        per_stage = {k: (ms / n if n else 0.0, n) for k, (ms, n) in stages.items() if n}
        dom = _dominant(per_stage)
    dom_live = stages.get(dom, (0.0, 0))
    # N = 1: the same unit captured once as a HIP graph and replayed (train_step.
    # CapturedUnit): every kernel of the unit runs every step, one graph launch
    # replaces the per-step Python, autograd and ~20 kernel launches; the line
    # reports the faster form, both beside (a slow host makes the eager form
    # host-bound: C 1,250 vs 1,478 it/s on one box, tools/graph_probe.py)
    eager_elapsed, graph_form = elapsed, None
    if world == 1 and args.glue == "fused" and not args.lambda_dssim and args.graph_steps > 0:
        del out
        unit = train_step.CapturedUnit(cam, g, target, bg, warmup=2)
        for _ in range(max(args.warmup, 1)):
            unit.replay()
        torch.cuda.synchronize()
        gt0 = time.perf_counter()  # the same K steps as the eager form
        ghost = 0.0
        for _ in range(args.steps):
            h0 = time.perf_counter()
            out = unit.replay()
            ghost += time.perf_counter() - h0
        torch.cuda.synchronize()
        gdt = time.perf_counter() - gt0
        graph_form = {"value": round(args.steps / gdt, 3), "ms_per_step": round(1e3 * gdt / args.steps, 4),
                      "steps": args.steps, "host_ms_per_step": round(1e3 * ghost / args.steps, 4),
                      "num_rendered": unit.check(), "capacity": unit.capacities[-1]}
        out = None
        del unit
        if graph_form["value"] > args.steps / elapsed:
            elapsed, host = gdt, ghost

    if rank == 0:
        steps = args.steps
        value = world * steps / elapsed
        dom_ms = dom_live[0] / dom_live[1] if dom_live[1] else 0.0
        ab = algorithmic_bytes(dom, P, I, W, H, M, True, S)
        achieved = ab / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
        pkey = pmc_key(args.config, _C.get_footprint())
        traffic = pmc_traffic(dom + pkey) if args.glue == "fused" else None
        fracs = stage_model_fracs(per_stage, P, I, W, H, M, True, S)
        coll = "RCCL" if backend == "nccl" else backend
        line = {
            # BASELINE.json's headline metric at C; the other backward configs name their own shape
            "metric": ("train iters/sec (fwd+bwd) + Mpix/sec, 1080p, 1M Gaussians @1/2/4/8 GPU" if args.config == "C"
                       else f"train iters/sec (fwd+bwd) + Mpix/sec, {W}x{H}, {P} Gaussians, SH{deg}"),
            "value": round(value, 3),
            "unit": "train-iters/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded Gaussians in a radius-2 ball, camera at distance 6, SURVEY.md §8d)",
            "config": {
                "workload": f"{args.config}: {WORKLOADS[args.config]}",
                "gaussians": P, "width": W, "height": H, "sh_degree": deg,
                "footprint": _C.get_footprint(), "binning": _C.get_binning_mode(), "num_rendered": I,
                "views_per_step": world,
                "loss": "L1" if not args.lambda_dssim else f"L1+{args.lambda_dssim}*(1-SSIM)",
                "glue": GLUE_NOTE[args.glue],
                "parallelism": f"view-parallel x{world}" + (
                    (f", {coll} all-gather of per-view colour-gradient records + all-reduce of xyz/opacity/scaling/"
                     f"rotation, {reducer.nbytes / 1e6:.0f} MB sent per rank per step"
                     if reducer.sh_exchange else f", {coll} all-reduce {reducer.nbytes / 1e6:.0f} MB/step")
                    if world > 1 else ""),
                **({"collective_backend": backend} if world > 1 else {}),
            },
            "mpix_per_s": round(value * W * H / 1e6, 2),
            "stages_ms": {k: round(v[0], 4) for k, v in per_stage.items()},
            "stages_source": STAGES_SOURCE[args.stage_events],
            # each stage's byte model (algorithmic_bytes) over its measured time, against 8 TB/s,
            # and any stage whose model would need more than the peak (none expected)
            "stage_hbm_frac": fracs, "model_over_peak": model_over_peak(fracs), "row_spans": S,
            # the rasterizer's own stages per step, and §8(d)'s bytes per unit at the
            # measured I against 8 TB/s (the north_star's iteration-level roofline)
            "raster_ms": raster_ms(per_stage),
            "iter_algorithmic_bytes": iter_bytes(P, I, W, H, M),
            "iter_hbm_frac": round(iter_bytes(P, I, W, H, M) * value / world / 1e9 / HBM_PEAK_GBS, 4),
            # the same with the PMC-measured HBM bytes per unit (profiles/pmc_summary.json,
            # tools/pmc.sh on the default footprint and glue; null for other workloads)
            "iter_hbm_frac_measured": (measured_frac("unit" + pkey, value / world)
                                       if args.glue == "fused" else None),
            # host time inside one_step per step (launches, autograd, the one read-back wait)
            "host_ms_per_step": round(1e3 * host / steps, 4),
            # which form the value is (eager steps, or replays of the captured unit), both beside
            "form": "graph" if elapsed != eager_elapsed else "eager",
            "eager": {"value": round(world * steps / eager_elapsed, 3), "ms_per_step": round(1e3 * eager_elapsed / steps, 4)},
            "graph": graph_form,
            "roofline": {
                "bound": "hbm",
                "kernel": dom,
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": ab,
                "avg_launch_ms": round(dom_ms, 4),
                # the blend loops are issue-bound, not byte-bound: PMC VALU issue share
                "valu_issue_frac": pmc_stage(dom + pkey).get("valu_issue_frac"),
            },
            **({"exchange": exchange} if exchange is not None else {}),
            "cpu_baseline": None,
            # SHA-256 of the sources the loaded libgsr.so was built from (tools/build_id.py)
            "build_id": _C.load_library().gsr_build_id().decode(),
        }
        if world == 1 and args.footprint_steps > 0:
            line["footprint_" + ("tight" if _C.get_footprint() == "rect" else "rect")] = footprint_rates(
                one_step, cam, g, bg, args.footprint_steps, args.warmup)
        if world == 1 and args.glue_steps > 0:
            other = "reference" if args.glue == "fused" else "fused"
            line[f"{other}_glue"] = glue_rates(cam, g, target, bg, other, args.glue_steps, args.warmup,
                                               args.lambda_dssim)
        if world == 1:
            # the unmodified drop-in: the reference's render() (gaussian_renderer/__init__.py:
            # 98-106) and torch L1 over this library, next to the headline (which uses the
            # stored-parameter render + fused L1: INTEGRATION.md's caller edit)
            dr = line if args.glue == "reference" else line.get("reference_glue")
            if dr:
                line["dropin"] = {"value": dr["value"], "unit": "train-iters/s", "ms_per_step": dr["ms_per_step"],
                                  "iter_hbm_frac": round(iter_bytes(P, I, W, H, M) * dr["value"] / 1e9
                                                         / HBM_PEAK_GBS, 4),
                                  "glue": GLUE_NOTE["reference"]}
        if world == 1 and args.config_b_steps > 0 and args.config == "C":
            line["config_B"] = train_config_rates("B", dev, args.config_b_steps, args.warmup, args.glue,
                                                  args.lambda_dssim)
        if world == 1 and args.full_steps > 0:
            line["full_step"] = full_step_rates(cam, P, deg, target, bg, args.full_steps)
        if world == 1 and args.render_steps > 0:
            out = None
            line["config_E_render"] = render_rates("E", dev, args.render_steps, 3, glue=args.glue)
            other_fp = "tight" if _C.get_footprint() == "rect" else "rect"  # the other footprint beside
            line["config_E_render_" + other_fp] = render_rates("E", dev, args.render_steps, 3, footprint=other_fp,
                                                               glue=args.glue)
            if args.glue_steps > 0:
                other = "reference" if args.glue == "fused" else "fused"
                line[f"config_E_render_{other}_glue"] = render_rates("E", dev, args.render_steps, 3, glue=other)
        if world == 1 and args.exchange_steps > 0:
            del out
            try:  # a side measurement: it must never cost the headline line
                line["exchange_1rank"] = exchange_one_rank_rates(cam, P, deg, target, bg, args.exchange_steps,
                                                                 args.warmup, line["ms_per_step"], args.glue)
            except Exception as e:  # noqa: BLE001
                line["exchange_1rank"] = {"status": "failed", "error": f"{type(e).__name__}: {e}"[:300]}
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline()
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


DOM_EVERY = 4  # timed region: events around the dominant stage on every 4th step
SPLIT_MIN_STEPS = 60  # the stage-split block before the timed region: past the device's ramp

STAGES_SOURCE = {
    "split": "HIP events around every rasterizer stage over a steady-state block of the same K steps right before "
             "the timed region (mean per launch); inside the timed region only the dominant stage carries events, "
             "on every 4th step",
    "all": "HIP events around every rasterizer stage inside the timed region (mean per launch)",
    "none": "not measured (--stage-events none)",
}


def stage_split(step_fn, steps: int):
    """Per-stage mean launch time over `steps` steady-state calls of step_fn, and the
    stage with the largest total: ({stage: (ms_per_launch, launches)}, dominant)."""
    import torch
    from diff_gaussian_rasterization import _C

    torch.cuda.synchronize()
    _C.timing_enable(True)
    for _ in range(steps):
        step_fn()
    torch.cuda.synchronize()
    stages = _C.timing_read()
    _C.timing_enable(False)
    per = {k: (ms / n, n) for k, (ms, n) in stages.items() if n}
    return per, _dominant(per)


# stages the caller marks around the exchange (multiview.GradAllReduce): regions of a
# step, not kernels, so never the roofline's kernel
EXCHANGE_STAGES = ("exchange_wait", "sh_rebuild")


def _dominant(per: dict) -> str:
    ks = [k for k in per if k not in EXCHANGE_STAGES]
    return max(ks, key=lambda k: per[k][0] * per[k][1]) if ks else "render_bwd"


def _exchange_split(stages: dict, calls: int) -> tuple:
    """Per-step means (ms) of the exchange's two regions from the library's stage
    events over the `calls` steps that recorded them (GradAllReduce.timing_every):
    the compute stream's wait for the collectives, the SH rebuild."""
    n = max(calls, 1)
    return tuple(stages.get(k, (0.0, 0))[0] / n for k in EXCHANGE_STAGES)


def footprint_rates(one_step, cam, g, bg, steps: int, warmup: int) -> dict:
    """The headline unit again with the other tile footprint (rect <-> tight):
    same image and gradients from lists of a different length."""
    import torch
    from diff_gaussian_rasterization import _C, set_footprint

    mode = "tight" if _C.get_footprint() == "rect" else "rect"
    prev = set_footprint(mode)
    try:
        for _ in range(max(warmup, 1)):
            one_step()
        I = num_rendered_seen()
        S = _C.last_spans(cam.image_width, cam.image_height)
        per, _ = stage_split(one_step, steps)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            one_step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    finally:
        set_footprint(prev)
    P, W, H, M = g.xyz.shape[0], cam.image_width, cam.image_height, g.features_rest.shape[1] + 1
    return {"footprint": mode, "value": round(steps / dt, 3), "unit": "train-iters/s",
            "iter_hbm_frac_measured": measured_frac("unit" + pmc_key("C", mode), steps / dt),
            "ms_per_step": round(1e3 * dt / steps, 4), "steps": steps, "num_rendered": I,
            "stages_ms": {k: round(v[0], 4) for k, v in per.items()}, "stages_source": STAGES_SOURCE["split"],
            "model_over_peak": model_over_peak(stage_model_fracs(per, P, I, W, H, M, True, S)),
            "raster_ms": raster_ms(per), "iter_algorithmic_bytes": iter_bytes(P, I, W, H, M),
            "iter_hbm_frac": round(iter_bytes(P, I, W, H, M) * steps / dt / 1e9 / HBM_PEAK_GBS, 4)}


GLUE_NOTE = {
    "fused": "fused: train_step.render_fused (rasterize_model over GaussianModel's stored parameters: the SH read "
             "from _features_dc/_features_rest without the cat, sigmoid/exp/normalize in the preprocess kernels, "
             "the leaves' gradients written by the backward) + the fused L1 kernel; same image, radii and "
             "gradients as the reference glue",
    "reference": "reference: train_step.render (gaussian_renderer/__init__.py:20-112 restated: activations, SH cat) "
                 "+ torch L1 (utils/loss_utils.py)",
}


def glue_rates(cam, g, target, bg, glue: str, steps: int, warmup: int, lambda_dssim: float) -> dict:
    """The headline unit again with the other glue around the rasterizer."""
    import torch

    import train_step

    params = g.params()

    def step():
        for p in params:
            p.grad = None
        train_step.train_step(cam, g, target, bg, lambda_dssim=lambda_dssim, glue=glue)

    for _ in range(warmup):
        step()
    per, _ = stage_split(step, steps)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"glue": GLUE_NOTE[glue], "value": round(steps / dt, 3), "unit": "train-iters/s",
            "ms_per_step": round(1e3 * dt / steps, 4), "steps": steps,
            "stages_ms": {k: round(v[0], 4) for k, v in per.items()}, "raster_ms": raster_ms(per)}


def train_config_rates(cfg_name: str, dev, steps: int, warmup: int, glue: str, lambda_dssim: float) -> dict:
    """Another training config's unit (B: 100k Gaussians, 800x800, SH3, render -> L1
    -> backward) at N = 1, the same way as the headline: stage split, timed steps,
    §8(d)'s iteration roofline, and the host's share (ms_per_step against the
    rasterizer's own device time, raster_ms)."""
    import torch
    from diff_gaussian_rasterization import _C

    import synthetic
    import train_step

    cfg = synthetic.CONFIGS[cfg_name]
    P, W, H, deg = cfg["P"], cfg["W"], cfg["H"], cfg["sh_degree"]
    M = (deg + 1) ** 2
    cam = synthetic.make_camera(W, H, view=0).to(dev)
    g = synthetic.make_gaussians(P, deg, seed=0).to(dev, requires_grad=True)
    target = synthetic.make_target(W, H, seed=1).to(dev)
    bg = torch.zeros(3, device=dev)
    params = g.params()

    def step():
        for p in params:
            p.grad = None
        train_step.train_step(cam, g, target, bg, lambda_dssim=lambda_dssim, glue=glue)

    for _ in range(max(warmup, 1)):
        step()
    torch.cuda.synchronize()
    I = num_rendered_seen()
    S = _C.last_spans(W, H)
    per, _ = stage_split(step, steps)
    torch.cuda.synchronize()
    _C.host_wait_ms(reset=True)
    t0 = time.perf_counter()
    host = 0.0
    for _ in range(steps):
        h0 = time.perf_counter()
        step()
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    wait = _C.host_wait_ms() * 1e-3
    ms = 1e3 * dt / steps
    eager = {"value": round(steps / dt, 3), "ms_per_step": round(ms, 4),
             "host_ms_per_step": round(1e3 * host / steps, 4), "host_wait_ms_per_step": round(1e3 * wait / steps, 4),
             "host_busy_ms_per_step": round(1e3 * (host - wait) / steps, 4)}
    # the same unit captured once as a HIP graph and replayed (train_step.CapturedUnit):
    # every kernel runs every step; one graph launch replaces the per-step Python,
    # autograd and ~20 kernel launches, which bound this small config
    graph = None
    if glue == "fused" and not lambda_dssim:
        unit = train_step.CapturedUnit(cam, g, target, bg, warmup=max(warmup // 4, 1))
        for _ in range(max(warmup, 1)):
            unit.replay()
        torch.cuda.synchronize()
        gt0 = time.perf_counter()
        ghost = 0.0
        for _ in range(steps):
            h0 = time.perf_counter()
            unit.replay()
            ghost += time.perf_counter() - h0
        torch.cuda.synchronize()
        gdt = time.perf_counter() - gt0
        n_graph = unit.check()  # raises if a replay's lists outgrew the captured capacity
        graph = {"value": round(steps / gdt, 3), "ms_per_step": round(1e3 * gdt / steps, 4),
                 "host_ms_per_step": round(1e3 * ghost / steps, 4),
                 "host_ms_per_step_vs_ms_per_step": round(ghost / gdt, 3), "num_rendered": n_graph,
                 "capacity": unit.capacities[-1]}
        del unit
    del g, params
    rms = raster_ms(per)
    if graph is not None and graph["value"] > eager["value"]:  # the line reports the faster form, both beside
        value, ms, host, wait, form = graph["value"], graph["ms_per_step"], ghost, 0.0, "graph"
    else:
        value, form = eager["value"], "eager"
    return {"metric": f"train iters/sec (fwd+bwd) + Mpix/sec, {W}x{H}, {P} Gaussians, SH{deg}",
            "value": value, "unit": "train-iters/s", "ms_per_step": round(ms, 4), "steps": steps,
            "form": form, "eager": eager, "graph": graph,
            "mpix_per_s": round(value * W * H / 1e6, 2),
            "config": {"workload": f"{cfg_name}: {WORKLOADS[cfg_name]}", "gaussians": P, "width": W, "height": H,
                       "sh_degree": deg, "num_rendered": I, "glue": GLUE_NOTE[glue]},
            "stages_ms": {k: round(v[0], 4) for k, v in per.items()}, "raster_ms": rms,
            "model_over_peak": model_over_peak(stage_model_fracs(per, P, I, W, H, M, True, S)),
            "host_ms_per_step": round(1e3 * host / steps, 4),
            "host_ms_per_step_vs_ms_per_step": round(1e3 * host / steps / ms, 3),
            # of which waiting for the device (the forward's num_rendered read-back), and the
            # host's own work: launches, autograd, Python
            "host_wait_ms_per_step": round(1e3 * wait / steps, 4),
            "host_busy_ms_per_step": round(1e3 * (host - wait) / steps, 4),
            "ms_per_step_vs_raster_ms": round(ms / rms, 3) if rms else None,
            "iter_algorithmic_bytes": iter_bytes(P, I, W, H, M),
            "iter_hbm_frac": round(iter_bytes(P, I, W, H, M) * value / 1e9 / HBM_PEAK_GBS, 4)}


def exchange_one_rank_rates(cam, P: int, deg: int, target, bg, steps: int, warmup: int, plain_ms: float,
                            glue: str = "fused") -> dict:
    """The headline unit with the N > 1 exchange forced on in a one-rank RCCL group
    ("nccl" backend, comm_force): the SH gradient leaves the backward as the view's
    colour-gradient record (all-gathered) and is rebuilt by sh_grad_from_colors, the
    xyz / opacity / scaling / rotation gradients are written by the rasterizer into
    the exchange's bucket and all-reduced — every collective of an N-rank step runs,
    over one rank.  What each rank of the driver's 1->8 run pays besides RCCL's
    transfers."""
    import socket

    import torch
    import torch.distributed as dist

    import diff_gaussian_rasterization as dgr
    import synthetic
    import train_step
    from diff_gaussian_rasterization import _C
    from multiview import GradAllReduce

    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    dev = bg.device
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    try:
        g = synthetic.make_gaussians(P, deg, seed=0).to(dev, requires_grad=True)
        params = g.params()
        ar = GradAllReduce(params, sh=(params[0], params[1], params[2]), comm_force=True, timing=True)

        def step():
            for p in params:
                p.grad = None
            train_step.train_step(cam, g, target, bg, glue=glue)
            ar()

        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        ar.reset_stats()
        _C.timing_enable(list(EXCHANGE_STAGES))
        _C.host_wait_ms(reset=True)
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        t_host = time.perf_counter() - t0
        t_wait = _C.host_wait_ms() * 1e-3
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        stages = _C.timing_read()
        _C.timing_enable(False)
        st = ar.stats()
        st["exchange_wait_ms"], st["sh_rebuild_ms"] = _exchange_split(stages, st["timed_calls"])
        plan = list(dgr.last_leaf_plan)
        ar.remove_hooks()
        del g, params
    finally:
        dist.destroy_process_group()
    ms = 1e3 * dt / steps
    return {"value": round(steps / dt, 3), "unit": "train-iters/s", "ms_per_step": round(ms, 4), "steps": steps,
            "vs_plain_ms": round(ms / plain_ms, 4) if plain_ms else None, "fused_leaves": plan,
            # the host's time in the forward's one wait: > 0 means the device, not the
            # host's Python / autograd / exchange work, sets the step
            "host_wait_ms_per_step": round(1e3 * t_wait / steps, 4),
            "host_busy_ms_per_step": round(1e3 * (t_host - t_wait) / steps, 4),
            "exchange_wait_ms": round(st["exchange_wait_ms"], 4), "sh_rebuild_ms": round(st["sh_rebuild_ms"], 4),
            "bytes_per_rank": st["bytes_per_rank"], "collective_backend": "RCCL (one rank, every collective forced)"}


def render_rates(cfg_name: str, dev, steps: int, warmup: int, view: int = 0, footprint=None,
                 glue: str = "fused") -> dict:
    """Forward-only throughput of reference render() (render.py:37-49 renders under
    torch.no_grad()) at a forward-only config (E: 5M Gaussians, 4K, SH3): frames/s,
    Mpix/s, the per-stage split, and the largest stage's algorithmic bytes ÷ its live
    time.  ``footprint`` ("rect": upstream's instance set, I = num_rendered as upstream
    bins it) overrides the package default for this measurement."""
    from diff_gaussian_rasterization import set_footprint

    prev = set_footprint(footprint) if footprint else None
    try:
        return _render_rates(cfg_name, dev, steps, warmup, view, glue)
    finally:
        if prev is not None:
            set_footprint(prev)


def _render_rates(cfg_name: str, dev, steps: int, warmup: int, view: int, glue: str = "fused") -> dict:
    import torch

    import synthetic
    import train_step
    from diff_gaussian_rasterization import _C

    cfg = synthetic.CONFIGS[cfg_name]
    P, W, H, deg = cfg["P"], cfg["W"], cfg["H"], cfg["sh_degree"]
    M = (deg + 1) ** 2
    cam = synthetic.make_camera(W, H, view=view).to(dev)
    g = synthetic.make_gaussians(P, deg, seed=0).to(dev)
    bg = torch.zeros(3, device=dev)
    render = train_step.render_fused if glue == "fused" else train_step.render
    with torch.no_grad():
        for _ in range(max(warmup, 1)):
            render(cam, g, bg)
        I = num_rendered_seen()
        S = _C.last_spans(W, H)
        # the largest stage by measured time, from a steady-state block of its own
        per, dom = stage_split(lambda: render(cam, g, bg), steps)
        _C.timing_enable([dom])  # only the dominant stage inside the timed region
        _C.timing_sample(DOM_EVERY)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            render(cam, g, bg)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        live = _C.timing_read()[dom]
        _C.timing_enable(False)
        _C.timing_sample(1)
    dom_ms = live[0] / live[1]
    ab = algorithmic_bytes(dom, P, I, W, H, M, False, S)
    fracs = stage_model_fracs(per, P, I, W, H, M, False, S)
    achieved = ab / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    fps = steps / dt
    sfx = pmc_key(cfg_name, _C.get_footprint())
    res = {
        "metric": render_metric(cfg_name), "value": round(fps, 3), "unit": "frames/s", "ms_per_frame": round(1e3 * dt / steps, 4),
        "mpix_per_s": round(fps * W * H / 1e6, 2), "steps": steps, "warmup": warmup,
        "config": {"workload": f"{cfg_name}: {WORKLOADS[cfg_name]}", "gaussians": P, "width": W, "height": H,
                   "sh_degree": deg, "footprint": _C.get_footprint(), "num_rendered": I, "glue": GLUE_NOTE[glue]},
        "stages_ms": {k: round(v[0], 4) for k, v in per.items()},
        "stages_source": STAGES_SOURCE["split"],
        "stage_hbm_frac": fracs, "model_over_peak": model_over_peak(fracs), "row_spans": S,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     # PMC bytes of this workload's own pass: keyed by config and footprint
                     "traffic": pmc_traffic(f"{dom}{sfx}") if glue == "fused" else None,
                     "algorithmic_bytes_per_launch": ab, "avg_launch_ms": round(dom_ms, 4)},
    }
    fwd_bytes = sum(algorithmic_bytes(k, P, I, W, H, M, False, S) for k in
                    ("preprocess", "scan", "depth_sort", "duplicate", "tile_sort", "render_fwd"))
    res["forward_algorithmic_bytes"] = fwd_bytes
    res["forward_hbm_frac"] = round(fwd_bytes * fps / 1e9 / HBM_PEAK_GBS, 4)
    res["raster_ms"] = raster_ms(per)
    res["iter_algorithmic_bytes"] = iter_bytes(P, I, W, H, M, backward=False)  # §8(d)'s forward formula
    res["iter_hbm_frac"] = round(res["iter_algorithmic_bytes"] * fps / 1e9 / HBM_PEAK_GBS, 4)
    res["iter_hbm_frac_measured"] = measured_frac(f"unit{sfx}", fps) if glue == "fused" else None
    del g
    torch.cuda.empty_cache()
    return res


def render_main(args, dev, world: int, rank: int) -> None:
    """--config E: the forward-only stress config as its own JSON line (views shard
    over ranks, no collective: each rank renders view rank % 8)."""
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.barrier()
    r = render_rates(args.config, dev, args.steps, args.warmup, view=rank % 8, glue=args.glue)
    elapsed = args.steps / r["value"]
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        W, H = r["config"]["width"], r["config"]["height"]
        value = world * args.steps / elapsed
        line = {"metric": render_metric(args.config), "value": round(value, 3), "unit": "frames/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
                "data": "synthetic (seeded Gaussians in a radius-2 ball, camera at distance 6, SURVEY.md §8d)",
                "config": dict(r["config"], views_per_step=world, parallelism=f"view-parallel x{world}"),
                "mpix_per_s": round(value * W * H / 1e6, 2), "stages_ms": r["stages_ms"], "roofline": r["roofline"],
                "forward_hbm_frac": r["forward_hbm_frac"], "cpu_baseline": None}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def full_step_rates(cam, P: int, deg: int, target, bg, steps: int) -> dict:
    """The reference-faithful training iteration (train.py:86-141 without logging and
    the periodic densify/prune): lr schedule, render, L1 + 0.2 (1 - SSIM), backward,
    densification statistics, Adam over the six groups, zero_grad — once with the
    reference's torch loss/Adam/statistics and once with the fused HIP kernels
    (SURVEY.md §8f rows 1-2).  Fresh Gaussians per variant; same seed."""
    import torch

    import synthetic
    import train_step

    out = {"definition": "render -> (1-0.2) L1 + 0.2 (1-SSIM) -> backward -> densification stats -> "
                         "Adam (6 groups, eps 1e-15) -> zero_grad; train.py:86-141 minus logging/densify-prune"}
    for name, fused in (("torch", False), ("fused", True)):
        g = synthetic.make_gaussians(P, deg, seed=0).to(bg.device, requires_grad=True)
        st = train_step.TrainState(g, spatial_lr_scale=6.6, fused=fused)
        it = 1
        for _ in range(3):
            train_step.full_train_step(it, cam, g, st, target, bg)
            it += 1
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            train_step.full_train_step(it, cam, g, st, target, bg)
            it += 1
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out[name] = {"it_per_s": round(steps / dt, 2), "ms_per_step": round(1e3 * dt / steps, 3)}
        del g, st
    return out


if __name__ == "__main__":
    main()
