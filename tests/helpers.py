"""Shared test helpers: run the same seeded case through the HIP library (via the
drop-in ``_C`` surface) and through the CPU oracle, and read the HIP scratch
buffers back as the upstream intermediates (radii, tiles_touched, offsets,
ranges, point_list, final_T, n_contrib)."""
from __future__ import annotations

import math

import numpy as np
import torch

import synthetic


def case(P, W, H, deg, seed=0, view=0, active=None, radius=2.0, scale_range=(0.003, 0.03), distance=6.0):
    cam = synthetic.make_camera(W, H, view, distance=distance)
    g = synthetic.make_gaussians(P, deg, seed=seed, radius=radius, scale_range=scale_range,
                                 active_sh_degree=active)
    return cam, g


def activated(g, python_branch=False, scale_modifier=1.0):
    """The tensors render() hands the rasterizer (CPU, float32, contiguous)."""
    from train_step import covariance, eval_sh  # noqa: F401

    with torch.no_grad():
        d = dict(means3D=g.get_xyz.contiguous(), opacities=g.get_opacity.contiguous())
        if python_branch:
            d["cov3D_precomp"] = covariance(g.get_scaling, scale_modifier, g.rotation).contiguous()
        else:
            d["scales"] = g.get_scaling.contiguous()
            d["rotations"] = g.get_rotation.contiguous()
        d["shs"] = g.get_features.contiguous()
    return d


def run_hip(cam, g, dev, bg=(0.0, 0.0, 0.0), scale_modifier=1.0, colors_precomp=None, python_branch=False,
            dL=None, debug=False, dsh_planar=False, footprint="rect", misalign_sh=False, prepare=None):
    """prepare: the forward's GSR_FLAG_PREPARE_BACKWARD (None: the binding's default,
    off here — the inputs need no grad); with it the backward replays the forward's
    chunk masks and, for long lists, its split-replay checkpoints."""
    from diff_gaussian_rasterization import _C

    a = activated(g, python_branch, scale_modifier)
    t = lambda x: x.to(dev) if x is not None else torch.empty(0, device=dev)  # noqa: E731
    bg_t = torch.tensor(bg, dtype=torch.float32, device=dev)
    shs = t(a["shs"]) if colors_precomp is None else t(None)
    if misalign_sh and shs.numel():  # contiguous, 4 B past a 16-B boundary: the LDS-staged row path
        buf = torch.empty(shs.numel() + 1, dtype=shs.dtype, device=dev)
        shs = buf[1:].view_as(shs).copy_(shs)
    colors = t(torch.as_tensor(colors_precomp, dtype=torch.float32)) if colors_precomp is not None else t(None)
    args = (bg_t, t(a["means3D"]), colors, t(a["opacities"]), t(a.get("scales")), t(a.get("rotations")),
            float(scale_modifier), t(a.get("cov3D_precomp")), t(cam.world_view_transform),
            t(cam.full_proj_transform), math.tan(cam.FoVx * 0.5), math.tan(cam.FoVy * 0.5), cam.image_height,
            cam.image_width, shs, g.active_sh_degree, t(cam.camera_center), False, debug)
    I, color, radii, geom, binning, img = _C.rasterize_gaussians(*args, footprint=footprint, prepare_backward=prepare)
    torch.cuda.synchronize()
    P, W, H = a["means3D"].shape[0], cam.image_width, cam.image_height
    out = dict(num_rendered=I, color=color.cpu().numpy(), radii=radii.cpu().numpy(), footprint=footprint)
    out.update(read_intermediates(geom, binning, img, P, W, H, I))
    out["keys64"] = _C.point_list_keys(P, W, H, geom, binning, I).cpu().numpy().view(np.uint64)
    if dL is not None:
        g_ = torch.as_tensor(dL, dtype=torch.float32).to(dev)
        bargs = (bg_t, args[1], radii, colors, args[4], args[5], float(scale_modifier), args[7], args[8], args[9],
                 args[10], args[11], g_, shs, g.active_sh_degree, args[16], geom, I, binning, img, debug)
        names = ("dmeans2D", "dcolors", "dopacity", "dmeans3D", "dcov3D", "dsh", "dscales", "drot")
        grads = _C.rasterize_gaussians_backward(*bargs, dsh_planar=dsh_planar)
        if dsh_planar and shs.numel():
            M = shs.size(1)
            assert grads[5].shape == shs.shape and grads[5].stride() == (3, 3 * shs.size(0), 1), grads[5].stride()
            assert grads[5].permute(1, 0, 2).is_contiguous() and M == grads[5].size(1)
        torch.cuda.synchronize()
        out["grads"] = {n: x.cpu().numpy() for n, x in zip(names, grads)}
    return out


def _view(buf, off, n, dtype, np_dtype):
    nbytes = n * np.dtype(np_dtype).itemsize
    if n == 0:
        return np.zeros(0, np_dtype)
    return buf[off:off + nbytes].view(dtype).cpu().numpy().view(np_dtype)


def read_intermediates(geom, binning, img, P, W, H, I):
    from diff_gaussian_rasterization import _C

    go, bo, io = _C.layouts(P, W, H, I)
    T = ((W + 15) // 16) * ((H + 15) // 16)
    d = {}
    d["depths"] = _view(geom, go["depths"], P, torch.float32, np.float32)
    d["means2D"] = _view(geom, go["means2D"], 2 * P, torch.float32, np.float32).reshape(P, 2)
    d["splats"] = _view(geom, go["splats"], 12 * P, torch.float32, np.float32).reshape(P, 12)
    d["clamped"] = _view(geom, go["clamped"], P, torch.uint8, np.uint8)
    d["tiles_touched"] = _view(geom, go["tiles_touched"], P, torch.int32, np.uint32)
    d["ctrl"] = _view(geom, go["ctrl"], 16, torch.int32, np.uint32)
    d["ranges"] = _view(geom, go["ranges"], 2 * T, torch.int32, np.uint32).reshape(T, 2)
    d["depth_order"] = _view(geom, go["depth_order"], P, torch.int32, np.uint32)
    d["dsort_ctrl"] = _view(geom, go["dsort_ctrl"], 16, torch.int32, np.uint32)
    d["point_list"] = _view(binning, bo["point_list"], I, torch.int32, np.uint32) if I > 0 else np.zeros(0, np.uint32)
    d["final_T"] = _view(img, io["final_T"], W * H, torch.float32, np.float32).reshape(H, W)
    d["n_contrib"] = _view(img, io["n_contrib"], W * H, torch.int32, np.uint32).reshape(H, W)
    return d


def run_oracle(oracle, cam, g, bg=(0.0, 0.0, 0.0), scale_modifier=1.0, colors_precomp=None, python_branch=False,
               mt=False):
    """mt: the oracle's OpenMP build (forward bit-identical; the render backward
    adds per-thread partial gradients, a different float order) for full-size cases."""
    a = activated(g, python_branch, scale_modifier)
    kw = dict(scale_modifier=scale_modifier, sh_degree=g.active_sh_degree, mt=mt)
    if colors_precomp is None:
        kw["shs"] = a["shs"].numpy()
    else:
        kw["colors_precomp"] = np.asarray(colors_precomp, np.float32)
    if python_branch:
        kw["cov3D_precomp"] = a["cov3D_precomp"].numpy()
    else:
        kw["scales"] = a["scales"].numpy()
        kw["rotations"] = a["rotations"].numpy()
    return oracle.forward(a["means3D"].numpy(), a["opacities"].numpy(), cam.world_view_transform.numpy(),
                          cam.full_proj_transform.numpy(), cam.camera_center.numpy(), np.asarray(bg, np.float32),
                          cam.image_height, cam.image_width, math.tan(cam.FoVx * 0.5), math.tan(cam.FoVy * 0.5),
                          **kw)


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = np.linalg.norm(b)
    if den == 0:
        return float(np.linalg.norm(a))
    return float(np.linalg.norm(a - b) / den)


def random_dL(H, W, seed=5):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal((3, H, W)) / (H * W)).astype(np.float32)
