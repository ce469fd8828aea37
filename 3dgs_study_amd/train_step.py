"""The render -> loss -> backward unit around the rasterizer (host side).

``render`` reproduces the reference's ``gaussian_renderer.render``
(gaussian_renderer/__init__.py:20-112) against this
package's ``diff_gaussian_rasterization``: the dummy screen-space means
(``zeros_like(xyz) + 0`` with ``retain_grad``), tan-FoV, the 12-field settings,
the SH-vs-precomputed-colour and scale/rotation-vs-cov3D branches, and the
returned dict.  It exists so that tests and ``bench.py`` can drive the boundary
exactly as the reference does on a machine where the reference is absent (the
GPU box).  ``eval_sh`` / ``covariance`` restate utils/sh_utils.py:57-112 and
utils/general_utils.py:86-128 + scene/gaussian_model.py:27-32 for the
``convert_SHs_python`` / ``compute_cov3D_python`` branches.

``render_fused`` is the same render over GaussianModel's stored parameters
(``diff_gaussian_rasterization.rasterize_model``): no SH cat, no activation
kernels, the leaves' gradients written by the rasterizer's backward — the same
image, radii and gradients.

``train_step`` is the unit bench.py times: one view's render, the loss of
train.py:102-104 (L1, or L1 + 0.2·(1 - SSIM)), and ``loss.backward()``; with
``glue="fused"`` through ``render_fused`` and the fused loss kernel
(``train_ops.l1_ssim_loss``), with ``glue="reference"`` through ``render`` and the
reference's torch loss.  ``CapturedUnit`` is the fused unit captured once as a HIP
graph and replayed (the same kernels, one graph launch per step).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396)
SH_C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435)


def eval_sh(deg: int, sh: torch.Tensor, dirs: torch.Tensor) -> torch.Tensor:
    """SH -> value for degree <= 3; sh [..., C, (deg+1)^2], dirs [..., 3] (utils/sh_utils.py:57-112)."""
    assert 0 <= deg <= 3 and sh.shape[-1] >= (deg + 1) ** 2
    out = SH_C0 * sh[..., 0]
    if deg > 0:
        x, y, z = dirs[..., 0:1], dirs[..., 1:2], dirs[..., 2:3]
        out = out - SH_C1 * y * sh[..., 1] + SH_C1 * z * sh[..., 2] - SH_C1 * x * sh[..., 3]
        if deg > 1:
            xx, yy, zz = x * x, y * y, z * z
            xy, yz, xz = x * y, y * z, x * z
            out = (out + SH_C2[0] * xy * sh[..., 4] + SH_C2[1] * yz * sh[..., 5] +
                   SH_C2[2] * (2.0 * zz - xx - yy) * sh[..., 6] + SH_C2[3] * xz * sh[..., 7] +
                   SH_C2[4] * (xx - yy) * sh[..., 8])
            if deg > 2:
                out = (out + SH_C3[0] * y * (3 * xx - yy) * sh[..., 9] + SH_C3[1] * xy * z * sh[..., 10] +
                       SH_C3[2] * y * (4 * zz - xx - yy) * sh[..., 11] +
                       SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[..., 12] +
                       SH_C3[4] * x * (4 * zz - xx - yy) * sh[..., 13] + SH_C3[5] * z * (xx - yy) * sh[..., 14] +
                       SH_C3[6] * x * (xx - 3 * yy) * sh[..., 15])
    return out


def rotation_matrix(q: torch.Tensor) -> torch.Tensor:
    """Normalised quaternion (r,x,y,z) -> R [P,3,3] (utils/general_utils.py:86-117)."""
    q = q / torch.sqrt((q * q).sum(dim=1, keepdim=True))
    r, x, y, z = q.unbind(dim=1)
    return torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
        2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
        2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], dim=1).view(-1, 3, 3)


def covariance(scaling: torch.Tensor, scaling_modifier: float, rotation: torch.Tensor) -> torch.Tensor:
    """Upper triangle of (R S)(R S)^T -> [P,6] (scene/gaussian_model.py:27-32)."""
    L = rotation_matrix(rotation) * (scaling_modifier * scaling)[:, None, :]
    S = L @ L.transpose(1, 2)
    return torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], dim=1)


def render(viewpoint_camera, pc, bg_color: torch.Tensor, scaling_modifier: float = 1.0, override_color=None,
           convert_SHs_python: bool = False, compute_cov3D_python: bool = False, debug: bool = False) -> dict:
    xyz = pc.get_xyz
    screenspace_points = torch.zeros_like(xyz, dtype=xyz.dtype, requires_grad=True, device=xyz.device) + 0
    try:
        screenspace_points.retain_grad()
    except Exception:
        pass
    tanfovx = math.tan(viewpoint_camera.FoVx * 0.5)
    tanfovy = math.tan(viewpoint_camera.FoVy * 0.5)
    raster_settings = GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=tanfovx, tanfovy=tanfovy, bg=bg_color, scale_modifier=scaling_modifier,
        viewmatrix=viewpoint_camera.world_view_transform, projmatrix=viewpoint_camera.full_proj_transform,
        sh_degree=pc.active_sh_degree, campos=viewpoint_camera.camera_center, prefiltered=False, debug=debug)
    rasterizer = GaussianRasterizer(raster_settings=raster_settings)
    scales = rotations = cov3D_precomp = None
    if compute_cov3D_python:
        cov3D_precomp = covariance(pc.get_scaling, scaling_modifier, pc.rotation)
    else:
        scales = pc.get_scaling
        rotations = pc.get_rotation
    shs = colors_precomp = None
    if override_color is None:
        if convert_SHs_python:
            feats = pc.get_features
            shs_view = feats.transpose(1, 2).view(-1, 3, (pc.max_sh_degree + 1) ** 2)
            dir_pp = xyz - viewpoint_camera.camera_center.repeat(feats.shape[0], 1)
            dir_pp_normalized = dir_pp / dir_pp.norm(dim=1, keepdim=True)
            colors_precomp = torch.clamp_min(eval_sh(pc.active_sh_degree, shs_view, dir_pp_normalized) + 0.5, 0.0)
        else:
            shs = pc.get_features
    else:
        colors_precomp = override_color
    rendered_image, radii = rasterizer(means3D=xyz, means2D=screenspace_points, shs=shs, colors_precomp=colors_precomp,
                                       opacities=pc.get_opacity, scales=scales, rotations=rotations,
                                       cov3D_precomp=cov3D_precomp)
    return {"render": rendered_image, "viewspace_points": screenspace_points, "visibility_filter": radii > 0,
            "radii": radii}


def stored_parameters(pc):
    """GaussianModel's leaves (scene/gaussian_model.py:44-49: _xyz, _features_dc,
    _features_rest, _opacity, _scaling, _rotation), from a reference GaussianModel or
    a synthetic.SynthGaussians (same tensors without the underscores)."""
    names = ("xyz", "features_dc", "features_rest", "opacity", "scaling", "rotation")
    if hasattr(pc, "_xyz"):
        return tuple(getattr(pc, "_" + n) for n in names)
    return tuple(getattr(pc, n) for n in names)


def render_fused(viewpoint_camera, pc, bg_color: torch.Tensor, scaling_modifier: float = 1.0,
                 debug: bool = False, l1_target: torch.Tensor = None) -> dict:
    """``render`` (gaussian_renderer/__init__.py:20-112, SH and scale/rotation
    branches) over the model's stored parameters: the rasterizer activates them and
    reads the SH from _features_dc / _features_rest itself (rasterize_model).  The
    screen-space gradient carrier is a leaf whose values nothing reads (upstream's
    ``zeros_like + 0`` with ``retain_grad`` carries the same gradient in ``.grad``;
    the rasterizer ignores the values, so they are left unset here: no fill launch).
    ``l1_target``: also the L1 loss against it (``out["l1"]``; rasterize_model), whose
    image gradient the render backward forms itself."""
    xyz, f_dc, f_rest, opacity, scaling, rotation = stored_parameters(pc)
    screenspace_points = torch.empty_like(xyz, dtype=xyz.dtype, device=xyz.device).requires_grad_(True)
    raster_settings = GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=math.tan(viewpoint_camera.FoVx * 0.5), tanfovy=math.tan(viewpoint_camera.FoVy * 0.5), bg=bg_color,
        scale_modifier=scaling_modifier, viewmatrix=viewpoint_camera.world_view_transform,
        projmatrix=viewpoint_camera.full_proj_transform, sh_degree=pc.active_sh_degree,
        campos=viewpoint_camera.camera_center, prefiltered=False, debug=debug)
    rasterizer = GaussianRasterizer(raster_settings=raster_settings)
    res = rasterizer.forward_model(xyz, screenspace_points, f_dc, f_rest, opacity, scaling, rotation, l1_target)
    out = {"render": res[0], "viewspace_points": screenspace_points,
           "visibility_filter": res[3] if l1_target is not None else res[1] > 0, "radii": res[1]}
    if l1_target is not None:
        out["l1"] = res[2]
    return out


# ---------------------------------------------------------------- losses (utils/loss_utils.py)
def l1_loss(network_output: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
    return torch.abs(network_output - gt).mean()


def _gaussian_window(window_size: int, sigma: float, channel: int, device, dtype) -> torch.Tensor:
    x = torch.arange(window_size, dtype=torch.float64) - window_size // 2
    g = torch.exp(-(x ** 2) / (2 * sigma ** 2))
    g = (g / g.sum()).to(dtype)
    w2 = g[:, None] @ g[None, :]
    return w2.expand(channel, 1, window_size, window_size).contiguous().to(device)


def ssim(img1: torch.Tensor, img2: torch.Tensor, window_size: int = 11) -> torch.Tensor:
    """SSIM with an 11x11 Gaussian window (sigma 1.5), depthwise conv2d, mean over pixels."""
    channel = img1.size(-3)
    w = _gaussian_window(window_size, 1.5, channel, img1.device, img1.dtype)
    x1 = img1.unsqueeze(0) if img1.dim() == 3 else img1
    x2 = img2.unsqueeze(0) if img2.dim() == 3 else img2
    pad = window_size // 2
    mu1 = F.conv2d(x1, w, padding=pad, groups=channel)
    mu2 = F.conv2d(x2, w, padding=pad, groups=channel)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    sigma1_sq = F.conv2d(x1 * x1, w, padding=pad, groups=channel) - mu1_sq
    sigma2_sq = F.conv2d(x2 * x2, w, padding=pad, groups=channel) - mu2_sq
    sigma12 = F.conv2d(x1 * x2, w, padding=pad, groups=channel) - mu1_mu2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    ssim_map = ((2 * mu1_mu2 + C1) * (2 * sigma12 + C2)) / ((mu1_sq + mu2_sq + C1) * (sigma1_sq + sigma2_sq + C2))
    return ssim_map.mean()


GLUES = ("fused", "reference")
_SEEDS: dict = {}


def _unit_seed(loss: torch.Tensor) -> torch.Tensor:
    """A cached 1.0 of the loss's device and dtype: ``loss.backward(seed)`` is
    ``loss.backward()`` without the per-step ``ones_like`` fill kernel.  Nothing
    writes the seed (the loss backward only reads dloss)."""
    key = (loss.device, loss.dtype)
    t = _SEEDS.get(key)
    if t is None:
        t = _SEEDS[key] = torch.ones((), device=loss.device, dtype=loss.dtype)
    return t


def train_step(camera, gaussians, target: torch.Tensor, bg: torch.Tensor, lambda_dssim: float = 0.0,
               glue: str = "reference") -> dict:
    """render -> loss -> backward for one view (train.py:98-105). lambda_dssim=0 is the
    L1-only headline unit; 0.2 is the reference's default loss.
    glue="reference": the reference's render() and torch loss; "fused": render_fused
    and the fused loss kernel (same values)."""
    if glue == "fused":
        import train_ops

        if lambda_dssim:
            out = render_fused(camera, gaussians, bg)
            loss = train_ops.l1_ssim_loss(out["render"], target, lambda_dssim)
        else:  # the L1 loss out of the rasterizer: its gradient formed in the render backward
            out = render_fused(camera, gaussians, bg, l1_target=target)
            loss = out["l1"]
        loss.backward(_unit_seed(loss))  # the seed dloss = 1 without a fill launch per step
        out["loss"] = loss
        return out
    elif glue == "reference":
        out = render(camera, gaussians, bg)
        image = out["render"]
        loss = l1_loss(image, target)
        if lambda_dssim:
            loss = (1.0 - lambda_dssim) * loss + lambda_dssim * (1.0 - ssim(image, target))
    else:
        raise ValueError(f"glue must be one of {GLUES} (got {glue!r})")
    loss.backward()
    out["loss"] = loss
    return out


class CapturedUnit:
    """One fused training unit (render -> L1 -> loss.backward(), ``train_step`` with
    glue="fused") captured once as a CUDA (HIP) graph and replayed: every kernel of
    the unit runs on every replay, over the same parameter, camera and target
    tensors (update them in place between replays: an optimizer step, a new view's
    matrices copied into the captured ones), with one graph launch instead of the
    per-step Python, autograd and ~20 kernel launches.  The gradients land in the
    leaves' ``.grad`` tensors the capture created (``self.out`` holds the image,
    loss, radii and visibility of the latest replay).

    The capture needs an eager step of the same scene size first (warm-up, which
    also sizes the binning buffer); inside it the forward queues everything without
    reading num_rendered back (gsr.h GSR_FLAG_NO_WAIT), so ``check()`` — after a
    synchronize — confirms the last replay's count fit the captured capacity and
    raises otherwise (capture again then)."""

    def __init__(self, camera, gaussians, target: torch.Tensor, bg: torch.Tensor, warmup: int = 3):
        from diff_gaussian_rasterization import _C

        self._C = _C
        params = gaussians.params()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up on a side stream (torch.cuda.graph's recipe)
            for _ in range(max(warmup, 1)):
                for p in params:
                    p.grad = None
                train_step(camera, gaussians, target, bg, glue="fused")
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        for p in params:
            p.grad = None
        n0 = len(_C.captured_forwards)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = train_step(camera, gaussians, target, bg, glue="fused")
        self.captured = _C.captured_forwards[n0:]  # (capacity, depth passes) per captured forward
        self.capacities = [c for c, _ in self.captured]
        del _C.captured_forwards[n0:]

    def replay(self) -> dict:
        self.graph.replay()
        return self.out

    def check(self) -> int:
        """num_rendered of the last replay (after torch.cuda.synchronize()); raises if
        it exceeded the captured binning capacity."""
        return self._C.forward_status(self.captured[-1])


# ---------------------------------------------------------------- the full training step (train.py:86-141)
def expon_lr(lr_init: float, lr_final: float, lr_delay_steps: int = 0, lr_delay_mult: float = 1.0,
             max_steps: int = 1_000_000):
    """utils/general_utils.py:30-69 get_expon_lr_func (log-linear decay, optional delay)."""

    def helper(step):
        if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
            return 0.0
        if lr_delay_steps > 0:
            delay = lr_delay_mult + (1 - lr_delay_mult) * math.sin(0.5 * math.pi * min(max(step / lr_delay_steps, 0), 1))
        else:
            delay = 1.0
        t = min(max(step / max_steps, 0), 1)
        return delay * math.exp(math.log(lr_init) * (1 - t) + math.log(lr_final) * t)

    return helper


# OptimizationParams defaults (arguments/__init__.py:79-93)
OPT = dict(position_lr_init=0.00016, position_lr_final=0.0000016, position_lr_delay_mult=0.01,
           position_lr_max_steps=30_000, feature_lr=0.0025, opacity_lr=0.05, scaling_lr=0.005, rotation_lr=0.001,
           lambda_dssim=0.2, densify_until_iter=15_000)


class TrainState:
    """The optimizer side of GaussianModel for a SynthGaussians: the six Adam groups
    (scene/gaussian_model.py:176-205, lr 0 default, eps 1e-15), the xyz learning-rate
    schedule and the densification statistics (:565-581).  ``fused`` swaps torch's
    Adam and statistics for the HIP kernels of train_ops.py."""

    def __init__(self, g, spatial_lr_scale: float, fused: bool = False, opt: dict = OPT):
        import train_ops

        self.opt, self.fused = opt, fused
        groups = [
            {"params": [g.xyz], "lr": opt["position_lr_init"] * spatial_lr_scale, "name": "xyz"},
            {"params": [g.features_dc], "lr": opt["feature_lr"], "name": "f_dc"},
            {"params": [g.features_rest], "lr": opt["feature_lr"] / 20.0, "name": "f_rest"},
            {"params": [g.opacity], "lr": opt["opacity_lr"], "name": "opacity"},
            {"params": [g.scaling], "lr": opt["scaling_lr"], "name": "scaling"},
            {"params": [g.rotation], "lr": opt["rotation_lr"], "name": "rotation"},
        ]
        if fused:
            self.optimizer = train_ops.FusedAdam(groups, lr=0.0, eps=1e-15)
        else:
            self.optimizer = torch.optim.Adam(groups, lr=0.0, eps=1e-15)
        self.xyz_scheduler = expon_lr(opt["position_lr_init"] * spatial_lr_scale,
                                      opt["position_lr_final"] * spatial_lr_scale,
                                      lr_delay_mult=opt["position_lr_delay_mult"],
                                      max_steps=opt["position_lr_max_steps"])
        P, dev = g.xyz.shape[0], g.xyz.device
        self.xyz_gradient_accum = torch.zeros((P, 1), device=dev)
        self.denom = torch.zeros((P, 1), device=dev)
        self.max_radii2D = torch.zeros((P,), device=dev)

    def update_learning_rate(self, iteration: int):
        for group in self.optimizer.param_groups:
            if group["name"] == "xyz":
                group["lr"] = self.xyz_scheduler(iteration)
                return group["lr"]

    def reduce_densification_stats(self, group=None):
        """View-parallel: the per-rank statistics SUM / SUM / MAX-reduced over the group
        for a densify step, as copies (xyz_gradient_accum, denom, max_radii2D); the
        per-rank accumulators are left alone (multiview.reduce_densification_stats)."""
        import multiview

        return multiview.reduce_densification_stats(self.xyz_gradient_accum, self.denom, self.max_radii2D, group)

    @torch.no_grad()
    def densification_stats(self, out: dict):
        radii, vis, vsp = out["radii"], out["visibility_filter"], out["viewspace_points"]
        if self.fused:
            import train_ops

            train_ops.densify_stats(radii, vsp.grad, self.max_radii2D, self.xyz_gradient_accum, self.denom)
        else:  # train.py:126-127 and scene/gaussian_model.py:565-581
            self.max_radii2D[vis] = torch.max(self.max_radii2D[vis], radii[vis])
            self.xyz_gradient_accum[vis] += torch.norm(vsp.grad[vis, :2], dim=-1, keepdim=True)
            self.denom[vis] += 1


def full_train_step(iteration: int, camera, gaussians, state: TrainState, target: torch.Tensor,
                    bg: torch.Tensor, reducer=None) -> torch.Tensor:
    """One iteration of train.py:86-141 without logging, checkpoints and the periodic
    densify/prune/opacity reset: lr schedule, render, L1 + lambda (1 - SSIM), backward,
    densification statistics, Adam step, zero_grad.  ``state.fused`` selects
    render_fused and the HIP loss/Adam/statistics kernels (train_ops.py) over the
    reference's render() glue and torch ops.

    View-parallel: ``reducer`` (multiview.GradAllReduce over the
    process group) finishes the gradient exchange started inside the backward before
    the optimizer step, so every rank steps on the sum of all ranks' views and the
    replicas stay identical; ``camera``/``target`` are this rank's view.  The
    densification statistics stay per rank until a densify step combines them
    (TrainState.reduce_densification_stats)."""
    state.update_learning_rate(iteration)
    out = render_fused(camera, gaussians, bg) if state.fused else render(camera, gaussians, bg)
    image = out["render"]
    lam = state.opt["lambda_dssim"]
    if state.fused:
        import train_ops

        loss = train_ops.l1_ssim_loss(image, target, lam)
    else:
        loss = (1.0 - lam) * l1_loss(image, target) + lam * (1.0 - ssim(image, target))
    loss.backward()
    if reducer is not None:
        reducer()
    with torch.no_grad():
        if iteration < state.opt["densify_until_iter"]:
            state.densification_stats(out)
        state.optimizer.step()
        state.optimizer.zero_grad(set_to_none=True)
    return loss
