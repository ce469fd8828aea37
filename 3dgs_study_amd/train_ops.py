"""Training-step ops after the rasterizer (SURVEY.md §8f "next" rows 1-2), host side.

* ``l1_ssim_loss(image, gt, lambda_dssim)`` — the reference's loss
  ``(1 - l) * l1_loss(image, gt) + l * (1 - ssim(image, gt))`` (train.py:103-105,
  utils/loss_utils.py:17-108) as ONE HIP pass that also produces d loss / d image;
  the autograd backward only scales that map by the incoming gradient.
* ``FusedAdam`` — torch.optim.Adam's update (scene/gaussian_model.py:176-205: six
  groups, lr 0 default, eps 1e-15) in one HIP launch over every parameter; state
  (``exp_avg``, ``exp_avg_sq``, ``step``) kept like torch's.
* ``densify_stats`` — train.py:126-127 + scene/gaussian_model.py:565-581
  (``max_radii2D``, ``xyz_gradient_accum``, ``denom``) in one HIP launch.
* ``dist_knn3`` — ``distCUDA2`` of the simple-knn submodule (scene/gaussian_model.py:
  153-155): mean squared distance to the 3 nearest other
  points, exact, through a uniform-grid HIP search.

All three call libgsr.so through the C ABI (include/gsr.h) on the current HIP
stream; there is no CPU path.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from diff_gaussian_rasterization import _C


def _cuda(t: torch.Tensor, name: str):
    if not t.is_cuda:
        raise RuntimeError(f"{name}: tensors must be on the GPU (no CPU implementation)")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name}: float32 expected, got {t.dtype}")


class _L1SSIM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, image, gt, lambda_dssim):
        lib = _C.load_library()
        _cuda(image, "l1_ssim_loss")
        _cuda(gt, "l1_ssim_loss")
        if image.shape != gt.shape or image.dim() != 3:
            raise RuntimeError(f"l1_ssim_loss: image {tuple(image.shape)} and gt {tuple(gt.shape)} must be equal [C,H,W]")
        x, y = image.contiguous(), gt.contiguous()
        C, H, W = x.shape
        # L1 alone (lambda 0): the loss here, its gradient in the backward from the
        # incoming dloss (gsr_l1_grad) — no map written here and scaled again there
        l1_only = float(lambda_dssim) == 0.0
        grad = None if l1_only else torch.empty_like(x)
        scratch = torch.empty(lib.gsr_l1_ssim_scratch_bytes(C, H, W), dtype=torch.uint8, device=x.device)
        out = torch.empty(3, dtype=torch.float32, device=x.device)
        _C._check(lib.gsr_l1_ssim(x.data_ptr(), y.data_ptr(), C, H, W, float(lambda_dssim),
                                  None if l1_only else grad.data_ptr(), scratch.data_ptr(), out.data_ptr(),
                                  _C._stream(x.device)), "gsr_l1_ssim")
        ctx.l1_only = l1_only
        ctx.save_for_backward(*((x, y) if l1_only else (grad,)))
        ctx.parts = out
        return out[0]

    @staticmethod
    def backward(ctx, g):
        if ctx.l1_only:
            x, y = ctx.saved_tensors
            lib = _C.load_library()
            grad = torch.empty_like(x)
            gd = g.detach().to(torch.float32).contiguous()
            _C._check(lib.gsr_l1_grad(x.data_ptr(), y.data_ptr(), x.numel(), gd.data_ptr(), grad.data_ptr(),
                                      _C._stream(x.device)), "gsr_l1_grad")
            return grad, None, None
        (grad,) = ctx.saved_tensors
        return grad * g, None, None


def l1_ssim_loss(image: torch.Tensor, gt: torch.Tensor, lambda_dssim: float = 0.2) -> torch.Tensor:
    """(1 - lambda) * L1 + lambda * (1 - SSIM) with the 11x11 sigma-1.5 window, mean over C*H*W."""
    return _L1SSIM.apply(image, gt, lambda_dssim)


class FusedAdam:
    """torch.optim.Adam (no weight decay, no amsgrad) over param groups, one launch per step.

    ``groups``: the reference's list of dicts (``params``, ``lr``, ``name``)."""

    def __init__(self, groups, lr: float = 0.0, betas=(0.9, 0.999), eps: float = 1e-15):
        self.param_groups = [dict(g) for g in groups]
        for g in self.param_groups:
            g.setdefault("lr", lr)
        if sum(len(g["params"]) for g in self.param_groups) > _C.ADAM_MAX_SEGS:
            raise ValueError(f"FusedAdam: at most {_C.ADAM_MAX_SEGS} tensors per launch")
        self.betas, self.eps = betas, eps
        self.state = {}

    @torch.no_grad()
    def step(self):
        """Validate every segment first, then advance the step counts and launch, so a
        rejected call leaves no parameter's state advanced."""
        lib = _C.load_library()
        segs = (_C.GsrAdamSegment * _C.ADAM_MAX_SEGS)()
        todo = []
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is None:
                    continue
                _cuda(p, "FusedAdam")
                if not (p.is_contiguous() and p.grad.is_contiguous()):
                    raise RuntimeError("FusedAdam: parameters and gradients must be contiguous")
                todo.append((g, p))
        if len(todo) > _C.ADAM_MAX_SEGS:
            raise RuntimeError(f"FusedAdam: at most {_C.ADAM_MAX_SEGS} tensors per launch")
        steps = {self.state[p]["step"] if p in self.state else 0 for _, p in todo}
        if len(steps) > 1:
            raise RuntimeError("FusedAdam: parameters at different step counts")
        if not todo:
            return
        step = steps.pop() + 1
        for n, (g, p) in enumerate(todo):
            st = self.state.get(p)
            if st is None:
                st = self.state[p] = {"step": 0, "exp_avg": torch.zeros_like(p), "exp_avg_sq": torch.zeros_like(p)}
            st["step"] = step
            segs[n] = _C.GsrAdamSegment(p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(),
                                        st["exp_avg_sq"].data_ptr(), p.numel(), float(g["lr"]))
        _C._check(lib.gsr_adam_step(segs, len(todo), step, self.betas[0], self.betas[1], self.eps,
                                    _C._stream(todo[0][1].device)), "gsr_adam_step")

    def zero_grad(self, set_to_none: bool = True):
        for g in self.param_groups:
            for p in g["params"]:
                if set_to_none:
                    p.grad = None
                elif p.grad is not None:
                    p.grad.zero_()


@torch.no_grad()
def densify_stats(radii: torch.Tensor, viewspace_grad: torch.Tensor, max_radii2D: torch.Tensor,
                  xyz_gradient_accum: torch.Tensor, denom: torch.Tensor):
    """In place, for radii > 0: max_radii2D = max(max_radii2D, radii); xyz_gradient_accum += |grad[:, :2]|;
    denom += 1 (train.py:126-127, scene/gaussian_model.py:565-581)."""
    lib = _C.load_library()
    for t, n in ((viewspace_grad, "viewspace_grad"), (max_radii2D, "max_radii2D"),
                 (xyz_gradient_accum, "xyz_gradient_accum"), (denom, "denom")):
        _cuda(t, f"densify_stats({n})")
    P = radii.shape[0]
    for t, n, shape in ((max_radii2D, "max_radii2D", (P,)), (xyz_gradient_accum, "xyz_gradient_accum", (P, 1)),
                        (denom, "denom", (P, 1))):
        # updated in place through their data pointers: a strided view would be misread
        if not t.is_contiguous() or t.dtype != torch.float32 or t.numel() != P:
            raise RuntimeError(f"densify_stats: {n} must be a contiguous float32 tensor of {P} elements "
                               f"(shape {shape}), got {tuple(t.shape)} {t.dtype}")
    vg = viewspace_grad.contiguous()
    _C._check(lib.gsr_densify_stats(P, radii.contiguous().data_ptr(), vg.data_ptr(), vg.shape[1],
                                    max_radii2D.data_ptr(), xyz_gradient_accum.data_ptr(), denom.data_ptr(),
                                    _C._stream(radii.device)), "gsr_densify_stats")


def dist_knn3(points: torch.Tensor) -> torch.Tensor:
    """distCUDA2(points): [P] mean of the squared distances from each point to its three
    nearest other points (FLT_MAX stands in for missing neighbours when P < 4)."""
    lib = _C.load_library()
    _cuda(points, "dist_knn3")
    if points.dim() != 2 or points.shape[1] != 3:
        raise RuntimeError(f"dist_knn3: points must be [P,3], got {tuple(points.shape)}")
    pts = points.detach().contiguous()
    P = pts.shape[0]
    out = torch.empty(P, dtype=torch.float32, device=pts.device)
    if P == 0:
        return out
    scratch = torch.empty(lib.gsr_knn_scratch_bytes(P), dtype=torch.uint8, device=pts.device)
    _C._check(lib.gsr_knn_mean_dist2(P, pts.data_ptr(), out.data_ptr(), scratch.data_ptr(), _C._stream(pts.device)),
              "gsr_knn_mean_dist2")
    return out


SH_C0 = 0.28209479177387814


def create_from_pcd(points, colors, max_sh_degree: int, device="cuda"):
    """GaussianModel.create_from_pcd (scene/gaussian_model.py:133-174) -> SynthGaussians:
    DC = RGB2SH(colors), higher SH zero, log scale = log(sqrt(max(dist_knn3, 1e-7))) x3,
    identity rotation, opacity = inverse_sigmoid(0.1)."""
    from synthetic import SynthGaussians

    xyz = torch.as_tensor(np.asarray(points), dtype=torch.float32).to(device)
    rgb = torch.as_tensor(np.asarray(colors), dtype=torch.float32).to(device)
    P = xyz.shape[0]
    M = (max_sh_degree + 1) ** 2
    features = torch.zeros((P, 3, M), dtype=torch.float32, device=device)
    features[:, :3, 0] = (rgb - 0.5) / SH_C0
    dist2 = torch.clamp_min(dist_knn3(xyz), 0.0000001)
    scales = torch.log(torch.sqrt(dist2))[..., None].repeat(1, 3)
    rots = torch.zeros((P, 4), device=device)
    rots[:, 0] = 1
    op = torch.full((P, 1), 0.1, dtype=torch.float32, device=device)
    opacities = torch.log(op / (1 - op))
    return SynthGaussians(xyz, features[:, :, 0:1].transpose(1, 2).contiguous(),
                          features[:, :, 1:].transpose(1, 2).contiguous(), scales, rots, opacities,
                          max_sh_degree, 0)
