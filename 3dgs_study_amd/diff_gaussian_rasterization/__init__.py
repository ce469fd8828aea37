"""diff_gaussian_rasterization — MI355X (gfx950) drop-in for the rasterizer the
reference imports at ``gaussian_renderer/__init__.py:14``.

Public surface (same names, field order, argument meaning and errors as the
upstream 2-output API the reference is written against):

* ``GaussianRasterizationSettings`` — NamedTuple with the 12 fields built at
  ``gaussian_renderer/__init__.py:47-60``;
* ``GaussianRasterizer(raster_settings)`` — ``nn.Module``; ``forward(means3D, means2D,
  opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
  cov3D_precomp=None) -> (color [3,H,W], radii [P] int32)`` as called at
  ``gaussian_renderer/__init__.py:98-106``; ``markVisible(positions) -> bool [P]``;
* ``rasterize_gaussians(...)`` — the functional form behind the module.

Autograd: ``backward`` maps the 8 native gradients onto the 9 inputs
``(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
cov3Ds_precomp, raster_settings)``; ``means2D.grad[:, :2]`` (NDC-scaled screen-space
gradient) feeds densification at ``scene/gaussian_model.py:576-580``.

View-parallel SH exchange (not upstream; ``3dgs_study_amd/multiview.py``): while a
sink is installed with ``set_sh_grad_sink``, a backward with SH input hands the
sink the view's colour gradient instead of returning dsh (the ``sh`` input then
gets no gradient through autograd; the sink rebuilds the SH leaf gradients summed
over all ranks' views).  ``set_sh_grad_sink(None)`` restores upstream behaviour.

Tile footprint (not upstream; ``set_footprint``, env ``GSR_FOOTPRINT``): "rect"
bins every tile of upstream's getRect rect, so ``num_rendered`` and the binning
buffer's lists are upstream's bit for bit; "tight" (default) bins only the tiles
the alpha >= 1/255 ellipse reaches — the same image, radii and gradients from
shorter lists (of upstream's outputs only the ``num_rendered`` integer differs).

Debug mode (``raster_settings.debug``): the native side synchronises after every
kernel; on failure a CPU copy of the arguments is written to
``snapshot_fw.dump`` / ``snapshot_bw.dump`` before the exception propagates.
"""
from __future__ import annotations

from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C

from ._C import get_footprint, set_footprint  # noqa: E402

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "set_sh_grad_sink",
           "set_footprint", "get_footprint"]

_sh_grad_sink = None


def set_sh_grad_sink(sink):
    """Install (or with None remove) the view-parallel SH-gradient sink.  The sink
    provides ``accepts(sh, means3D) -> bool``, ``record(P) -> float32 tensor`` of
    ``_C.sh_record_floats(P)`` elements, and ``push(record, campos, sh_degree)``."""
    global _sh_grad_sink
    prev, _sh_grad_sink = _sh_grad_sink, sink
    return prev


def _cpu_snapshot(args):
    return tuple(a.detach().cpu().clone() if isinstance(a, torch.Tensor) else a for a in args)


def _call_native(fn, args, debug: bool, dump: str, stage: str):
    if not debug:
        return fn(*args)
    saved = _cpu_snapshot(args)  # copy before a faulting kernel can corrupt them
    try:
        return fn(*args)
    except Exception:
        torch.save(saved, dump)
        print(f"\nAn error occured in {stage}. Please forward {dump} for debugging.")
        raise


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings):
        rs = raster_settings
        args = (rs.bg, means3D, colors_precomp, opacities, scales, rotations, rs.scale_modifier, cov3Ds_precomp,
                rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width, sh,
                rs.sh_degree, rs.campos, rs.prefiltered, rs.debug)
        num_rendered, color, radii, geom, binning, img = _call_native(
            _C.rasterize_gaussians, args, rs.debug, "snapshot_fw.dump", "forward")
        ctx.raster_settings = rs
        ctx.num_rendered = num_rendered
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geom, binning,
                              img)
        ctx.mark_non_differentiable(radii)
        return color, radii

    @staticmethod
    def backward(ctx, grad_out_color, _grad_radii):
        rs = ctx.raster_settings
        colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geom, binning, img = ctx.saved_tensors
        args = (rs.bg, means3D, radii, colors_precomp, scales, rotations, rs.scale_modifier, cov3Ds_precomp,
                rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, grad_out_color, sh, rs.sh_degree, rs.campos,
                geom, ctx.num_rendered, binning, img, rs.debug)
        sink = _sh_grad_sink
        if sink is not None and sh.numel() > 0 and colors_precomp.numel() == 0 and sink.accepts(sh, means3D):
            rec = sink.record(means3D.size(0))
            # the record's exchange starts as soon as the colour gradient is queued,
            # under the per-Gaussian backward
            push = lambda: sink.push(rec, rs.campos, rs.sh_degree)  # noqa: E731
            (d_means2D, d_colors, d_opacities, d_means3D, d_cov3D, d_sh, d_scales, d_rotations) = _call_native(
                lambda *a: _C.rasterize_gaussians_backward(*a, drgb_out=rec[4:], on_drgb=push), args, rs.debug,
                "snapshot_bw.dump", "backward")
        else:
            # dsh as the [P,M,3] view of coefficient planes: the reference's SH cat
            # backward (get_features) then slices an f_dc gradient that already has
            # _features_dc's layout, and AccumulateGrad keeps it without a copy
            (d_means2D, d_colors, d_opacities, d_means3D, d_cov3D, d_sh, d_scales, d_rotations) = _call_native(
                lambda *a: _C.rasterize_gaussians_backward(*a, dsh_planar=True), args, rs.debug, "snapshot_bw.dump",
                "backward")
        return (d_means3D, d_means2D, d_sh, d_colors, d_opacities, d_scales, d_rotations, d_cov3D, None)


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings)


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool


def _empty_like_device(ref: torch.Tensor) -> torch.Tensor:
    return torch.empty(0, dtype=torch.float32, device=ref.device)


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings: GaussianRasterizationSettings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions: torch.Tensor) -> torch.Tensor:
        """Frustum (near-plane) test per point: view-space z > 0.2."""
        with torch.no_grad():
            rs = self.raster_settings
            return _C.mark_visible(positions, rs.viewmatrix, rs.projmatrix)

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None):
        if (shs is None) == (colors_precomp is None):
            raise Exception("Please provide excatly one of either SHs or precomputed colors!")
        have_sr = scales is not None or rotations is not None
        if ((scales is None or rotations is None) and cov3D_precomp is None) or (have_sr and cov3D_precomp is not None):
            raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
        empty = _empty_like_device(means3D)
        shs = empty if shs is None else shs
        colors_precomp = empty if colors_precomp is None else colors_precomp
        scales = empty if scales is None else scales
        rotations = empty if rotations is None else rotations
        cov3D_precomp = empty if cov3D_precomp is None else cov3D_precomp
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp,
                                   self.raster_settings)
