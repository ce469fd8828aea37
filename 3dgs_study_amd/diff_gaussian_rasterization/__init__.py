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

View-parallel gradient exchange (not upstream; ``3dgs_study_amd/multiview.py``):
while an exchange is installed with ``set_grad_exchange`` (alias
``set_sh_grad_sink``), a backward with SH input may hand it the view's colour
gradient instead of returning dsh (the ``sh`` input then gets no gradient through
autograd; the exchange rebuilds the SH leaf gradients summed over all ranks'
views), and the fused leaf gradients below are written straight into the
exchange's all-reduce bucket.  ``set_grad_exchange(None)`` restores upstream
behaviour.

Tile footprint (not upstream; ``set_footprint``, env ``GSR_FOOTPRINT``): "rect"
(default) bins every tile of upstream's getRect rect, so ``num_rendered`` and the
binning buffer's lists are upstream's bit for bit; "tight" bins only the tiles
the alpha >= 1/255 ellipse reaches — the same image, radii and gradients from
shorter lists (of upstream's outputs only the ``num_rendered`` integer differs).
Binning form (``set_binning_mode``): "rowspan" (default; row spans sorted by tile
row, then their tiles by column) or "lsd" (a radix sort by tile index); both give
upstream's lists.

Debug mode (``raster_settings.debug``): the native side synchronises after every
kernel; on failure a CPU copy of the arguments is written to
``snapshot_fw.dump`` / ``snapshot_bw.dump`` before the exception propagates.
"""
from __future__ import annotations

import os
from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C

from ._C import get_binning_mode, get_footprint, set_binning_mode, set_footprint  # noqa: E402

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "rasterize_model",
           "set_sh_grad_sink",
           "set_grad_exchange", "set_footprint", "get_footprint", "set_binning_mode", "get_binning_mode",
           "set_fused_leaf_grads"]

_exchange = None
# None = automatic (on, except in a multi-rank process group with no exchange of
# ours installed: DDP's reducer hooks AccumulateGrad nodes from C++, where the plan
# cannot see them); True / False = forced (env GSR_FUSED_LEAF_GRADS=1 / 0)
_fused_leaf_grads = {"0": False, "1": True}.get(os.environ.get("GSR_FUSED_LEAF_GRADS", ""))
last_leaf_plan = ()  # the inputs whose leaf gradients the last backward wrote itself


def set_fused_leaf_grads(on) -> object:
    """Writing the leaf gradients of the caller's activations from the rasterizer
    backward (see ``_leaf_plan``): True / False forces it on / off, None (the
    default) = on unless torch.distributed runs more than one rank without an
    exchange of this package installed (a DDP-wrapped model: its reducer's
    AccumulateGrad hooks are invisible here).  Returns the previous setting."""
    global _fused_leaf_grads
    prev, _fused_leaf_grads = _fused_leaf_grads, (None if on is None else bool(on))
    return prev


def _fusion_on(ex) -> bool:
    if _fused_leaf_grads is not None:
        return _fused_leaf_grads
    if ex is not None:
        return True
    try:
        import torch.distributed as dist

        return not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1)
    except (ImportError, RuntimeError, ValueError):
        return True


# ---------------------------------------------------------------- fused leaf gradients
# The reference hands the rasterizer activations of GaussianModel's leaves
# (scene/gaussian_model.py:106-126): shs = cat(_features_dc, _features_rest, dim=1),
# scales = exp(_scaling), opacities = sigmoid(_opacity), rotations =
# F.normalize(_rotation).  Upstream's backward returns the activation gradients and
# torch then runs the cat's slice copies (a 192 MB transposing copy for f_rest at
# 1M Gaussians, SH3), the exp / sigmoid / normalize backwards (~20 small kernels)
# and AccumulateGrad.  When the autograd graph is exactly that — checked node by
# node at backward time — the library writes each leaf's gradient itself, with
# torch's operation order (bit-identical results), and the Function returns None
# for that input, so torch skips the activation's backward.  Anything else keeps
# upstream's path for that input: another graph shape, hooks on the activation or
# the leaf (tensor hooks, retain_grad, post-accumulate hooks other than the
# installed exchange's own), create_graph, autograd.grad / backward(inputs=...)
# not accumulating into the leaf, or an existing .grad that is not a dense
# contiguous float32 tensor.  Hooks registered directly on an AccumulateGrad node
# are invisible from Python (DDP's): _fusion_on turns the path off by itself in a
# multi-rank group without our exchange, and set_fused_leaf_grads(False) always.
# With an exchange that offers an all-reduce bucket (multiview.GradAllReduce at
# N > 1) the means3D input — the _xyz leaf itself — joins the plan, and every
# planned gradient is written into the bucket, whose single all-reduce the
# exchange starts when the backward ends.
def _acc_leaf(node):
    return node.variable if node is not None and type(node).__name__ == "AccumulateGrad" else None


def _leaf_state(leaf, shape, device, ex=None):
    """-1: not fusable; 0: no .grad yet (write it); 1: add into the existing .grad."""
    if (leaf is None or not leaf.is_leaf or not leaf.requires_grad or leaf.dtype is not torch.float32
            or leaf.device != device or leaf.shape != shape or not leaf.is_contiguous() or leaf._backward_hooks):
        return -1
    owns = getattr(ex, "owns_hooks", None)  # (a round-1 sink has no bucket protocol)
    if getattr(leaf, "_post_accumulate_grad_hooks", None) and not (owns is not None and owns(leaf)):
        return -1
    g = leaf.grad
    if g is None:
        return 0
    if (g.layout != torch.strided or g.dtype is not torch.float32 or g.device != device
            or g.shape != shape or not g.is_contiguous() or g.requires_grad):
        return -1
    return 1


def _plain_activation(t) -> bool:
    return not t._backward_hooks and not t.retains_grad


def _will_run(node) -> bool:
    try:  # raises inside autograd.grad for leaf nodes: not an accumulating backward
        return bool(torch._C._will_engine_execute_node(node))
    except Exception:
        return False


def _leaf_plan(ctx, needs, sh, colors_precomp, opacities, scales, rotations, means3D, sink_takes_sh, ex):
    """{name: (leaf tensors, state, extras, bucket views or None)} for the inputs
    whose leaf gradients the backward may write itself (see above); called inside
    backward.  ``needs``: needs_input_grad in _RasterizeGaussians' input order;
    ``ctx.next_functions[0]`` is means3D's."""
    if torch.is_grad_enabled():  # create_graph: the activations' backwards must be recorded
        return {}
    plan = {}
    device = opacities.device
    P = opacities.shape[0]
    st = lambda leaf, shape: _leaf_state(leaf, shape, device, ex)  # noqa: E731
    try:
        if needs[2] and not sink_takes_sh and sh.numel() and colors_precomp.numel() == 0 and _plain_activation(sh):
            n = sh.grad_fn
            nf = n.next_functions if type(n).__name__ == "CatBackward0" else ()
            if len(nf) == 2 and n._saved_dim in (1, -2) and sh.dim() == 3 and sh.shape[2] == 3:
                M = sh.shape[1]
                dc, rest = _acc_leaf(nf[0][0]), _acc_leaf(nf[1][0])
                a, b = st(dc, (P, 1, 3)), st(rest, (P, M - 1, 3))
                if a >= 0 and a == b and _will_run(nf[0][0]) and _will_run(nf[1][0]):
                    plan["sh"] = ((dc, rest), a, None)
        if needs[5] and scales.numel() and _plain_activation(scales):
            n = scales.grad_fn
            if type(n).__name__ == "ExpBackward0" and n._saved_result.data_ptr() == scales.data_ptr():
                acc = n.next_functions[0][0]
                leaf = _acc_leaf(acc)
                s_ = st(leaf, (P, 3))
                if s_ >= 0 and _will_run(acc):
                    plan["scales"] = ((leaf,), s_, None)
        if needs[4] and opacities.numel() and _plain_activation(opacities):
            n = opacities.grad_fn
            if type(n).__name__ == "SigmoidBackward0" and n._saved_result.data_ptr() == opacities.data_ptr():
                acc = n.next_functions[0][0]
                leaf = _acc_leaf(acc)
                s_ = st(leaf, (P, 1))
                if s_ >= 0 and _will_run(acc):
                    plan["opacities"] = ((leaf,), s_, None)
        if needs[6] and rotations.numel() and _plain_activation(rotations):
            d = rotations.grad_fn
            df = d.next_functions if type(d).__name__ == "DivBackward0" else ()
            if len(df) == 2:
                acc, e = df[0][0], df[1][0]
                c = e.next_functions[0][0] if type(e).__name__ == "ExpandBackward0" else None
                nrm = c.next_functions[0][0] if type(c).__name__ == "ClampMinBackward0" else None
                if (type(nrm).__name__ == "LinalgVectorNormBackward0" and float(nrm._saved_ord) == 2.0
                        and tuple(nrm._saved_dim) in ((1,), (-1,)) and nrm._saved_keepdim
                        and nrm.next_functions[0][0] is acc):
                    leaf = _acc_leaf(acc)
                    s_ = st(leaf, (P, 4))
                    norm = nrm._saved_result
                    if (s_ >= 0 and norm.shape == (P, 1) and norm.dtype == torch.float32 and norm.device == device
                            and d._saved_self.data_ptr() == leaf.data_ptr() and _will_run(acc)):
                        plan["rotations"] = ((leaf,), s_, (norm.contiguous(), float(c._saved_min)))
        # means3D is the _xyz leaf itself (scene/gaussian_model.py:114-116): only worth
        # planning when its gradient can land in the exchange's bucket directly
        if ex is not None and needs[0] and means3D.is_leaf:
            acc = ctx.next_functions[0][0]
            s_ = st(means3D, (P, 3))
            if s_ >= 0 and _acc_leaf(acc) is means3D and _will_run(acc):
                plan["means3D"] = ((means3D,), s_, None)
    except (AttributeError, RuntimeError, TypeError):
        return {}
    bucket = getattr(ex, "leaf_bucket", None)  # (a round-1 sink offers no bucket)
    views = bucket({k: v[0] for k, v in plan.items()}) if bucket is not None and plan else {}
    if "means3D" not in views:
        plan.pop("means3D", None)
    return {k: (v[0], v[1], v[2], views.get(k)) for k, v in plan.items()}


def _leaf_outputs(plan):
    """The LeafGrads of a plan and the (leaf, tensor) pairs to install as .grad: a
    bucket view of the exchange, else the existing .grad where it accumulates,
    else a fresh tensor."""
    kw, fresh, acc = {}, [], 0

    def out(leaf, state, bit, view):
        nonlocal acc
        if state == 1:
            acc |= bit
            return leaf.grad if view is None else view
        t = torch.empty_like(leaf, memory_format=torch.contiguous_format) if view is None else view
        fresh.append((leaf, t))
        return t

    if "sh" in plan:
        (dc, rest), st, _, v = plan["sh"]
        v = v or (None, None)
        kw["dsh_dc"], kw["dsh_rest"] = out(dc, st, 1, v[0]), out(rest, st, 1, v[1])
    if "scales" in plan:
        (leaf,), st, _, v = plan["scales"]
        kw["dscaling"] = out(leaf, st, 2, v and v[0])
    if "opacities" in plan:
        (leaf,), st, _, v = plan["opacities"]
        kw["dopacity"] = out(leaf, st, 4, v and v[0])
    if "rotations" in plan:
        (leaf,), st, (norm, eps), v = plan["rotations"]
        kw["drotation"] = out(leaf, st, 8, v and v[0])
        kw["rotation_norm"], kw["rotation_eps"] = norm, eps
    if "means3D" in plan:
        (leaf,), st, _, v = plan["means3D"]
        kw["dmeans3D"] = out(leaf, st, 16, v[0])
    return _C.LeafGrads(accumulate=acc, **kw), fresh


def set_grad_exchange(ex):
    """Install (or with None remove) the view-parallel gradient exchange
    (multiview.GradAllReduce); returns the previous one.  The exchange provides
    ``accepts(sh, means3D) -> bool`` (True: it takes this backward's SH gradient as
    the view's colour gradient), ``record(P, campos, sh_degree)`` (a float32 tensor
    of ``_C.sh_record_floats(P)`` elements, its [campos, degree] header written) and
    ``push(record, campos, sh_degree, ready)`` for that (``ready``: an event after
    which the record's colour gradient is written); ``owns_hooks(leaf) -> bool`` (the leaf's post-accumulate hooks are its own,
    so the fused path may write that leaf's gradient) and
    ``leaf_bucket({name: leaves}) -> {name: views}`` (where the fused leaf gradients
    go: views of its all-reduce bucket, for the names it can take)."""
    global _exchange
    prev, _exchange = _exchange, ex
    return prev


set_sh_grad_sink = set_grad_exchange  # the round-1 name


def _drgb_hooks(ex, rec, rs) -> dict:
    """The backward's keywords that hand the view's colour-gradient record to the
    exchange: with ``colours_apart`` the exchange queues the colour kernel itself (on
    its own stream, beside the per-Gaussian backward) and then its all-gather
    (``push(..., write=)``); otherwise the gather starts after the library wrote it."""
    if getattr(ex, "colours_apart", False):
        return {"drgb_apart": True,
                "on_drgb": lambda write: ex.push(rec, rs.campos, rs.sh_degree, write=write)}
    return {"on_drgb": lambda ready: ex.push(rec, rs.campos, rs.sh_degree, ready)}


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


# the forward's validated inputs (_C._rasterize), by name: where each comes from
_INPUT_SRC = ("background", "means3D", "colors", "opacity", "scales", "rotations", "cov3D_precomp", "viewmatrix",
              "projmatrix", "sh", "campos", "sh_rest")


def _input_sources(rs, means3D, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, sh, sh_rest=None):
    return dict(zip(_INPUT_SRC, (rs.bg, means3D, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                                 rs.viewmatrix, rs.projmatrix, sh, rs.campos, sh_rest)))


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings, grad_on=True):
        rs = raster_settings
        args = (rs.bg, means3D, colors_precomp, opacities, scales, rotations, rs.scale_modifier, cov3Ds_precomp,
                rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width, sh,
                rs.sh_degree, rs.campos, rs.prefiltered, rs.debug)
        # a backward may follow: the forward zeroes its accumulator beside the blend
        # (needs_input_grad is set under no_grad too: the caller's grad mode decides)
        prep = grad_on and any(ctx.needs_input_grad[:8])
        num_rendered, color, radii, geom, binning, img, vin = _call_native(
            lambda *a: _C._rasterize(*a, prepare_backward=prep), args, rs.debug, "snapshot_fw.dump", "forward")
        ctx.raster_settings = rs
        ctx.num_rendered = num_rendered
        # The backward reuses the forward's validated inputs (the C struct).  The
        # tensors it points at stay alive through save_for_backward (the inputs) and
        # the raster settings (camera, background), as upstream; only contiguous
        # copies the forward had to make are saved besides, so nothing outlives the
        # backward (the saved tensors are freed after it unless the graph is
        # retained), and an in-place change of a saved input raises.
        copies = {}
        ctx.inputs = None
        if vin is not None:
            s, keep, device, M = vin
            src = _input_sources(rs, means3D, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, sh)
            copies = {k: t for k, t in keep.items() if t is not None and t is not src[k]}
            ctx.inputs = (s, device, M, frozenset(k for k, t in keep.items() if t is not None), tuple(copies))
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geom, binning,
                              img, opacities, *copies.values())
        ctx.mark_non_differentiable(radii)
        # radii never carry a gradient: no zero int32 [P] tensor materialised per backward
        ctx.set_materialize_grads(False)
        return color, radii

    @staticmethod
    def backward(ctx, grad_out_color, _grad_radii):
        rs = ctx.raster_settings
        saved = ctx.saved_tensors
        if grad_out_color is None:  # the image was not used (set_materialize_grads(False))
            grad_out_color = torch.zeros((3, rs.image_height, rs.image_width), dtype=torch.float32,
                                         device=saved[1].device)
        colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geom, binning, img, opacities = saved[:11]
        inputs = None
        if ctx.inputs is not None:
            s, device, M, present, copy_names = ctx.inputs
            src = _input_sources(rs, means3D, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, sh)
            src.update(zip(copy_names, saved[11:]))
            inputs = (s, {k: (src[k] if k in present else None) for k in _INPUT_SRC}, device, M)
        args = (rs.bg, means3D, radii, colors_precomp, scales, rotations, rs.scale_modifier, cov3Ds_precomp,
                rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, grad_out_color, sh, rs.sh_degree, rs.campos,
                geom, ctx.num_rendered, binning, img, rs.debug)
        ex = _exchange
        sink_takes_sh = (ex is not None and sh.numel() > 0 and colors_precomp.numel() == 0
                         and ex.accepts(sh, means3D))
        plan = (_leaf_plan(ctx, ctx.needs_input_grad, sh, colors_precomp, opacities, scales, rotations, means3D,
                           sink_takes_sh, ex)
                if _fusion_on(ex) and means3D.size(0) > 0 else {})
        global last_leaf_plan
        last_leaf_plan = tuple(sorted(plan))
        kw = dict(opacities=opacities, inputs=inputs)
        if plan:
            leaf, fresh = _leaf_outputs(plan)
            kw["leaf"] = leaf
        if sink_takes_sh:
            rec = ex.record(means3D.size(0), rs.campos, rs.sh_degree)
            # the record's exchange starts right after the colour gradient is written,
            # under the per-Gaussian backward (an exchange that runs the colour kernel
            # on its own stream gets it as a function: colours_apart)
            kw["drgb_out"] = rec[4:]
            kw.update(_drgb_hooks(ex, rec, rs))
        else:
            # a dsh that autograd receives is the [P,M,3] view of coefficient planes:
            # the reference's SH cat backward (get_features) then slices an f_dc
            # gradient that already has _features_dc's layout, and AccumulateGrad
            # keeps it without a copy
            kw["dsh_planar"] = True
        (d_means2D, d_colors, d_opacities, d_means3D, d_cov3D, d_sh, d_scales, d_rotations) = _call_native(
            lambda *a: _C.rasterize_gaussians_backward(*a, **kw), args, rs.debug, "snapshot_bw.dump", "backward")
        if plan:
            views = {k: v[3] for k, v in plan.items() if v[3] is not None}
            # the exchange may start right away; when it does, the bucket is its own
            # and the leaves get their .grad back from it (multiview.GradAllReduce)
            took = views and ex is not None and hasattr(ex, "rasterizer_done") and ex.rasterizer_done(views)
            for p, g in fresh:
                if not (took and any(g is v for vs in views.values() for v in vs)):
                    p.grad = g
        return (d_means3D, d_means2D, d_sh, d_colors, d_opacities, d_scales, d_rotations, d_cov3D, None, None)


class _RasterizeModel(torch.autograd.Function):
    """The rasterizer over GaussianModel's stored parameters (not upstream; see
    ``rasterize_model``): the library applies the activations and reads the SH from
    the two leaves, and its backward writes the stored parameters' gradients."""

    @staticmethod
    def forward(ctx, means3D, means2D, features_dc, features_rest, opacity, scaling, rotation, raster_settings,
                grad_on=True, l1_target=None):
        rs = raster_settings
        empty = _empty_like_device(means3D)
        rest = features_rest if features_rest.numel() else None
        args = (rs.bg, means3D, empty, opacity, scaling, rotation, rs.scale_modifier, empty, rs.viewmatrix,
                rs.projmatrix, rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width, features_dc, rs.sh_degree,
                rs.campos, rs.prefiltered, rs.debug)
        prep = grad_on and any(ctx.needs_input_grad[:7])
        # l1_target: the L1 loss mean|color - target| as a third output — its partial
        # sums in the same launch as the backward's preparation (gsr_forward_render_l1),
        # its image gradient formed inside the render backward (GSR_FLAG_L1_SEED)
        fwd_l1 = l1_target is not None and os.environ.get("GSR_FWD_L1", "1") != "0"  # (A/B switch)
        res = _call_native(
            lambda *a: _C._rasterize(*a, prepare_backward=prep, sh_rest=rest, activations=_C.ACT_ALL,
                                     l1_target=l1_target if fwd_l1 else None), args, rs.debug,
            "snapshot_fw.dump", "forward")
        num_rendered, color, radii, geom, binning, img, (s, keep, device, M) = res[:7]
        ctx.raster_settings = rs
        ctx.num_rendered = num_rendered
        src = _input_sources(rs, means3D, None, opacity, scaling, rotation, None, features_dc, rest)
        copies = {k: t for k, t in keep.items() if t is not None and t is not src[k]}
        ctx.inputs = (s, device, M, frozenset(k for k, t in keep.items() if t is not None), tuple(copies))
        l1 = l1_target is not None
        ctx.l1 = l1
        loss = (res[7] if fwd_l1 else _C.l1_loss(color, l1_target)) if l1 else None
        visible = (res[8] if fwd_l1 else radii > 0) if l1 else None
        ctx.save_for_backward(means3D, features_dc, features_rest, opacity, scaling, rotation, radii, geom, binning,
                              img, *copies.values(), *((color, l1_target) if l1 else ()))
        ctx.mark_non_differentiable(radii)
        if l1:
            ctx.mark_non_differentiable(visible)
        # radii never carry a gradient: no zero int32 [P] tensor materialised per backward
        ctx.set_materialize_grads(False)
        return (color, radii, loss, visible) if l1 else (color, radii)

    @staticmethod
    def backward(ctx, grad_out_color, _grad_radii, grad_loss=None, _grad_visible=None):
        rs = ctx.raster_settings
        saved = ctx.saved_tensors
        s, device, M, present, copy_names = ctx.inputs
        nc = 10 + len(copy_names)
        seed = None
        if ctx.l1 and grad_loss is not None:
            color, gt = saved[nc:nc + 2]
            if grad_out_color is None:  # the image only feeds the loss: no gradient map at all
                seed = (color, gt, grad_loss)
            else:
                grad_out_color = grad_out_color + _C.l1_grad(color, gt, grad_loss)
        if grad_out_color is None and seed is None:  # the image was not used (set_materialize_grads(False))
            grad_out_color = torch.zeros((3, rs.image_height, rs.image_width), dtype=torch.float32,
                                         device=saved[1].device)
        means3D, f_dc, f_rest, opacity, scaling, rotation, radii, geom, binning, img = saved[:10]
        rest = f_rest if f_rest.numel() else None
        src = _input_sources(rs, means3D, None, opacity, scaling, rotation, None, f_dc, rest)
        src.update(zip(copy_names, saved[10:nc]))
        inputs = (s, {k: (src[k] if k in present else None) for k in _INPUT_SRC}, device, M)
        needs = ctx.needs_input_grad
        ex = _exchange
        # the view-parallel exchange takes the SH gradient as the view's colour
        # gradient, and the all-reduced gradients land in its bucket where it offers one
        sink_takes_sh = (ex is not None and (needs[2] or needs[3])
                         and ex.accepts((f_dc, f_rest), means3D))
        views = {}
        bucket = getattr(ex, "leaf_bucket", None)  # (a round-1 sink offers no bucket)
        if bucket is not None and not torch.is_grad_enabled():
            # only leaves nothing else observes go to the bucket (the written view is
            # their .grad and autograd never sees the gradient): no tensor hooks,
            # retain_grad or post-accumulate hooks but the exchange's own, and no
            # create_graph — the rest come back through autograd
            want = {k: (t,) for k, t, n in (("means3D", means3D, needs[0]), ("opacities", opacity, needs[4]),
                                            ("scales", scaling, needs[5]), ("rotations", rotation, needs[6]))
                    if n and _leaf_state(t, t.shape, device, ex) >= 0}
            views = bucket(want) if want else {}
        fresh, acc = [], 0

        def out(name, leaf, shape, bit):
            nonlocal acc
            v = views.get(name)
            if v is None:
                return torch.empty(shape, dtype=torch.float32, device=device)
            if leaf.grad is not None:  # a later backward of the step: add into the bucket view
                acc |= bit
            else:
                fresh.append((leaf, v[0]))
            return v[0]

        P = means3D.size(0)
        kw = {}
        if not sink_takes_sh and (needs[2] or needs[3]):
            kw["dsh_dc"] = torch.empty((P, 1, 3), dtype=torch.float32, device=device)
            kw["dsh_rest"] = torch.empty((P, M - 1, 3), dtype=torch.float32, device=device)
        kw["dopacity"] = out("opacities", opacity, (P, 1), 4)
        kw["dscaling"] = out("scales", scaling, (P, 3), 2)
        kw["drotation"] = out("rotations", rotation, (P, 4), 8)
        kw["dmeans3D"] = out("means3D", means3D, (P, 3), 16)
        leaf = _C.LeafGrads(accumulate=acc, **kw)
        bkw = dict(inputs=inputs, leaf=leaf, l1_seed=seed)
        if sink_takes_sh:
            rec = ex.record(P, rs.campos, rs.sh_degree)
            bkw["drgb_out"] = rec[4:]
            bkw.update(_drgb_hooks(ex, rec, rs))
        args = (rs.bg, means3D, radii, None, scaling, rotation, rs.scale_modifier, None, rs.viewmatrix, rs.projmatrix,
                rs.tanfovx, rs.tanfovy, grad_out_color, f_dc, rs.sh_degree, rs.campos, geom, ctx.num_rendered, binning,
                img, rs.debug)
        d_means2D = _call_native(lambda *a: _C.rasterize_gaussians_backward(*a, **bkw), args, rs.debug,
                                 "snapshot_bw.dump", "backward")[0]
        # the exchange may start right away; when it does, the bucket is its own and
        # the leaves get their .grad back from it (multiview.GradAllReduce)
        took = views and hasattr(ex, "rasterizer_done") and ex.rasterizer_done(views)
        if not took:
            for p, g in fresh:
                p.grad = g
        global last_leaf_plan
        last_leaf_plan = tuple(sorted(["means3D", "opacities", "rotations", "scales"] +
                                      ([] if sink_takes_sh else ["sh"])))
        bucketed = lambda name, g: None if name in views else g  # noqa: E731
        d_rest = kw.get("dsh_rest") if rest is not None else (
            torch.zeros_like(f_rest) if "dsh_rest" in kw else None)
        return (bucketed("means3D", kw["dmeans3D"]), d_means2D, kw.get("dsh_dc"), d_rest,
                bucketed("opacities", kw["dopacity"]), bucketed("scales", kw["dscaling"]),
                bucketed("rotations", kw["drotation"]), None, None, None)


def rasterize_model(means3D, means2D, features_dc, features_rest, opacity, scaling, rotation, raster_settings,
                    l1_target=None):
    """The rasterizer over GaussianModel's stored parameters (not upstream).

    The reference renders with activations of the model's leaves
    (gaussian_renderer/__init__.py:81-96 -> scene/gaussian_model.py:107-126):
    ``shs = cat(_features_dc, _features_rest)`` (a 192 MB copy per view at 1M
    Gaussians, SH3), ``opacities = sigmoid(_opacity)``, ``scales = exp(_scaling)``,
    ``rotations = F.normalize(_rotation)``.  Here those leaves go in as they are: the
    library reads the SH rows from both tensors and applies the activations with
    torch's own operations in torch's order (include/gsr.h gsr_activations), so the
    image and radii equal ``rasterize_gaussians`` on the activations bit for bit,
    and the backward writes the leaves' gradients (through the activations'
    backwards) — the same values the reference's autograd produces, without the cat,
    the activation kernels, their backwards or the cat's slice copies.
    ``means2D`` is the screen-space gradient carrier, as upstream.
    ``l1_target`` (a [3,H,W] float32 image, or None): also return the L1 loss
    mean|image - target| (utils/loss_utils.py l1_loss, train.py:102) and render()'s
    ``visibility_filter`` (radii > 0, bool [P]) as a third and fourth output —
    both computed in the backward preparation's launch; when the image feeds nothing
    but that loss, the backward forms the loss's pixel gradient inside the render
    backward (no gradient map, no separate loss node or kernel).  Values equal
    ``l1_loss(image, target)``, ``radii > 0`` and the L1 backward."""
    return _RasterizeModel.apply(means3D, means2D, features_dc, features_rest, opacity, scaling, rotation,
                                 raster_settings, torch.is_grad_enabled(), l1_target)


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings, torch.is_grad_enabled())


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

    def forward_model(self, means3D, means2D, features_dc, features_rest, opacity, scaling, rotation,
                      l1_target=None):
        """``rasterize_model`` with these settings: GaussianModel's stored parameters
        (_xyz, _features_dc, _features_rest, _opacity, _scaling, _rotation) in place of
        the activations ``forward`` takes (``l1_target``: also the L1 loss)."""
        return rasterize_model(means3D, means2D, features_dc, features_rest, opacity, scaling, rotation,
                               self.raster_settings, l1_target)

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
