"""CPU oracle for the differentiable Gaussian rasterizer — TEST INFRASTRUCTURE ONLY.

This module wraps ``liboracle.so`` (``gsr_oracle.c``, a plain-C restatement of the
upstream ``diff-gaussian-rasterization`` algorithm that the reference calls at
``gaussian_renderer/__init__.py:98-106``) with numpy.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it;
the product path (``3dgs_study_amd/diff_gaussian_rasterization``) never does.

Parity status (see gsr_oracle.c header and DESIGN.md §Oracle): the CUDA original
is not in the snapshot (empty git submodule), so the oracle is pinned by golden
vectors captured from the reference's own Python (eval_sh, cov3D, camera
matrices), by float64 autograd of the same forward, and by analytic KATs.

The orchestration mirrors upstream ``Rasterizer::forward`` / ``Rasterizer::backward``
(``cuda_rasterizer/rasterizer_impl.cu``): preprocess ->
inclusive scan -> duplicateWithKeys -> stable sort -> identifyTileRanges -> render;
backward: render-backward -> computeCov2D-backward -> preprocess-backward.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB_PATH = _HERE / "liboracle.so"
_LIB_MT_PATH = _HERE / "liboracle_mt.so"  # same source with OpenMP (bench.py's CPU baseline)
_libs = {}

BLOCK_X = 16
BLOCK_Y = 16


def build() -> Path:
    """Compile liboracle.so and liboracle_mt.so with the committed Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)
    return _LIB_PATH


def _load(mt: bool = False):
    """The single-threaded checker library, or (mt) its OpenMP build."""
    if mt not in _libs:
        path = _LIB_MT_PATH if mt else _LIB_PATH
        if not path.exists():
            build()
        lib = ctypes.CDLL(str(path))
        lib.oracle_inclusive_scan.restype = ctypes.c_int64
        lib.oracle_preprocess.restype = ctypes.c_int
        lib.oracle_num_threads.restype = ctypes.c_int
        _libs[mt] = lib
    return _libs[mt]


def num_threads(mt: bool = True) -> int:
    """Threads the (mt) library's parallel loops use (OMP_NUM_THREADS)."""
    return int(_load(mt).oracle_num_threads())


def _p(a):
    """ctypes pointer to a C-contiguous numpy array, or NULL for None."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "oracle arrays must be contiguous"
    return ctypes.c_void_p(a.ctypes.data)


def _f32(a):
    if a is None:
        return None
    a = np.asarray(a, dtype=np.float32)
    if a.size == 0:
        return None
    return np.ascontiguousarray(a)


def forward(means3D, opacities, viewmatrix, projmatrix, campos, bg, image_height, image_width, tanfovx, tanfovy,
            scale_modifier=1.0, sh_degree=0, shs=None, colors_precomp=None, scales=None, rotations=None,
            cov3D_precomp=None, prefiltered=False, mt=False):
    """Full forward. All array inputs are numpy (or array-likes); matrices are the
    16-float row-major storage of the reference's transposed matrices.  mt: the
    OpenMP build (same results)."""
    lib = _load(mt)
    means3D = _f32(means3D).reshape(-1, 3)
    P = means3D.shape[0]
    H, W = int(image_height), int(image_width)
    opacities = _f32(opacities).reshape(P)
    shs = _f32(shs)
    colors_precomp = _f32(colors_precomp)
    scales = _f32(scales)
    rotations = _f32(rotations)
    cov3D_precomp = _f32(cov3D_precomp)
    viewmatrix = _f32(viewmatrix).reshape(16)
    projmatrix = _f32(projmatrix).reshape(16)
    campos = _f32(campos).reshape(3)
    bg = _f32(bg).reshape(3)
    if (shs is None) == (colors_precomp is None):
        raise ValueError("Please provide excatly one of either SHs or precomputed colors!")
    if ((scales is None) or (rotations is None)) == (cov3D_precomp is None):
        raise ValueError("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
    M = 0
    if shs is not None:
        shs = shs.reshape(P, -1, 3)
        M = shs.shape[1]
    gx = (W + BLOCK_X - 1) // BLOCK_X
    gy = (H + BLOCK_Y - 1) // BLOCK_Y
    T = gx * gy

    radii = np.zeros(P, np.int32)
    means2D = np.zeros((P, 2), np.float32)
    depths = np.zeros(P, np.float32)
    cov3Ds = np.zeros((P, 6), np.float32)
    rgb = np.zeros((P, 3), np.float32)
    conic_opacity = np.zeros((P, 4), np.float32)
    tiles_touched = np.zeros(P, np.uint32)
    rects = np.zeros((P, 4), np.int32)
    clamped = np.zeros((P, 3), np.uint8)
    bad = lib.oracle_preprocess(
        ctypes.c_int(P), ctypes.c_int(int(sh_degree)), ctypes.c_int(M), _p(means3D), _p(scales),
        ctypes.c_float(scale_modifier), _p(rotations), _p(opacities), _p(shs), _p(clamped), _p(cov3D_precomp),
        _p(colors_precomp), _p(viewmatrix), _p(projmatrix), _p(campos), ctypes.c_int(W), ctypes.c_int(H),
        ctypes.c_float(tanfovx), ctypes.c_float(tanfovy), _p(radii), _p(means2D), _p(depths), _p(cov3Ds), _p(rgb),
        _p(conic_opacity), _p(tiles_touched), _p(rects), ctypes.c_int(1 if prefiltered else 0))
    if bad:
        raise RuntimeError("Point is filtered although prefiltered is set. This shouldn't happen!")
    point_offsets = np.zeros(P, np.uint32)
    num_rendered = int(lib.oracle_inclusive_scan(ctypes.c_int(P), _p(tiles_touched), _p(point_offsets)))
    n = max(num_rendered, 1)
    keys_unsorted = np.zeros(n, np.uint64)
    values_unsorted = np.zeros(n, np.uint32)
    lib.oracle_duplicate_with_keys(ctypes.c_int(P), _p(means2D), _p(depths), _p(point_offsets), _p(radii),
                                   ctypes.c_int(W), ctypes.c_int(H), _p(keys_unsorted), _p(values_unsorted))
    keys = np.zeros(n, np.uint64)
    point_list = np.zeros(n, np.uint32)
    lib.oracle_sort_pairs(ctypes.c_int64(num_rendered), _p(keys_unsorted), _p(values_unsorted), _p(keys),
                          _p(point_list))
    ranges = np.zeros((T, 2), np.uint32)
    lib.oracle_identify_tile_ranges(ctypes.c_int64(num_rendered), _p(keys), ctypes.c_int(T), _p(ranges))
    colors = colors_precomp.reshape(P, 3) if colors_precomp is not None else rgb
    colors = np.ascontiguousarray(colors, dtype=np.float32)
    final_T = np.zeros((H, W), np.float32)
    n_contrib = np.zeros((H, W), np.uint32)
    color = np.zeros((3, H, W), np.float32)
    lib.oracle_render_forward(_p(ranges), _p(point_list), ctypes.c_int(W), ctypes.c_int(H), _p(means2D),
                              _p(colors), _p(conic_opacity), _p(final_T), _p(n_contrib), _p(bg), _p(color))
    return dict(color=color, radii=radii, num_rendered=num_rendered, means2D=means2D, depths=depths,
                cov3Ds=cov3Ds if cov3D_precomp is None else cov3D_precomp.reshape(P, 6), rgb=rgb,
                conic_opacity=conic_opacity, tiles_touched=tiles_touched, rects=rects, clamped=clamped,
                point_offsets=point_offsets, keys_unsorted=keys_unsorted[:num_rendered],
                values_unsorted=values_unsorted[:num_rendered], keys=keys[:num_rendered],
                point_list=point_list[:num_rendered], ranges=ranges, final_T=final_T, n_contrib=n_contrib,
                # inputs kept for backward
                _in=dict(means3D=means3D, shs=shs, colors_precomp=colors_precomp, scales=scales, rotations=rotations,
                         cov3D_precomp=cov3D_precomp, viewmatrix=viewmatrix, projmatrix=projmatrix, campos=campos,
                         bg=bg, W=W, H=H, tanfovx=float(tanfovx), tanfovy=float(tanfovy),
                         scale_modifier=float(scale_modifier), sh_degree=int(sh_degree), M=M, colors=colors,
                         point_list_full=point_list, mt=mt))


def backward(state, dL_dout_color):
    """Full backward from the forward state; returns the 8 native gradients of
    ``_C.rasterize_gaussians_backward`` plus dL/dconic."""
    inp = state["_in"]
    lib = _load(inp.get("mt", False))
    P = inp["means3D"].shape[0]
    W, H, M = inp["W"], inp["H"], inp["M"]
    g = np.ascontiguousarray(np.asarray(dL_dout_color, np.float32).reshape(3, H, W))
    dmean2D = np.zeros((P, 3), np.float32)
    dconic = np.zeros((P, 4), np.float32)
    dopacity = np.zeros((P, 1), np.float32)
    dcolors = np.zeros((P, 3), np.float32)
    lib.oracle_render_backward_p(ctypes.c_int(P), _p(state["ranges"]), _p(inp["point_list_full"]), ctypes.c_int(W),
                               ctypes.c_int(H),
                               _p(inp["bg"]), _p(state["means2D"]), _p(state["conic_opacity"]), _p(inp["colors"]),
                               _p(state["final_T"]), _p(state["n_contrib"]), _p(g), _p(dmean2D), _p(dconic),
                               _p(dopacity), _p(dcolors))
    # rasterizer_impl.cu computes focal in float: H / (2.0f * tan_fovy)
    focal_y = float(np.float32(H) / (np.float32(2.0) * np.float32(inp["tanfovy"])))
    focal_x = float(np.float32(W) / (np.float32(2.0) * np.float32(inp["tanfovx"])))
    dmeans3D = np.zeros((P, 3), np.float32)
    dcov3D = np.zeros((P, 6), np.float32)
    cov3Ds = np.ascontiguousarray(state["cov3Ds"], np.float32)
    lib.oracle_cov2d_backward(ctypes.c_int(P), _p(inp["means3D"]), _p(state["radii"]), _p(cov3Ds),
                              ctypes.c_float(focal_x), ctypes.c_float(focal_y), ctypes.c_float(inp["tanfovx"]),
                              ctypes.c_float(inp["tanfovy"]), _p(inp["viewmatrix"]), _p(dconic), _p(dmeans3D),
                              _p(dcov3D))
    dsh = np.zeros((P, max(M, 0), 3), np.float32)
    dscales = np.zeros((P, 3), np.float32)
    drot = np.zeros((P, 4), np.float32)
    lib.oracle_preprocess_backward(
        ctypes.c_int(P), ctypes.c_int(inp["sh_degree"]), ctypes.c_int(M), _p(inp["means3D"]), _p(state["radii"]),
        _p(inp["shs"]), _p(state["clamped"]), _p(inp["scales"]), _p(inp["rotations"]),
        ctypes.c_float(inp["scale_modifier"]), _p(inp["projmatrix"]), _p(inp["campos"]), _p(dmean2D), _p(dmeans3D),
        _p(dcolors), _p(dcov3D), _p(dsh) if M > 0 else None, _p(dscales), _p(drot))
    return dict(dmeans2D=dmean2D, dcolors=dcolors, dopacity=dopacity, dmeans3D=dmeans3D, dcov3D=dcov3D, dsh=dsh,
                dscales=dscales, drot=drot, dconic=dconic)


def mark_visible(means3D, viewmatrix):
    lib = _load()
    means3D = _f32(means3D).reshape(-1, 3)
    out = np.zeros(means3D.shape[0], np.uint8)
    lib.oracle_mark_visible(ctypes.c_int(means3D.shape[0]), _p(means3D), _p(_f32(viewmatrix).reshape(16)), _p(out))
    return out.astype(bool)


def sh_to_rgb(means, campos, shs, deg):
    """forward.cu computeColorFromSH on its own: rgb [P,3] (clamped at 0), clamped [P,3]."""
    lib = _load()
    means = _f32(means).reshape(-1, 3)
    P = means.shape[0]
    shs = _f32(shs).reshape(P, -1, 3)
    rgb = np.zeros((P, 3), np.float32)
    clamped = np.zeros((P, 3), np.uint8)
    lib.oracle_sh_to_rgb(ctypes.c_int(P), ctypes.c_int(deg), ctypes.c_int(shs.shape[1]), _p(means),
                         _p(_f32(campos).reshape(3)), _p(shs), _p(clamped), _p(rgb))
    return rgb, clamped.astype(bool)


def sh_grad_sum(means, campos, degs, drgb, M):
    """Sum over views of backward.cu computeColorFromSH's dL/dsh for clamp-masked
    colour gradients (the view-parallel SH exchange's contract, multiview.py):
    campos [V,3], degs [V], drgb [V,P,3] -> dsh [P,M,3], added in view order."""
    lib = _load()
    means = _f32(means).reshape(-1, 3)
    P = means.shape[0]
    campos = _f32(campos).reshape(-1, 3)
    V = campos.shape[0]
    degs = np.ascontiguousarray(np.asarray(degs, np.int32).reshape(V))
    drgb = _f32(drgb).reshape(V, P, 3)
    out = np.zeros((P, M, 3), np.float32)
    lib.oracle_sh_grad_sum(ctypes.c_int(P), ctypes.c_int(V), ctypes.c_int(M), _p(means), _p(campos), _p(degs),
                           _p(drgb), _p(out))
    return out


def cov3d(scales, scale_modifier, rotations):
    """forward.cu computeCov3D on its own: [P,6] upper triangle."""
    lib = _load()
    scales = _f32(scales).reshape(-1, 3)
    P = scales.shape[0]
    out = np.zeros((P, 6), np.float32)
    lib.oracle_cov3d(ctypes.c_int(P), _p(scales), ctypes.c_float(scale_modifier), _p(_f32(rotations).reshape(P, 4)),
                     _p(out))
    return out


def activation_leaf_grads(dsh, dopacity, dscales, drot, opacities, scales, rotations, rotation_norm,
                          rotation_eps=1e-12, sum_order="pairwise"):
    """Leaf gradients of the reference's activations (scene/gaussian_model.py:106-126)
    from the rasterizer's activation gradients, in float32 with torch autograd's
    operation order — what gsr_leaf_grads asks the library for (include/gsr.h):
    get_features' cat -> the two slices of dsh; exp(_scaling) -> dscales * scales;
    sigmoid(_opacity) -> (dopacity * (1 - o)) * o; F.normalize(_rotation) -> the
    Div / Expand (sum) / ClampMin / LinalgVectorNorm backwards, summed, written
    with the quotient q = rotations torch produced for every x / n it divides
    (rotation_norm: the norms torch computed).  numpy
    float32 scalar ops round like the kernel (no contraction).  ``sum_order``: how
    the normalize backward's 4-term sum (ExpandBackward0) is added — "pairwise"
    ((a + b) + (c + d)) as torch's GPU reduction and the library do, "sequential"
    as torch's CPU reduction does."""
    f = np.float32
    out = {"dsh_dc": dsh[:, :1].copy(), "dsh_rest": dsh[:, 1:].copy(),
           "dscaling": (dscales.astype(f) * scales.astype(f)).astype(f),
           "dopacity": ((dopacity.astype(f) * (f(1) - opacities.astype(f))) * opacities.astype(f)).astype(f)}
    g, q = drot.astype(f), rotations.astype(f)
    nr = rotation_norm.reshape(-1, 1).astype(f)
    eps = f(rotation_eps)
    n = np.where(np.isnan(nr), nr, np.maximum(nr, eps))
    og = -g * (q / n)
    if sum_order == "pairwise":
        s = (og[:, 0:1] + og[:, 1:2]) + (og[:, 2:3] + og[:, 3:4])
    else:
        s = ((og[:, 0:1] + og[:, 1:2]) + og[:, 2:3]) + og[:, 3:4]
    gm = np.where(nr >= eps, s, f(0))
    xn = np.where(nr == 0, f(0), q)
    out["drotation"] = (g / n + gm * xn).astype(f)
    return out
