"""``_C`` — the native entry points of ``diff_gaussian_rasterization``, bound to the
C ABI of ``libgsr.so`` (``include/gsr.h``) with ctypes.

Upstream this module is a pybind11 extension (``ext.cpp`` + ``rasterize_points.cu``)
exporting ``rasterize_gaussians``, ``rasterize_gaussians_backward`` and ``mark_visible``
([UPSTREAM-SPEC]); the reference calls them through the autograd
wrapper in ``__init__.py`` from ``gaussian_renderer/__init__.py:98-106``.  This module
keeps those three names, their positional argument order, their return tuples and
their error behaviour, and does the work the C++ glue did upstream:

* ``.contiguous()`` on every input, ``torch.Tensor([])`` / empty -> NULL pointer,
  ``M = sh.size(1)`` when ``sh`` is non-empty;
* output and scratch allocation through torch's caching allocator (the library
  never allocates device memory): color [3,H,W] f32, radii [P] i32 and three
  uint8 scratch buffers whose sizes come from the library;
* the launches go to ``torch.cuda.current_stream()``.

There is no CPU path: the library must be present and the tensors must live on a
ROCm device, otherwise these functions raise.
"""
from __future__ import annotations

import ctypes
import math
import os
from pathlib import Path

import torch

_LIB_NAME = "libgsr.so"
_DEFAULT = Path(__file__).resolve().parent.parent / "lib" / _LIB_NAME


class GsrInputs(ctypes.Structure):
    """Mirror of ``struct gsr_inputs`` in include/gsr.h."""
    _fields_ = [
        ("P", ctypes.c_int32), ("D", ctypes.c_int32), ("M", ctypes.c_int32),
        ("W", ctypes.c_int32), ("H", ctypes.c_int32),
        ("tan_fovx", ctypes.c_float), ("tan_fovy", ctypes.c_float), ("scale_modifier", ctypes.c_float),
        ("prefiltered", ctypes.c_int32), ("debug", ctypes.c_int32),
        ("footprint", ctypes.c_int32), ("flags", ctypes.c_int32),
        ("bg", ctypes.c_void_p), ("means3D", ctypes.c_void_p), ("colors_precomp", ctypes.c_void_p),
        ("opacities", ctypes.c_void_p), ("scales", ctypes.c_void_p), ("rotations", ctypes.c_void_p),
        ("cov3D_precomp", ctypes.c_void_p), ("viewmatrix", ctypes.c_void_p), ("projmatrix", ctypes.c_void_p),
        ("sh", ctypes.c_void_p), ("campos", ctypes.c_void_p),
        ("sh_rest", ctypes.c_void_p), ("activations", ctypes.c_int32), ("reserved", ctypes.c_int32),
    ]


# gsr_activations (include/gsr.h): the inputs are GaussianModel's stored parameters
# and the library applies sigmoid / exp / F.normalize itself (bit-identical to torch)
ACT_OPACITY, ACT_SCALE, ACT_ROTATION = 1, 2, 4
ACT_ALL = ACT_OPACITY | ACT_SCALE | ACT_ROTATION


# every symbol include/gsr.h declares (checked by tests/test_abi.py)
EXPORTED = (
    "gsr_geom_bytes", "gsr_binning_bytes", "gsr_img_bytes", "gsr_accum_bytes",
    "gsr_forward_preprocess", "gsr_forward_render", "gsr_backward", "gsr_mark_visible",
    "gsr_geom_layout", "gsr_binning_layout", "gsr_img_layout", "gsr_last_error", "gsr_abi_version",
    "gsr_timing_enable", "gsr_timing_read", "gsr_stage_name",
    "gsr_l1_ssim_scratch_bytes", "gsr_l1_ssim", "gsr_adam_step", "gsr_densify_stats",
    "gsr_knn_scratch_bytes", "gsr_knn_mean_dist2",
    "gsr_backward_colors", "gsr_sh_record_floats", "gsr_sh_grad_from_colors", "gsr_backward_planar",
    "gsr_backward_colors_render", "gsr_backward_colors_finish", "gsr_point_list_keys", "gsr_backward_leaves",
    "gsr_build_id", "gsr_backward_phase", "gsr_timing_begin", "gsr_timing_end", "gsr_l1_grad",
    "gsr_forward_render_l1", "gsr_forward", "gsr_timing_sample", "gsr_binning_mode", "gsr_split_mode",
    "gsr_host_wait_us", "gsr_forward_status", "gsr_depth_passes_hint", "gsr_colour_mode",
)

# gsr_footprint (include/gsr.h): which bounding-rect tiles of a Gaussian are binned
FOOTPRINTS = {"rect": 0, "tight": 1}
# The package default is "rect" (DESIGN.md §2): upstream's getRect footprint, so
# num_rendered, point_list, ranges and n_contrib are upstream's bit for bit.
# GSR_FOOTPRINT=tight (or set_footprint("tight")) bins only the rect tiles the
# alpha >= 1/255 ellipse reaches: the same image, radii, final_T and gradients with
# shorter lists (num_rendered counts those).  (The C struct's zero value is RECT.)
_footprint = os.environ.get("GSR_FOOTPRINT", "rect")
if _footprint not in FOOTPRINTS:
    raise ImportError(f"GSR_FOOTPRINT={_footprint!r}: expected one of {sorted(FOOTPRINTS)}")


def set_footprint(mode: str) -> str:
    """Select the tile footprint of later forwards; returns the previous mode.

    "rect" (default): upstream's getRect footprint — num_rendered, the sorted keys,
    point_list, ranges and n_contrib are upstream's.  "tight": only the rect tiles the
    Gaussian's alpha >= 1/255 ellipse reaches (same image, radii and gradients, ~40 %
    fewer list entries at config C; num_rendered counts the shorter lists)."""
    global _footprint
    if mode not in FOOTPRINTS:
        raise ValueError(f"footprint must be one of {sorted(FOOTPRINTS)} (got {mode!r})")
    prev, _footprint = _footprint, mode
    return prev


def get_footprint() -> str:
    return _footprint


# gsr_binning_mode (include/gsr.h): how the (tile, Gaussian) lists are sorted.  Both
# forms give upstream's point_list and ranges bit for bit.
BINNING_MODES = {"rowspan": 0, "lsd": 1}


def set_binning_mode(mode: str) -> str:
    """Select the binning of later forwards; returns the previous mode.  "rowspan"
    (default): the footprints' row spans sorted by tile row, then their tiles by
    column (grids of at most 256 x 256 tiles; larger grids take the LSD sort);
    "lsd": an emission in depth order and a stable LSD radix sort by tile index."""
    if mode not in BINNING_MODES:
        raise ValueError(f"binning mode must be one of {sorted(BINNING_MODES)} (got {mode!r})")
    lib = load_library()
    prev = lib.gsr_binning_mode(BINNING_MODES[mode])
    if prev < 0:
        raise RuntimeError(lib.gsr_last_error().decode())
    return {v: k for k, v in BINNING_MODES.items()}[prev]


def get_binning_mode() -> str:
    return {v: k for k, v in BINNING_MODES.items()}[load_library().gsr_binning_mode(-1)]


def set_split(seg) -> int:
    """Split replay of long tile lists in the backward (include/gsr.h gsr_split_mode):
    -1 automatic (the default), 0 off, or a segment length in list entries.  Returns
    the previous setting; takes effect at the next forward."""
    prev = load_library().gsr_split_mode(int(seg))
    if prev < -1:
        raise ValueError(load_library().gsr_last_error().decode())
    return prev


def set_colour_apart(on: bool) -> bool:
    """Preprocess's colour half on a side stream beside the binning (include/gsr.h
    gsr_colour_mode; opt-in, measured slower) or one fused kernel (the default).
    Returns the previous setting."""
    return load_library().gsr_colour_mode(1 if on else 0) == 1


def get_colour_apart() -> bool:
    return load_library().gsr_colour_mode(-2) == 1


def set_colour_mode(mode: int) -> int:
    """Where preprocess's colour half runs (include/gsr.h gsr_colour_mode): 0 in the
    fused kernel, 1 on a side stream, 2 as extra workgroups of the depth sort's
    downsweeps.  The same bits in every mode.  Returns the previous mode."""
    prev = load_library().gsr_colour_mode(int(mode))
    if prev < -1:
        raise ValueError(load_library().gsr_last_error().decode())
    return prev


def get_colour_mode() -> int:
    return load_library().gsr_colour_mode(-2)


def get_split() -> int:
    return load_library().gsr_split_mode(-2)


def host_wait_ms(reset: bool = False) -> float:
    """Milliseconds the host spent in the forward's num_rendered wait (gsr_host_wait_us)."""
    return load_library().gsr_host_wait_us(int(bool(reset))) * 1e-3


class GsrLeafGrads(ctypes.Structure):
    """Mirror of ``gsr_leaf_grads`` in include/gsr.h."""
    _fields_ = [("dsh_dc", ctypes.c_void_p), ("dsh_rest", ctypes.c_void_p), ("dscaling", ctypes.c_void_p),
                ("dopacity", ctypes.c_void_p), ("drotation", ctypes.c_void_p), ("rotation_norm", ctypes.c_void_p),
                ("rotation_eps", ctypes.c_float), ("accumulate", ctypes.c_int32), ("dsh_planar", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class GsrL1Seed(ctypes.Structure):  # gsr.h gsr_l1_seed
    _fields_ = [("image", ctypes.c_void_p), ("gt", ctypes.c_void_p), ("dloss", ctypes.c_void_p),
                ("n", ctypes.c_int64)]


class LeafGrads:
    """Outputs (and their inputs) of ``rasterize_gaussians_backward(leaf=...)``: the
    leaf gradients of the caller's activations written by the library itself
    (gsr_backward_leaves, include/gsr.h).  Every tensor is float32, contiguous, on
    the rasterizer's device; ``accumulate`` bits add into an output instead of
    overwriting it (1 dsh, 2 dscaling, 4 dopacity, 8 drotation, 16 dmeans3D).
    ``dopacity`` needs the backward's ``opacities``; ``drotation`` needs
    ``rotation_norm`` (the norms torch's F.normalize computed, [P,1]).
    ``dmeans3D`` [P,3]: where the backward writes (or, bit 16, adds) its means3D
    gradient instead of a fresh tensor (means3D is the _xyz leaf itself: the
    caller points it at that leaf's gradient, e.g. a slice of an all-reduce
    bucket); the returned dmeans3D is then None."""

    _SHAPES = {"dsh_dc": lambda P, M: (P, 1, 3), "dsh_rest": lambda P, M: (P, M - 1, 3),
               "dscaling": lambda P, M: (P, 3), "dopacity": lambda P, M: (P, 1), "drotation": lambda P, M: (P, 4),
               "rotation_norm": lambda P, M: (P, 1)}

    def __init__(self, dsh_dc=None, dsh_rest=None, dscaling=None, dopacity=None, drotation=None,
                 rotation_norm=None, rotation_eps=1e-12, accumulate=0, dmeans3D=None):
        self.dsh_dc, self.dsh_rest, self.dscaling, self.dopacity, self.drotation = (dsh_dc, dsh_rest, dscaling,
                                                                                    dopacity, drotation)
        self.dmeans3D = dmeans3D
        self.rotation_norm = rotation_norm
        self.rotation_eps, self.accumulate = float(rotation_eps), int(accumulate)

    def struct(self, P, M, device, dsh_planar=False) -> GsrLeafGrads:
        ptr = {}
        for name, shape in self._SHAPES.items():
            t = getattr(self, name)
            if t is None or (name == "dsh_rest" and M <= 1):
                ptr[name] = None
                continue
            if (t.dtype != torch.float32 or t.device != device or not t.is_contiguous()
                    or t.numel() != math.prod(shape(P, M))):
                raise RuntimeError(f"leaf gradient {name}: expected a contiguous float32 tensor of shape "
                                   f"{shape(P, M)} on {device}")
            ptr[name] = t.data_ptr()
        return GsrLeafGrads(rotation_eps=self.rotation_eps, accumulate=self.accumulate,
                            dsh_planar=int(bool(dsh_planar)), **ptr)


class GsrAdamSegment(ctypes.Structure):
    """Mirror of ``gsr_adam_segment`` in include/gsr.h."""
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("n", ctypes.c_int64), ("lr", ctypes.c_double)]


ADAM_MAX_SEGS = 8
ABI_VERSION = 12

_lib = None


def library_path() -> Path:
    return Path(os.environ.get("GSR_LIBRARY", str(_DEFAULT)))


def load_library():
    """Load libgsr.so; raise loudly if it is missing (no fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    if not path.exists():
        raise ImportError(
            f"diff_gaussian_rasterization: native library {path} not found; build it with "
            "`python -c 'import __graft_entry__; __graft_entry__.build()'` (hipcc --offload-arch=gfx950)")
    lib = ctypes.CDLL(str(path))
    sz, i32, i64, vp = ctypes.c_size_t, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p
    lib.gsr_geom_bytes.argtypes = [i32, i32, i32]
    lib.gsr_geom_bytes.restype = sz
    lib.gsr_binning_bytes.argtypes = [i64, i32, i32]
    lib.gsr_binning_bytes.restype = sz
    lib.gsr_img_bytes.argtypes = [i32, i32]
    lib.gsr_img_bytes.restype = sz
    lib.gsr_accum_bytes.argtypes = [i32]
    lib.gsr_accum_bytes.restype = sz
    pin = ctypes.POINTER(GsrInputs)
    lib.gsr_forward_preprocess.argtypes = [pin, vp, vp, ctypes.POINTER(i64), vp]
    lib.gsr_forward_preprocess.restype = ctypes.c_int
    lib.gsr_forward_render.argtypes = [pin, vp, vp, vp, i64, vp, vp, vp]
    lib.gsr_forward_render.restype = ctypes.c_int
    lib.gsr_forward_render_l1.argtypes = [pin, vp, vp, vp, i64, vp, vp, vp, vp, vp, vp]
    lib.gsr_forward_render_l1.restype = ctypes.c_int
    lib.gsr_forward.argtypes = [pin, vp, vp, vp, i64, vp, vp, vp, vp, vp, ctypes.POINTER(i64), vp]
    lib.gsr_forward.restype = ctypes.c_int
    lib.gsr_backward.argtypes = [pin, vp, vp, vp, vp, i64, vp, vp] + [vp] * 8 + [vp]
    lib.gsr_backward.restype = ctypes.c_int
    lib.gsr_backward_planar.argtypes = [pin, vp, vp, vp, vp, i64, vp, vp] + [vp] * 8 + [vp]
    lib.gsr_backward_planar.restype = ctypes.c_int
    lib.gsr_backward_leaves.argtypes = [pin, vp, vp, vp, vp, i64, vp, vp] + [vp] * 8 + [ctypes.POINTER(GsrLeafGrads), vp]
    lib.gsr_backward_leaves.restype = ctypes.c_int
    lib.gsr_backward_phase.argtypes = ([pin, vp, vp, vp, vp, i64, vp, vp] + [vp] * 9 +
                                       [ctypes.POINTER(GsrLeafGrads), i32, vp])
    lib.gsr_backward_phase.restype = ctypes.c_int
    for name in ("gsr_backward_colors", "gsr_backward_colors_render", "gsr_backward_colors_finish"):
        getattr(lib, name).argtypes = [pin, vp, vp, vp, vp, i64, vp, vp] + [vp] * 8 + [vp]
        getattr(lib, name).restype = ctypes.c_int
    lib.gsr_sh_record_floats.argtypes = [i32]
    lib.gsr_sh_record_floats.restype = i64
    lib.gsr_sh_grad_from_colors.argtypes = [i32, i32, i32, vp, vp, vp, vp, vp]
    lib.gsr_sh_grad_from_colors.restype = ctypes.c_int
    lib.gsr_point_list_keys.argtypes = [i32, i32, i32, vp, vp, i64, vp, vp]
    lib.gsr_point_list_keys.restype = ctypes.c_int
    lib.gsr_mark_visible.argtypes = [i32, vp, vp, vp, vp, vp]
    lib.gsr_mark_visible.restype = ctypes.c_int
    for name in ("gsr_geom_layout", "gsr_binning_layout", "gsr_img_layout"):
        getattr(lib, name).restype = ctypes.c_int
    lib.gsr_geom_layout.argtypes = [i32, i32, i32, ctypes.POINTER(sz), ctypes.c_int]
    lib.gsr_binning_layout.argtypes = [i64, i32, i32, ctypes.POINTER(sz), ctypes.c_int]
    lib.gsr_img_layout.argtypes = [i32, i32, ctypes.POINTER(sz), ctypes.c_int]
    lib.gsr_timing_enable.argtypes = [ctypes.c_int]
    lib.gsr_timing_enable.restype = ctypes.c_int
    lib.gsr_binning_mode.argtypes = [ctypes.c_int]
    lib.gsr_binning_mode.restype = ctypes.c_int
    lib.gsr_split_mode.argtypes = [ctypes.c_int]
    lib.gsr_split_mode.restype = ctypes.c_int
    lib.gsr_host_wait_us.argtypes = [ctypes.c_int]
    lib.gsr_host_wait_us.restype = ctypes.c_double
    lib.gsr_forward_status.argtypes = [i64, ctypes.c_int, ctypes.POINTER(i64)]
    lib.gsr_forward_status.restype = ctypes.c_int
    lib.gsr_depth_passes_hint.restype = ctypes.c_int
    lib.gsr_colour_mode.argtypes = [ctypes.c_int]
    lib.gsr_colour_mode.restype = ctypes.c_int
    lib.gsr_timing_sample.argtypes = [ctypes.c_int]
    lib.gsr_timing_sample.restype = ctypes.c_int
    lib.gsr_timing_read.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64), ctypes.c_int]
    lib.gsr_timing_read.restype = ctypes.c_int
    lib.gsr_stage_name.argtypes = [ctypes.c_int]
    lib.gsr_stage_name.restype = ctypes.c_char_p
    for name in ("gsr_timing_begin", "gsr_timing_end"):
        getattr(lib, name).argtypes = [ctypes.c_int, vp]
        getattr(lib, name).restype = ctypes.c_int
    lib.gsr_l1_ssim_scratch_bytes.argtypes = [i32, i32, i32]
    lib.gsr_l1_ssim_scratch_bytes.restype = sz
    lib.gsr_l1_ssim.argtypes = [vp, vp, i32, i32, i32, ctypes.c_float, vp, vp, vp, vp]
    lib.gsr_l1_ssim.restype = ctypes.c_int
    lib.gsr_l1_grad.argtypes = [vp, vp, i64, vp, vp, vp]
    lib.gsr_l1_grad.restype = ctypes.c_int
    lib.gsr_adam_step.argtypes = [ctypes.POINTER(GsrAdamSegment), i32, i32, ctypes.c_double, ctypes.c_double,
                                  ctypes.c_double, vp]
    lib.gsr_adam_step.restype = ctypes.c_int
    lib.gsr_densify_stats.argtypes = [i32, vp, vp, i32, vp, vp, vp, vp]
    lib.gsr_densify_stats.restype = ctypes.c_int
    lib.gsr_knn_scratch_bytes.argtypes = [i32]
    lib.gsr_knn_scratch_bytes.restype = sz
    lib.gsr_knn_mean_dist2.argtypes = [i32, vp, vp, vp, vp]
    lib.gsr_knn_mean_dist2.restype = ctypes.c_int
    lib.gsr_last_error.restype = ctypes.c_char_p
    lib.gsr_abi_version.restype = ctypes.c_int
    lib.gsr_build_id.restype = ctypes.c_char_p
    if lib.gsr_abi_version() != ABI_VERSION:
        raise ImportError(f"{path}: ABI version {lib.gsr_abi_version()} != {ABI_VERSION}; rebuild")
    if os.environ.get("GSR_COLOUR_APART"):  # preprocess's colour half on a side stream (set_colour_apart)
        if lib.gsr_colour_mode(int(os.environ["GSR_COLOUR_APART"])) < -1:
            raise ImportError(f"GSR_COLOUR_APART={os.environ['GSR_COLOUR_APART']!r}: {lib.gsr_last_error().decode()}")
    if os.environ.get("GSR_SPLIT"):  # the split replay's setting (set_split), e.g. 0 for A/B timing
        if lib.gsr_split_mode(int(os.environ["GSR_SPLIT"])) < -1:
            raise ImportError(f"GSR_SPLIT={os.environ['GSR_SPLIT']!r}: {lib.gsr_last_error().decode()}")
    _lib = lib
    return lib


def _check(rc: int, what: str):
    if rc != 0:
        msg = _lib.gsr_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {rc}): {msg}")


def _ptr(t):
    """Device pointer of a tensor, or None (NULL) for an empty/absent tensor."""
    if t is None or t.numel() == 0:
        return None
    return t.data_ptr()


def _prep(t, name, device):
    """upstream `.contiguous()` + dtype/device checks; empty stays empty."""
    if t is None or t.numel() == 0:
        return None
    if t.dtype is not torch.float32:
        raise TypeError(f"{name} must be float32 (got {t.dtype})")
    if t.device != device:
        raise RuntimeError(f"{name} is on {t.device}, expected {device}")
    return t if t.is_contiguous() else t.contiguous()


# Test hook (tests/test_poisoned_scratch.py): a byte value every output and scratch
# buffer the entry points allocate is filled with, instead of being left
# uninitialised (None, the default).  0xFF makes every float a NaN and every integer
# all ones, so a kernel that reads a word the same call did not write (a stale
# flag or counter the caching allocator handed back) shows up.
_poison = None


def _alloc(shape, dtype, device):
    if _poison is None:
        return torch.empty(shape, dtype=dtype, device=device)
    n = math.prod(shape) * torch.tensor([], dtype=dtype).element_size()
    return torch.full((n,), _poison, dtype=torch.uint8, device=device).view(dtype).view(shape)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


FLAG_PREPARE_BACKWARD = 1  # gsr.h gsr_flags
FLAG_L1_SEED = 2
FLAG_NO_WAIT = 4
NEED_BINNING = 5  # gsr.h gsr_status: gsr_forward's binning capacity was too small
PHASE_COLOURS_APART = 4  # gsr.h gsr_backward_phase: the colour gradient in a call of its own


# ------------------------------------------------------------------ binning capacity
# gsr_forward queues the whole forward before the host reads num_rendered, into a
# binning buffer sized from the last forward of the same image size and footprint
# (its count scaled by the Gaussian count, plus a margin); a count above that
# capacity costs one extra render call (gsr.h GSR_NEED_BINNING), never a wrong
# result.  The first forward of a size takes the two-call form.
_CAP_SLACK = 1.0625
_CAP_PAD = 4096
_capacity_level = {}  # (W, H, footprint) -> (P, num_rendered) of the last forward
capacity_override = None  # test hook: an int capacity for every forward (0: always the two-call form)
last_forward = {}  # how the last forward ran: {"capacity", "num_rendered", "path"} (tests, bench)
captured_forwards = []  # capacities of the forwards queued under stream capture (forward_status)


def forward_status(captured) -> int:
    """After a captured forward (GSR_FLAG_NO_WAIT; ``captured`` = its (capacity,
    depth passes) record in ``captured_forwards``) has run — a graph replay, then a
    synchronize — the num_rendered its preprocess published on this thread; raises
    if it exceeded the capacity or the keys needed a fourth depth pass (that
    replay's lists, image and gradients are then incomplete: capture again after an
    eager forward, which re-sizes the buffer and the pass hint)."""
    capacity, passes = captured
    n = ctypes.c_int64(0)
    _check(load_library().gsr_forward_status(int(capacity), int(passes), ctypes.byref(n)), "captured forward")
    return n.value


def _capacity_for(key, P):
    if capacity_override is not None:
        return int(capacity_override) or None
    lv = _capacity_level.get(key)
    if lv is None:
        return None
    P0, I0 = lv
    scaled = I0 * P / P0 if P0 > 0 else I0
    return min(int(scaled * _CAP_SLACK) + _CAP_PAD, 0xFFFFFFFF)


def _note_count(key, P, I):
    """Grow the scene's level at once; shrink it slowly (1/128 per forward), so one
    sparse view does not make the next dense one overflow."""
    lv = _capacity_level.get(key)
    if lv is not None and lv[0] == P and I < lv[1]:
        I = max(I, lv[1] - (lv[1] >> 7))
    if len(_capacity_level) > 64 and key not in _capacity_level:
        _capacity_level.clear()
    _capacity_level[key] = (P, I)


def l1_loss(image: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
    """mean|image - gt| (utils/loss_utils.py l1_loss) as a 0-dim float32 device
    tensor: gsr_l1_ssim's loss-only form (lambda 0), no gradient map."""
    lib = load_library()
    x, y = image.contiguous(), gt.contiguous()
    if x.shape != y.shape or x.dim() != 3 or x.dtype != torch.float32 or y.dtype != torch.float32:
        raise RuntimeError(f"l1_loss: image {tuple(x.shape)} and gt {tuple(y.shape)} must be equal float32 [C,H,W]")
    C, H, W = x.shape
    scratch = torch.empty(lib.gsr_l1_ssim_scratch_bytes(C, H, W), dtype=torch.uint8, device=x.device)
    out = torch.empty(3, dtype=torch.float32, device=x.device)
    _check(lib.gsr_l1_ssim(x.data_ptr(), y.data_ptr(), C, H, W, 0.0, None, scratch.data_ptr(), out.data_ptr(),
                           _stream(x.device)), "gsr_l1_ssim")
    return out[0]


def l1_grad(image: torch.Tensor, gt: torch.Tensor, dloss: torch.Tensor) -> torch.Tensor:
    """(dloss / n) * sign(image - gt): the L1 mean's image gradient (gsr_l1_grad)."""
    lib = load_library()
    x, y = image.contiguous(), gt.contiguous()
    g = torch.empty_like(x)
    d = dloss.detach().to(torch.float32).contiguous()
    _check(lib.gsr_l1_grad(x.data_ptr(), y.data_ptr(), x.numel(), d.data_ptr(), g.data_ptr(), _stream(x.device)),
           "gsr_l1_grad")
    return g


def _inputs(bg, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix, projmatrix,
            tan_fovx, tan_fovy, H, W, sh, degree, campos, prefiltered, debug, footprint=None, flags=0, sh_rest=None,
            activations=0):
    if means3D.ndim != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    device = means3D.device
    if device.type != "cuda":
        raise RuntimeError("diff_gaussian_rasterization: tensors must be on a ROCm device (got %s); "
                           "there is no CPU implementation" % device)
    keep = {}
    for name, t in (("background", bg), ("means3D", means3D), ("colors", colors), ("opacity", opacity),
                    ("scales", scales), ("rotations", rotations), ("cov3D_precomp", cov3D_precomp),
                    ("viewmatrix", viewmatrix), ("projmatrix", projmatrix), ("sh", sh), ("campos", campos),
                    ("sh_rest", sh_rest)):
        keep[name] = _prep(t, name, device)
    P = means3D.size(0)
    sh_t, rest_t = keep["sh"], keep["sh_rest"]
    M = sh_t.size(1) if (sh_t is not None and sh_t.size(0) != 0) else 0
    if rest_t is not None:  # GaussianModel's split SH storage: sh = _features_dc [P,1,3]
        if sh_t is None or sh_t.shape[1:] != (1, 3) or rest_t.dim() != 3 or rest_t.size(0) != P or rest_t.size(2) != 3:
            raise RuntimeError("sh_rest: expected sh = features_dc [P,1,3] and sh_rest = features_rest [P,M-1,3]")
        M += rest_t.size(1)
    s = GsrInputs(P=P, D=int(degree), M=M, W=int(W), H=int(H), tan_fovx=float(tan_fovx), tan_fovy=float(tan_fovy),
                  scale_modifier=float(scale_modifier), prefiltered=int(bool(prefiltered)), debug=int(bool(debug)),
                  footprint=FOOTPRINTS[footprint or _footprint], flags=int(flags),
                  bg=_ptr(keep["background"]), means3D=_ptr(keep["means3D"]), colors_precomp=_ptr(keep["colors"]),
                  opacities=_ptr(keep["opacity"]), scales=_ptr(keep["scales"]), rotations=_ptr(keep["rotations"]),
                  cov3D_precomp=_ptr(keep["cov3D_precomp"]), viewmatrix=_ptr(keep["viewmatrix"]),
                  projmatrix=_ptr(keep["projmatrix"]), sh=_ptr(sh_t), campos=_ptr(keep["campos"]),
                  sh_rest=_ptr(rest_t), activations=int(activations))
    return s, keep, device, M


def rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                        viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                        prefiltered, debug, footprint=None, prepare_backward=None):
    """-> (num_rendered, color [3,H,W], radii [P] int32, geomBuffer, binningBuffer, imgBuffer)

    ``footprint`` (keyword, not upstream): "rect" | "tight" for this call; None =
    the module setting (``set_footprint``, env GSR_FOOTPRINT, default "tight").
    ``prepare_backward`` (keyword, not upstream; gsr.h GSR_FLAG_PREPARE_BACKWARD):
    also zero the backward's accumulator beside the blend; None = when grad mode is
    on and an input requires grad.  A speed hint only."""
    if prepare_backward is None:
        prepare_backward = torch.is_grad_enabled() and any(
            isinstance(t, torch.Tensor) and t.requires_grad
            for t in (means3D, colors, opacity, scales, rotations, cov3D_precomp, sh))
    return _rasterize(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                      viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                      prefiltered, debug, footprint, prepare_backward)[:6]


def _rasterize(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
               projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos, prefiltered, debug,
               footprint=None, prepare_backward=False, sh_rest=None, activations=0, l1_target=None):
    """rasterize_gaussians plus its validated inputs ``(struct, kept tensors, device,
    M)``, which the autograd Function hands back to the backward (``inputs=``) so the
    same tensors are not re-checked there: the host's backward path is on the
    step's critical path once the GPU work is short.  ``sh_rest`` / ``activations``
    (not upstream; gsr_inputs): GaussianModel's stored parameters as the inputs —
    ``sh`` = _features_dc and ``sh_rest`` = _features_rest instead of their cat, and
    the ACT_* bits of the opacity / scale / rotation inputs the library activates.
    ``l1_target`` (not upstream; gsr_forward_render_l1): also the L1 loss
    mean|color - l1_target|, appended to the result as a 0-dim tensor, and the
    visibility ``radii > 0`` (bool [P]) after it — from the backward preparation's
    launch when ``prepare_backward``, else computed here."""
    lib = load_library()
    H, W = int(image_height), int(image_width)
    if footprint is not None and footprint not in FOOTPRINTS:
        raise ValueError(f"footprint must be one of {sorted(FOOTPRINTS)} (got {footprint!r})")
    s, keep, device, M = _inputs(background, means3D, colors, opacity, scales, rotations, scale_modifier,
                                 cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, H, W, sh, degree, campos,
                                 prefiltered, debug, footprint, FLAG_PREPARE_BACKWARD if prepare_backward else 0,
                                 sh_rest, activations)
    P = s.P
    out_color = _alloc((3, H, W), torch.float32, device)
    radii = _alloc((P,), torch.int32, device)
    geom = _alloc((lib.gsr_geom_bytes(P, W, H),), torch.uint8, device)
    img = _alloc((lib.gsr_img_bytes(W, H),), torch.uint8, device)
    stream = _stream(device)
    num_rendered = ctypes.c_int64(0)
    gt = loss = vis = None
    if l1_target is not None:
        gt = _prep(l1_target, "l1_target", device)
        if gt is None or gt.shape != (3, H, W):
            raise RuntimeError(f"l1_target must be a float32 [3,{H},{W}] tensor on {device}")
        loss = torch.empty(3, dtype=torch.float32, device=device)
        vis = torch.empty(P, dtype=torch.bool, device=device) if prepare_backward and P > 0 else None
    key = (W, H, s.footprint)
    cap = None if s.debug or P == 0 else _capacity_for(key, P)
    done = False
    if P > 0 and torch.cuda.is_current_stream_capturing():
        # stream capture (torch.cuda.graph): nothing may wait for the device, so the
        # forward is queued whole into the capacity a forward of this scene size set
        # (gsr.h GSR_FLAG_NO_WAIT); forward_status() checks the count after a replay
        if cap is None or s.debug:
            raise RuntimeError("rasterize_gaussians under stream capture needs an eager forward of the same image "
                               "size and footprint first (it sizes the binning buffer) and debug off")
        s.flags |= FLAG_NO_WAIT
        passes = lib.gsr_depth_passes_hint()
        binning = _alloc((lib.gsr_binning_bytes(cap, W, H),), torch.uint8, device)
        _check(lib.gsr_forward(ctypes.byref(s), geom.data_ptr(), _ptr(radii), binning.data_ptr(), cap, img.data_ptr(),
                               out_color.data_ptr(), _ptr(gt), _ptr(loss), _ptr(vis), ctypes.byref(num_rendered),
                               stream), "rasterize_gaussians (captured)")
        s.flags &= ~FLAG_NO_WAIT
        captured_forwards.append((cap, passes))
        last_forward.update(capacity=cap, num_rendered=None, path="captured", binning=binning)
        if vis is None and gt is not None:
            vis = radii > 0
        if gt is None:
            return num_rendered.value, out_color, radii, geom, binning, img, (s, keep, device, M)
        return num_rendered.value, out_color, radii, geom, binning, img, (s, keep, device, M), loss[0], vis
    if cap is not None:  # one call, queued before the count is read (gsr_forward)
        binning = _alloc((lib.gsr_binning_bytes(cap, W, H),), torch.uint8, device)
        rc = lib.gsr_forward(ctypes.byref(s), geom.data_ptr(), _ptr(radii), binning.data_ptr(), cap, img.data_ptr(),
                             out_color.data_ptr(), _ptr(gt), _ptr(loss), _ptr(vis), ctypes.byref(num_rendered), stream)
        done = rc != NEED_BINNING
        if done:
            _check(rc, "rasterize_gaussians")
        last_forward.update(capacity=cap, num_rendered=num_rendered.value, path="one call" if done else "regrown",
                            binning=binning if done else None)
    else:
        _check(lib.gsr_forward_preprocess(ctypes.byref(s), geom.data_ptr(), _ptr(radii), ctypes.byref(num_rendered),
                                          stream), "rasterize_gaussians (preprocess)")
        last_forward.update(capacity=None, num_rendered=num_rendered.value, path="two calls")
    if not done:
        binning = _alloc((lib.gsr_binning_bytes(num_rendered.value, W, H),), torch.uint8, device)
        last_forward.update(binning=binning)
        if gt is None:
            _check(lib.gsr_forward_render(ctypes.byref(s), geom.data_ptr(), binning.data_ptr(), img.data_ptr(),
                                          num_rendered.value, _ptr(radii), out_color.data_ptr(), stream),
                   "rasterize_gaussians (render)")
        else:
            _check(lib.gsr_forward_render_l1(ctypes.byref(s), geom.data_ptr(), binning.data_ptr(), img.data_ptr(),
                                             num_rendered.value, _ptr(radii), out_color.data_ptr(), gt.data_ptr(),
                                             loss.data_ptr(), _ptr(vis), stream),
                   "rasterize_gaussians (render + L1)")
    if P > 0:
        _note_count(key, P, num_rendered.value)
    if gt is None:
        return num_rendered.value, out_color, radii, geom, binning, img, (s, keep, device, M)
    if vis is None:
        vis = radii > 0
    return num_rendered.value, out_color, radii, geom, binning, img, (s, keep, device, M), loss[0], vis


def rasterize_gaussians_backward(background, means3D, radii, colors, scales, rotations, scale_modifier, cov3D_precomp,
                                 viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, sh, degree, campos,
                                 geomBuffer, R, binningBuffer, imageBuffer, debug, drgb_out=None, dsh_planar=False,
                                 on_drgb=None, leaf=None, opacities=None, inputs=None, l1_seed=None, drgb_apart=False):
    """-> (dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, dsh, dscales, drot)

    Not upstream (keyword-only extensions; the defaults are upstream's behaviour):
    ``drgb_out`` — the view-parallel SH exchange (multiview.py): a float32 device
    tensor of at least 3P elements; the library writes the clamp-masked colour
    gradient [P,3] there (gsr_backward_colors) and the returned ``dsh`` is None.
    ``dsh_planar`` — dsh is the [P,M,3] view of [M,P,3] coefficient planes
    (strides (3, 3P, 1); gsr_backward_planar), same values.
    ``on_drgb`` (with ``drgb_out``) — called (with None: no event) between the
    kernels that write drgb (gsr_backward_phase 1) and the per-Gaussian backward
    (phase 2): what the caller queues then — the exchange of drgb — follows drgb
    and runs under the per-Gaussian backward.  With ``drgb_apart`` the render half
    leaves drgb out (GSR_PHASE_COLOURS_APART) and ``on_drgb`` gets a function that
    queues drgb's kernel on the current stream: the caller runs it on its exchange
    stream (after the render half), beside the per-Gaussian backward.
    ``leaf`` — a ``LeafGrads``: the library writes the requested leaf gradients of
    the caller's activations itself (gsr_backward_phase) and returns None in place
    of the activation gradients they replace (dsh, dopacity, dscales, drot, and
    dmeans3D when ``leaf.dmeans3D`` is given); it combines with ``drgb_out`` (the
    exchange takes the SH gradient, the library writes the other leaves).
    ``opacities`` — the forward's opacity input [P,1] (upstream's backward reads
    it from the geom buffer; passed here it is read coalesced); required with a
    leaf opacity gradient.
    ``inputs`` (private) — the forward's validated inputs (``_rasterize``): the
    same tensors as the positional ones, not re-checked.
    ``l1_seed`` — ``(image, gt, dloss)``: the image's gradient is the L1 loss
    mean|image - gt|'s (gsr.h GSR_FLAG_L1_SEED), formed per pixel by the render
    backward; ``dL_dout_color`` is then ignored (may be None)."""
    lib = load_library()
    if inputs is None:
        ref = l1_seed[0] if l1_seed is not None else dL_dout_color
        H, W = int(ref.size(1)), int(ref.size(2))
        inputs = _inputs(background, means3D, colors, opacities, scales, rotations, scale_modifier, cov3D_precomp,
                         viewmatrix, projmatrix, tan_fovx, tan_fovy, H, W, sh, degree, campos, False, debug)
    s, keep, device, M = inputs
    P = s.P
    empty = lambda *shape: _alloc(shape, torch.float32, device)  # noqa: E731
    # on the leaf path the gradients it replaces, and those of absent inputs
    # (upstream's zeros, discarded by the autograd wrapper: 36 B per Gaussian), are
    # neither allocated nor written
    bare = leaf is not None
    own_xyz = bare and leaf.dmeans3D is not None
    if own_xyz:
        t = leaf.dmeans3D
        if t.dtype != torch.float32 or t.device != device or not t.is_contiguous() or t.numel() != 3 * P:
            raise RuntimeError(f"leaf gradient dmeans3D: expected a contiguous float32 tensor of shape ({P}, 3) "
                               f"on {device}")
    dmeans2D = empty(P, 3)
    dmeans3D = leaf.dmeans3D if own_xyz else empty(P, 3)
    dcolors = None if bare and keep["colors"] is None else empty(P, 3)
    dcov3D = None if bare and keep["cov3D_precomp"] is None else empty(P, 6)
    dopacity = None if bare and leaf.dopacity is not None else empty(P, 1)
    dscales = None if bare and leaf.dscaling is not None else empty(P, 3)
    drot = None if bare and leaf.drotation is not None else empty(P, 4)
    if (bare and leaf.dsh_dc is not None) or drgb_out is not None:
        dsh = None
    elif dsh_planar:
        dsh = empty(M, P, 3).permute(1, 0, 2)
    else:
        dsh = empty(P, M, 3)
    ret = (dmeans2D, dcolors, dopacity, None if own_xyz else dmeans3D, dcov3D, dsh, dscales, drot)
    if P == 0:
        return ret
    if l1_seed is not None:
        image, gt, dloss = (_prep(t, n, device) for t, n in zip(l1_seed, ("l1 image", "l1 gt", "l1 dloss")))
        if image.shape != (3, s.H, s.W) or gt.shape != image.shape or dloss.numel() != 1:
            raise RuntimeError(f"l1_seed: image and gt must be [3,{s.H},{s.W}] and dloss one element")
        seed = GsrL1Seed(image.data_ptr(), gt.data_ptr(), dloss.data_ptr(), 3 * s.H * s.W)
        s = GsrInputs.from_buffer_copy(s)  # the forward's struct, with the backward flag
        s.flags |= FLAG_L1_SEED
        grad_ptr = ctypes.addressof(seed)
    else:
        grad = _prep(dL_dout_color, "dL_dout_color", device)
        grad_ptr = grad.data_ptr()
    if not radii.is_contiguous():
        radii = radii.contiguous()
    if drgb_out is not None and (drgb_out.dtype != torch.float32 or drgb_out.device != device
                                 or not drgb_out.is_contiguous() or drgb_out.numel() < 3 * P):
        raise RuntimeError("drgb_out must be a contiguous float32 tensor of >= 3P elements on the input device")
    head = (ctypes.byref(s), radii.data_ptr(), geomBuffer.data_ptr(),
            binningBuffer.data_ptr() if binningBuffer.numel() else None, imageBuffer.data_ptr(), int(R),
            grad_ptr, None, dmeans2D.data_ptr(), _ptr(dcolors), _ptr(dopacity),
            dmeans3D.data_ptr(), _ptr(dcov3D))
    stream = _stream(device)
    if leaf is None and drgb_out is None:
        fn = lib.gsr_backward_planar if dsh_planar and dsh is not None and M > 0 else lib.gsr_backward
        _check(fn(*head, _ptr(dsh), _ptr(dscales), _ptr(drot), stream), "rasterize_gaussians_backward")
        return ret
    # gsr_backward_phase: the leaf gradients and / or the exchange's colour gradient
    lg = ctypes.byref(leaf.struct(P, M, device, dsh_planar)) if leaf is not None else None
    tail = (_ptr(dsh), _ptr(drgb_out), _ptr(dscales), _ptr(drot), lg)
    if drgb_out is not None and on_drgb is not None:
        # the caller's exchange of drgb starts between the phases: a collective
        # launched then waits for exactly what the stream holds so far (drgb
        # written), and runs under the per-Gaussian backward.  The device has the
        # rest of the forward and the render backward queued at this point, so the
        # launch's host time delays nothing (an event and a second stream for it
        # cost the host ~25 us a step, and the exchange path is host-bound)
        if drgb_apart:
            _check(lib.gsr_backward_phase(*head, *tail, 1 | PHASE_COLOURS_APART, stream),
                   "rasterize_gaussians_backward")

            def write_drgb():
                _check(lib.gsr_backward_phase(*head, *tail, PHASE_COLOURS_APART, _stream(device)),
                       "rasterize_gaussians_backward (colour gradient)")
            on_drgb(write_drgb)
        else:
            _check(lib.gsr_backward_phase(*head, *tail, 1, stream), "rasterize_gaussians_backward")
            on_drgb(None)
        _check(lib.gsr_backward_phase(*head, *tail, 2, stream), "rasterize_gaussians_backward")
    else:
        _check(lib.gsr_backward_phase(*head, *tail, 3, stream), "rasterize_gaussians_backward")
    return ret


def sh_record_floats(P: int) -> int:
    """Floats per view record of the SH exchange: [campos(3), degree, drgb(3P), pad]."""
    return int(load_library().gsr_sh_record_floats(int(P)))


def sh_grad_from_colors(means3D, records, nviews: int, dsh_dc, dsh_rest):
    """dsh_dc [P,1,3], dsh_rest [P,M-1,3] <- sum over the nviews records of
    basis(normalize(mean - campos_v)) (x) drgb_v (gsr_sh_grad_from_colors)."""
    lib = load_library()
    device = means3D.device
    P = means3D.size(0)
    M = dsh_dc.size(1) + (dsh_rest.size(1) if dsh_rest is not None else 0)
    m = _prep(means3D, "means3D", device)
    rec = _prep(records, "records", device)
    if rec.numel() < nviews * sh_record_floats(P):
        raise RuntimeError("sh_grad_from_colors: records hold fewer than nviews records")
    for t, name in ((dsh_dc, "dsh_dc"), (dsh_rest, "dsh_rest")):
        if t is not None and (not t.is_contiguous() or t.dtype != torch.float32 or t.device != device
                              or t.size(0) != P):
            raise RuntimeError(f"{name} must be a contiguous float32 [P,*,3] tensor on the input device")
    _check(lib.gsr_sh_grad_from_colors(P, M, int(nviews), _ptr(m), _ptr(rec), _ptr(dsh_dc), _ptr(dsh_rest),
                                       _stream(device)), "sh_grad_from_colors")


def mark_visible(means3D, viewmatrix, projmatrix):
    """-> present [P] bool (view-space z > 0.2)"""
    lib = load_library()
    if means3D.ndim != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    device = means3D.device
    P = means3D.size(0)
    present = torch.empty((P,), dtype=torch.bool, device=device)
    m = _prep(means3D, "means3D", device)
    v = _prep(viewmatrix, "viewmatrix", device)
    p = _prep(projmatrix, "projmatrix", device)
    _check(lib.gsr_mark_visible(P, _ptr(m), _ptr(v), _ptr(p), _ptr(present), _stream(device)), "mark_visible")
    return present


# ------------------------------------------------------------------ timing hooks
def timing_enable(on=True):
    """Start per-stage event timing: True = every stage, False = off, or an
    iterable of stage names (only those stages get events)."""
    lib = load_library()
    if isinstance(on, bool):
        mask = -1 if on else 0
    else:
        names = [lib.gsr_stage_name(i).decode() for i in range(16)]
        mask = 0
        for n in on:
            mask |= 1 << names.index(n)
    lib.gsr_timing_enable(mask)


_stage_ids = {}


def _stage_id(name: str) -> int:
    if not _stage_ids:
        lib = load_library()
        for i in range(32):
            n = lib.gsr_stage_name(i).decode()
            if not n:
                break
            _stage_ids[n] = i
    return _stage_ids[name]


def timing_begin(name: str, device) -> None:
    """Open a caller-marked region of stage `name` on the current stream (recorded
    only while timing_enable has that stage on; fence-free events)."""
    lib = load_library()
    _check(lib.gsr_timing_begin(_stage_id(name), _stream(device)), "gsr_timing_begin")


def timing_end(name: str, device) -> None:
    lib = load_library()
    _check(lib.gsr_timing_end(_stage_id(name), _stream(device)), "gsr_timing_end")


def timing_sample(every: int = 1) -> None:
    """Events on every `every`-th launch of a stage only (gsr_timing_sample)."""
    _check(load_library().gsr_timing_sample(int(every)), "gsr_timing_sample")


def timing_read() -> dict:
    """{stage: (total_ms, launches)} accumulated since timing_enable (waits for events)."""
    lib = load_library()
    ms = (ctypes.c_double * 16)()
    n_ = (ctypes.c_int64 * 16)()
    n = lib.gsr_timing_read(ms, n_, 16)
    if n < 0:
        _check(-n, "gsr_timing_read")
    return {lib.gsr_stage_name(i).decode(): (ms[i], n_[i]) for i in range(n)}


# ------------------------------------------------------------------ test hooks
def point_list_keys(P, W, H, geomBuffer, binningBuffer, num_rendered):
    """upstream's sorted 64-bit keys (tile << 32 | depth bits) of a forward's lists,
    as an int64 tensor holding the uint64 bit patterns (gsr_point_list_keys)."""
    lib = load_library()
    # all ones where no tile range covers an entry (never, for a consistent binning)
    keys = torch.full((max(int(num_rendered), 0),), -1, dtype=torch.int64, device=geomBuffer.device)
    if keys.numel():
        _check(lib.gsr_point_list_keys(int(P), int(W), int(H), geomBuffer.data_ptr(), binningBuffer.data_ptr(),
                                       int(num_rendered), keys.data_ptr(), _stream(geomBuffer.device)),
               "point_list_keys")
    return keys


def last_spans(W: int, H: int):
    """Row spans of the last forward (the row-span binning's pass-A output, for the
    byte model of bench.py), or None when it took the LSD sort.  Synchronises."""
    b = last_forward.get("binning")
    if b is None or get_binning_mode() != "rowspan" or (W + 15) // 16 > 256 or (H + 15) // 16 > 256:
        return None
    cap = last_forward.get("capacity") or last_forward.get("num_rendered", 0)
    off = layouts(1, W, H, cap)[1].get("rowspan")
    if off is None or not last_forward.get("num_rendered"):
        return None
    return int(b[off + 4 * 513:off + 4 * 514].view(torch.int32).item())


def layouts(P, W, H, num_rendered):
    """Byte offsets of the named scratch sub-arrays (parity tests read intermediates)."""
    lib = load_library()
    g = (ctypes.c_size_t * 16)()
    n = lib.gsr_geom_layout(P, W, H, g, 16)
    b = (ctypes.c_size_t * 16)()
    nb = lib.gsr_binning_layout(num_rendered, W, H, b, 16)
    im = (ctypes.c_size_t * 16)()
    ni = lib.gsr_img_layout(W, H, im, 16)
    geom_names = ("depths", "means2D", "splats", "clamped", "tiles_touched", "ranges", "ctrl", "depth_order",
                  "dsort_ctrl")  # (binning: point_list at offset 0 for every capacity)
    return (dict(zip(geom_names, list(g)[:n])), dict(zip(("keys", "point_list", "rowspan"), list(b)[:nb])),
            dict(zip(("final_T", "n_contrib"), list(im)[:ni])))
