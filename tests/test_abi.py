"""The C ABI library loads without a GPU, exports every symbol include/gsr.h
declares, and its host-side logic (argument validation, scratch layouts, error
strings) behaves — no kernel is launched here."""
import ctypes
import re

import pytest

from conftest import ROOT


def header_functions():
    text = (ROOT / "include" / "gsr.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gsr_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from diff_gaussian_rasterization import _C

    return _C.load_library()


def test_every_declared_symbol_is_exported(lib):
    from diff_gaussian_rasterization import _C

    names = header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), f"libgsr.so lacks {n}"
    assert sorted(_C.EXPORTED) == names


def test_abi_version_and_struct_layout(lib):
    from diff_gaussian_rasterization import _C

    assert lib.gsr_abi_version() == _C.ABI_VERSION == 12
    assert ctypes.sizeof(_C.GsrL1Seed) == 32  # struct gsr_l1_seed: three pointers and an int64
    # 12 x 4-byte scalars, 11 pointers, then sh_rest and two int32 (include/gsr.h struct gsr_inputs)
    assert ctypes.sizeof(_C.GsrInputs) == 48 + 12 * 8 + 8
    assert _C.GsrInputs.footprint.offset == 40
    assert _C.GsrInputs.bg.offset == 48
    assert _C.GsrInputs.sh_rest.offset == 136 and _C.GsrInputs.activations.offset == 144
    # 6 pointers, then rotation_eps and three int32 (struct gsr_leaf_grads)
    assert ctypes.sizeof(_C.GsrLeafGrads) == 6 * 8 + 16
    assert _C.GsrLeafGrads.rotation_eps.offset == 48 and _C.GsrLeafGrads.dsh_planar.offset == 56


def test_scratch_layouts_are_aligned_and_disjoint(lib):
    from diff_gaussian_rasterization import _C

    for P, W, H, I in ((1, 16, 16, 1), (10_000, 256, 256, 18_267), (1_000_000, 1920, 1080, 8_023_099),
                       (5_000_000, 3840, 2160, 110_000_000)):
        g, b, im = _C.layouts(P, W, H, I)
        for d in (g, b, im):
            offs = list(d.values())
            assert all(o % 256 == 0 for o in offs)
            assert len(set(offs)) == len(offs)
        assert list(g.values()) == sorted(g.values()) and list(im.values()) == sorted(im.values())
        # the point list sits at offset 0 whatever the capacity (gsr_forward's
        # buffers are sized before the count is known; the backward needs the pointer)
        assert b["point_list"] == 0 and b["keys"] >= 4 * I
        assert lib.gsr_geom_bytes(P, W, H) > g["ctrl"]
        assert lib.gsr_binning_bytes(I, W, H) >= I * 12
        assert lib.gsr_img_bytes(W, H) >= W * H * 8
        assert lib.gsr_accum_bytes(P) == P * 64
        # per-Gaussian sub-arrays hold P entries each
        assert g["means2D"] - g["depths"] >= 4 * P
        assert g["splats"] - g["means2D"] >= 8 * P


def _inputs(**kw):
    from diff_gaussian_rasterization import _C

    base = dict(P=4, D=0, M=1, W=16, H=16, tan_fovx=0.5, tan_fovy=0.5, scale_modifier=1.0, prefiltered=0, debug=0,
                bg=1, means3D=1, opacities=1, viewmatrix=1, projmatrix=1, campos=1, sh=1, scales=1, rotations=1)
    base.update(kw)
    return _C.GsrInputs(**base)


@pytest.mark.parametrize("kw,msg", [
    (dict(colors_precomp=1), "excatly one of either SHs or precomputed colors"),
    (dict(sh=None), "excatly one of either SHs or precomputed colors"),
    (dict(cov3D_precomp=1), "exactly one of either scale/rotation pair or precomputed 3D covariance"),
    (dict(scales=None), "exactly one of either scale/rotation pair or precomputed 3D covariance"),
    (dict(D=3, M=4), "degree 3 needs 16"),
    (dict(D=4, M=25), "sh_degree must be in [0, 3]"),
    (dict(P=-1), "num_points, 3"),
    (dict(W=0), "image size"),
    (dict(footprint=2), "footprint must be"),
    (dict(activations=8), "unknown activations"),
    (dict(sh_rest=1), "sh_rest needs sh"),
    (dict(sh_rest=1, sh=None, colors_precomp=1, M=16), "sh_rest needs sh"),
])
def test_argument_validation_mirrors_upstream_errors(lib, kw, msg):
    s = _inputs(**kw)
    n = ctypes.c_int64(-1)
    rc = lib.gsr_forward_preprocess(ctypes.byref(s), None, None, ctypes.byref(n), None)
    assert rc != 0
    assert msg in lib.gsr_last_error().decode()


def test_zero_gaussians_is_a_host_side_no_op(lib):
    s = _inputs(P=0)
    n = ctypes.c_int64(-1)
    assert lib.gsr_forward_preprocess(ctypes.byref(s), None, None, ctypes.byref(n), None) == 0
    assert n.value == 0
    assert lib.gsr_backward(ctypes.byref(s), None, None, None, None, 0, *([None] * 11)) == 0
    assert lib.gsr_mark_visible(0, None, None, None, None, None) == 0


def test_sh_exchange_entry_points_validate(lib):
    """gsr_backward_colors / gsr_sh_record_floats / gsr_sh_grad_from_colors: host-side
    checks only (no device work without a GPU)."""
    assert lib.gsr_sh_record_floats(0) == 4
    assert lib.gsr_sh_record_floats(1) == 8 and lib.gsr_sh_record_floats(4) == 16
    assert lib.gsr_sh_record_floats(1_000_000) == 3_000_004
    assert lib.gsr_sh_record_floats(-1) == -1
    assert lib.gsr_sh_grad_from_colors(10, 5, 1, None, None, None, None, None) != 0
    assert "M must be" in lib.gsr_last_error().decode()
    assert lib.gsr_sh_grad_from_colors(10, 16, 1, None, None, None, None, None) != 0
    assert "NULL" in lib.gsr_last_error().decode()
    assert lib.gsr_sh_grad_from_colors(0, 16, 1, None, None, None, None, None) == 0
    s = _inputs(P=0)
    assert lib.gsr_backward_colors(ctypes.byref(s), None, None, None, None, 0, *([None] * 11)) == 0


def test_stage_names(lib):
    from diff_gaussian_rasterization import _C

    names = [lib.gsr_stage_name(i).decode() for i in range(12)]
    assert names == ["preprocess", "scan", "depth_sort", "duplicate", "tile_sort", "render_fwd", "render_bwd",
                     "preprocess_bwd", "bwd_prepare", "exchange_wait", "sh_rebuild", "colour"]
    assert lib.gsr_stage_name(99).decode() == ""
    assert lib.gsr_timing_sample(0) != 0 and "sample period" in lib.gsr_last_error().decode()
    assert lib.gsr_timing_sample(4) == 0 and lib.gsr_timing_sample(1) == 0
    _C.timing_enable(True)
    assert _C.timing_read() == {n: (0.0, 0) for n in names}
    _C.timing_enable(False)


def test_cpu_tensors_are_rejected_loudly():
    import torch
    from diff_gaussian_rasterization import _C

    with pytest.raises(RuntimeError, match="no CPU implementation"):
        _C.rasterize_gaussians(torch.zeros(3), torch.zeros(2, 3), torch.empty(0), torch.ones(2, 1), torch.ones(2, 3),
                               torch.ones(2, 4), 1.0, torch.empty(0), torch.eye(4), torch.eye(4), 0.5, 0.5, 8, 8,
                               torch.zeros(2, 1, 3), 0, torch.zeros(3), False, False)
    with pytest.raises(RuntimeError, match="num_points, 3"):
        _C.rasterize_gaussians(torch.zeros(3), torch.zeros(2, 4), torch.empty(0), torch.ones(2, 1), torch.ones(2, 3),
                               torch.ones(2, 4), 1.0, torch.empty(0), torch.eye(4), torch.eye(4), 0.5, 0.5, 8, 8,
                               torch.zeros(2, 1, 3), 0, torch.zeros(3), False, False)


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    from diff_gaussian_rasterization import _C

    monkeypatch.setattr(_C, "_lib", None)
    monkeypatch.setenv("GSR_LIBRARY", str(tmp_path / "nope.so"))
    with pytest.raises(ImportError, match="not found"):
        _C.load_library()


def test_footprint_selector():
    from diff_gaussian_rasterization import _C, get_footprint, set_footprint

    assert get_footprint() == "rect"  # package default: upstream's lists
    prev = set_footprint("tight")
    try:
        assert prev == "rect" and get_footprint() == "tight"
        with pytest.raises(ValueError, match="footprint must be"):
            set_footprint("box")
    finally:
        set_footprint(prev)
    assert _C.FOOTPRINTS == {"rect": 0, "tight": 1}
    assert lib_point_list_keys_validates()


def test_binning_mode_selector():
    from diff_gaussian_rasterization import get_binning_mode, set_binning_mode

    assert get_binning_mode() == "rowspan"  # the default
    prev = set_binning_mode("lsd")
    try:
        assert prev == "rowspan" and get_binning_mode() == "lsd"
        with pytest.raises(ValueError, match="binning mode must be"):
            set_binning_mode("bitonic")
    finally:
        set_binning_mode(prev)
    from diff_gaussian_rasterization import _C

    lib = _C.load_library()
    assert lib.gsr_binning_mode(7) == -1 and "binning mode 7" in lib.gsr_last_error().decode()
    assert lib.gsr_binning_mode(-1) == 0


def lib_point_list_keys_validates():
    from diff_gaussian_rasterization import _C

    lib = _C.load_library()
    assert lib.gsr_point_list_keys(10, 16, 16, None, None, 0, None, None) == 0  # nothing to write
    assert lib.gsr_point_list_keys(10, 16, 16, None, None, 5, None, None) != 0
    assert "NULL" in lib.gsr_last_error().decode()
    return True


def test_library_was_built_from_this_tree(lib):
    """Build provenance: the shipped libgsr.so carries the SHA-256 of the sources it
    was compiled from (Makefile -> gsr_build_id); it must be this tree's."""
    import sys

    sys.path.insert(0, str(ROOT / "tools"))
    from build_id import build_id

    assert lib.gsr_build_id().decode() == build_id(), "libgsr.so is stale: rebuild (make -C 3dgs_study_amd/csrc)"


def test_l1_seed_flag_validates(lib):
    """GSR_FLAG_L1_SEED: a backward flag (a forward rejects it), and the backward
    checks the seed struct before any device work."""
    from diff_gaussian_rasterization import _C

    s = _inputs(flags=_C.FLAG_L1_SEED)
    n = ctypes.c_int64(-1)
    assert lib.gsr_forward_preprocess(ctypes.byref(s), None, None, ctypes.byref(n), None) != 0
    assert "backward flag" in lib.gsr_last_error().decode()
    for seed in (_C.GsrL1Seed(1, 1, 1, 3 * 16 * 16 + 1), _C.GsrL1Seed(None, 1, 1, 3 * 16 * 16),
                 _C.GsrL1Seed(1, 1, None, 3 * 16 * 16)):
        # (in, radii, geom, binning, img, num_rendered, seed, accum, dmeans2D, dcolors, dopacity,
        #  dmeans3D, dcov3D, dsh, dscales, drot, stream)
        rc = lib.gsr_backward(ctypes.byref(s), 1, 1, 1, 1, 0, ctypes.addressof(seed), None, 1, None, 1, 1, None,
                              1, 1, 1, None)
        assert rc != 0
        assert "l1 seed" in lib.gsr_last_error().decode()


def test_forward_render_l1_validates(lib):
    """gsr_forward_render_l1: gt, loss_out and img required (host-side checks)."""
    s = _inputs()
    assert lib.gsr_forward_render_l1(ctypes.byref(s), 1, 1, 1, 0, 1, 1, None, 1, None, None) != 0
    assert "gt is NULL" in lib.gsr_last_error().decode()
    assert lib.gsr_forward_render_l1(ctypes.byref(s), 1, 1, None, 0, 1, 1, 1, 1, None, None) != 0
    assert "loss_out and img required" in lib.gsr_last_error().decode()
    assert lib.gsr_forward_render_l1(ctypes.byref(s), 1, 1, 1, 0, 1, 1, 1, None, None, None) != 0
    assert "loss_out and img required" in lib.gsr_last_error().decode()
    assert lib.gsr_forward_render_l1(ctypes.byref(s), 1, 1, 1, 0, 1, 1, 1, 1, 1, None) != 0  # visible, no flag
    assert "needs GSR_FLAG_PREPARE_BACKWARD" in lib.gsr_last_error().decode()


def test_l1_grad_validates(lib):
    """gsr_l1_grad (the L1 loss's backward): host-side checks only."""
    assert lib.gsr_l1_grad(None, None, 0, None, None, None) == 0  # nothing to do
    assert lib.gsr_l1_grad(None, None, -1, None, None, None) != 0
    assert "negative" in lib.gsr_last_error().decode()
    assert lib.gsr_l1_grad(None, None, 5, None, None, None) != 0
    assert "NULL" in lib.gsr_last_error().decode()
    # with lambda 0 the loss alone may be asked for (no gradient map), else it is required
    assert lib.gsr_l1_ssim(1, 1, 3, 4, 4, ctypes.c_float(0.5), None, 1, 1, None) != 0
    assert "NULL" in lib.gsr_last_error().decode()


def test_forward_one_call_validates(lib):
    """gsr_forward (the one-call forward, binning sized before the count is known):
    host-side checks only."""
    s = _inputs()
    n = ctypes.c_int64(-1)
    # (in, geom, radii, binning, capacity, img, out_color, gt, loss_out, visible_out, num_rendered, stream)
    assert lib.gsr_forward(ctypes.byref(s), 1, 1, 1, 16, 1, 1, None, None, None, None, None) != 0
    assert "num_rendered is NULL" in lib.gsr_last_error().decode()
    assert lib.gsr_forward(ctypes.byref(s), 1, 1, 1, -1, 1, 1, None, None, None, ctypes.byref(n), None) != 0
    assert "capacity out of range" in lib.gsr_last_error().decode()
    assert lib.gsr_forward(ctypes.byref(s), 1, 1, 1, 1 << 32, 1, 1, None, None, None, ctypes.byref(n), None) != 0
    assert lib.gsr_forward(ctypes.byref(s), 1, 1, 1, 16, 1, None, None, None, None, ctypes.byref(n), None) != 0
    assert "out_color is NULL" in lib.gsr_last_error().decode()
    assert lib.gsr_forward(ctypes.byref(s), 1, 1, 1, 16, 1, 1, 1, None, None, ctypes.byref(n), None) != 0
    assert "loss_out and img required" in lib.gsr_last_error().decode()
    assert lib.gsr_forward(ctypes.byref(s), 1, 1, 1, 16, 1, 1, None, None, 1, ctypes.byref(n), None) != 0
    assert "visible_out needs gt" in lib.gsr_last_error().decode()
    assert lib.gsr_forward(ctypes.byref(s), None, 1, 1, 16, 1, 1, None, None, None, ctypes.byref(n), None) != 0
    assert "scratch buffers are NULL" in lib.gsr_last_error().decode()
    assert n.value == 0
    bad = _inputs(D=3, M=4)
    assert lib.gsr_forward(ctypes.byref(bad), 1, 1, 1, 16, 1, 1, None, None, None, ctypes.byref(n), None) != 0
    assert "degree 3 needs 16" in lib.gsr_last_error().decode()


def test_binning_capacity_policy():
    """The binding's capacity for gsr_forward: none before the first forward of an
    image size and footprint, then the last count scaled by the Gaussian count with
    a margin; it grows at once and shrinks by 1/128 per forward."""
    from diff_gaussian_rasterization import _C

    key = (123, 45, 1)
    _C._capacity_level.pop(key, None)
    assert _C._capacity_for(key, 1000) is None
    _C._note_count(key, 1000, 50_000)
    cap = _C._capacity_for(key, 1000)
    assert cap == int(50_000 * _C._CAP_SLACK) + _C._CAP_PAD
    assert _C._capacity_for(key, 2000) == int(100_000 * _C._CAP_SLACK) + _C._CAP_PAD  # densified: scaled
    _C._note_count(key, 1000, 10_000)  # a sparse view: the level decays, it does not drop
    assert _C._capacity_level[key] == (1000, 50_000 - (50_000 >> 7))
    _C._note_count(key, 1000, 80_000)
    assert _C._capacity_level[key] == (1000, 80_000)
    prev = _C.capacity_override
    try:
        _C.capacity_override = 7
        assert _C._capacity_for(key, 1000) == 7
        _C.capacity_override = 0
        assert _C._capacity_for(key, 1000) is None
    finally:
        _C.capacity_override = prev
        _C._capacity_level.pop(key, None)


def test_bench_measured_roofline_helpers():
    """bench.py's iteration roofline from PMC bytes: per-unit bytes come
    from profiles/pmc_summary.json's "units" records (tools/pmc_summary.py), keyed by
    workload and footprint; a workload without a record reports null, never a guess."""
    import json as _json
    import sys as _sys

    _sys.path.insert(0, str(ROOT))
    import bench

    assert bench.pmc_unit_bytes("unit_no_such_workload") is None
    assert bench.measured_frac("unit_no_such_workload", 1000.0) is None
    f = ROOT / "profiles" / "pmc_summary.json"
    units = _json.loads(f.read_text()).get("units", {})
    for key, rec in units.items():
        b = rec["hbm_bytes_per_unit"]
        assert b > 0 and rec["units"] > 0
        assert bench.measured_frac(key, 1000.0) == round(b * 1000.0 / 1e9 / bench.HBM_PEAK_GBS, 4)


def test_backward_phase_validates(lib):
    """gsr_backward_phase: phases 1 .. 7 (GSR_PHASE_COLOURS_APART = 4: the colour
    gradient in a call of its own); anything else is refused before any work."""
    from diff_gaussian_rasterization import _C

    assert _C.PHASE_COLOURS_APART == 4
    s = _inputs(P=0)
    for bad in (0, 8, -1):
        rc = lib.gsr_backward_phase(ctypes.byref(s), None, None, None, None, 0, *([None] * 12), bad, None)
        assert rc != 0 and "phases must be 1 .. 7" in lib.gsr_last_error().decode(), bad
    for ok in (1, 2, 3, 4, 5, 6, 7):  # P = 0: accepted, nothing to do
        assert lib.gsr_backward_phase(ctypes.byref(s), None, None, None, None, 0, *([None] * 12), ok, None) == 0, ok


def test_split_mode_values():
    """gsr_split_mode: set / query / reject (no GPU call)."""
    from diff_gaussian_rasterization import _C

    prev = _C.get_split()
    try:
        assert _C.set_split(0) == prev
        assert _C.get_split() == 0
        with pytest.raises(ValueError):
            _C.set_split(-5)
        assert _C.get_split() == 0
    finally:
        _C.set_split(prev)


def test_colour_mode_values():
    """gsr_colour_mode: set / query / reject (no GPU call)."""
    from diff_gaussian_rasterization import _C

    prev = _C.get_colour_mode()
    try:
        assert _C.set_colour_mode(0) == prev
        assert _C.get_colour_apart() is False
        assert _C.set_colour_mode(2) == 0
        assert _C.get_colour_mode() == 2 and _C.get_colour_apart() is False
        assert _C.set_colour_apart(True) is False and _C.get_colour_mode() == 1
        assert _C.load_library().gsr_colour_mode(7) == -3
        with pytest.raises(ValueError):
            _C.set_colour_mode(3)
        assert _C.get_colour_mode() == 1
    finally:
        _C.set_colour_mode(prev)
