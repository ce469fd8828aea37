"""Preprocess's colour half on a side stream (include/gsr.h gsr_colour_mode; abi.hip
queue_preprocess / queue_render; preprocess.hip preprocess_colour_kernel): the
one-call forward with the geometry half in line and the colour half beside the
binning gives the fused kernel's outputs bit for bit — records, clamp bits, image,
final_T, n_contrib — and the same gradients, with and without the backward's
preparation (the SH Jacobian), at SH degree 3 (register rows), 2 (LDS rows) and 0."""
import numpy as np
import pytest

from helpers import case, random_dL, rel_l2, run_hip, run_oracle
from test_gpu_parity import check_backward, check_forward

pytestmark = pytest.mark.gpu

FWD = ("color", "final_T", "n_contrib", "splats", "clamped", "radii", "point_list", "ranges", "depths")
GRADS = ("dmeans2D", "dcolors", "dopacity", "dmeans3D", "dcov3D", "dsh", "dscales", "drot")


@pytest.fixture
def one_call():
    """Every forward takes the one-call form (gsr_forward), which is where the colour
    half runs apart (the two-call form keeps the fused kernel)."""
    from diff_gaussian_rasterization import _C

    prev = _C.capacity_override
    _C.capacity_override = 2_000_000
    yield
    _C.capacity_override = prev


@pytest.mark.parametrize("deg", [3, 2, 0])
@pytest.mark.parametrize("prepare", [True, False])
def test_colour_apart_bit_identical(dev, oracle, one_call, deg, prepare):
    from diff_gaussian_rasterization import _C

    cam, g = case(20_000, 320, 200, deg, seed=4, view=3)
    dL = random_dL(200, 320)
    out = {}
    prev = _C.get_colour_apart()
    try:
        for apart in (False, True):
            _C.set_colour_apart(apart)
            out[apart] = run_hip(cam, g, dev, dL=dL, prepare=prepare)
            assert _C.last_forward["path"] == "one call"
    finally:
        _C.set_colour_apart(prev)
    a, b = out[False], out[True]
    for k in FWD:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    for n in GRADS:
        if a["grads"][n].size:
            assert rel_l2(b["grads"][n], a["grads"][n]) <= 1e-6, n
    r = run_oracle(oracle, cam, g)
    check_forward(b, r)
    check_backward(b, oracle.backward(r, dL))
