"""Preprocess's colour half apart from its geometry half (include/gsr.h
gsr_colour_mode; abi.hip queue_preprocess / queue_render): on a side stream (mode
1; preprocess.hip preprocess_colour_kernel) or as extra workgroups of the depth
sort's downsweeps (mode 2; binning.hip radix_downsweep_kernel<..., RIDE>,
gsr_colour.hpp), the one-call forward gives the fused kernel's outputs bit for bit — records, clamp bits, image,
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


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("deg", [3, 2, 0])
@pytest.mark.parametrize("prepare", [True, False])
def test_colour_apart_bit_identical(dev, oracle, one_call, mode, deg, prepare):
    from diff_gaussian_rasterization import _C

    cam, g = case(20_000, 320, 200, deg, seed=4, view=3)
    dL = random_dL(200, 320)
    out = {}
    prev = _C.get_colour_mode()
    try:
        for m in (0, mode):
            _C.set_colour_mode(m)
            out[m] = run_hip(cam, g, dev, dL=dL, prepare=prepare)
            assert _C.last_forward["path"] == "one call"
    finally:
        _C.set_colour_mode(prev)
    a, b = out[0], out[mode]
    for k in FWD:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    for n in GRADS:
        if a["grads"][n].size:
            assert rel_l2(b["grads"][n], a["grads"][n]) <= 1e-6, n
    r = run_oracle(oracle, cam, g)
    check_forward(b, r)
    check_backward(b, oracle.backward(r, dL))


@pytest.mark.parametrize("P", [1, 255, 257, 70_000])
def test_colour_riders_sizes(dev, P):
    """Riders at sizes around the workgroup size and at a size whose colour blocks do
    not divide evenly over the three downsweeps (the two-call form too): the same
    bits as the fused kernel."""
    from diff_gaussian_rasterization import _C

    cam, g = case(P, 256, 160, 3, seed=7, view=1)
    dL = random_dL(160, 256)
    out = {}
    prev = _C.get_colour_mode()
    try:
        for m in (0, 2):
            _C.set_colour_mode(m)
            out[m] = run_hip(cam, g, dev, dL=dL, prepare=True)
    finally:
        _C.set_colour_mode(prev)
    for k in FWD:
        np.testing.assert_array_equal(out[0][k], out[2][k], err_msg=k)
    for n in GRADS:  # (the backward's atomics add in a run-dependent order)
        if out[0]["grads"][n].size:
            assert rel_l2(out[2]["grads"][n], out[0]["grads"][n]) <= 1e-6, n


def test_colour_riders_model_path(dev):
    """The stored-parameter render (the SH rows from GaussianModel's two leaves, the
    bench's path): riders give the fused kernel's image and radii bit for bit and the
    same leaf gradients."""
    import torch

    import train_step
    from diff_gaussian_rasterization import _C

    cam, g = case(60_000, 640, 360, 3, seed=9, view=2)
    dL = torch.from_numpy(random_dL(360, 640)).to(dev)
    bg = torch.zeros(3, device=dev)
    out = {}
    prev = _C.get_colour_mode()
    try:
        for m in (0, 2):
            _C.set_colour_mode(m)
            gd = g.to(dev, requires_grad=True)
            r = train_step.render_fused(cam.to(dev), gd, bg)
            (r["render"] * dL).sum().backward()
            torch.cuda.synchronize()
            out[m] = (r["render"].detach().cpu(), r["radii"].cpu(), [p.grad.cpu() for p in gd.params()])
    finally:
        _C.set_colour_mode(prev)
    assert torch.equal(out[0][0], out[2][0])
    assert torch.equal(out[0][1], out[2][1])
    for a, b in zip(out[0][2], out[2][2]):
        assert rel_l2(b.numpy(), a.numpy()) <= 1e-6
