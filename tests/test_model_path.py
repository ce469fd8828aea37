"""The rasterizer over GaussianModel's stored parameters (diff_gaussian_rasterization
.rasterize_model, train_step.render_fused) against the reference glue
(train_step.render: torch's sigmoid / exp / F.normalize and the SH cat, then the
rasterizer), and the fused L1 loss against the reference's torch L1.

The library applies the activations with torch's operations in torch's order
(include/gsr.h gsr_activations), so the forward must equal the reference glue's bit
for bit (image, radii).  Gradients: the render backward's accumulator atomics add in
a run-dependent order, so two runs of either path differ in the last bits; the two
paths are held to that noise floor (rel-L2 within 4e-6 or 4x the run-to-run spread),
except the deterministic isolated-Gaussian scene, where they must be equal bit for
bit.  The reference glue itself is pinned to the CPU oracle by test_gpu_parity.py /
test_leaf_grads.py; the oracle check here is direct, at a small size."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import diff_gaussian_rasterization as dgr

NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")


def _run(cam, g, dev, dL, glue, bg=(0.0, 0.0, 0.0), grad=True):
    import train_step

    gd = g.to(dev, requires_grad=grad)
    bg_t = torch.tensor(bg, dtype=torch.float32, device=dev)
    render = train_step.render_fused if glue == "fused" else train_step.render
    out = render(cam.to(dev), gd, bg_t)
    res = {"image": out["render"].detach().cpu(), "radii": out["radii"].cpu()}
    if grad:
        (out["render"] * dL).sum().backward()
        torch.cuda.synchronize()
        res["grads"] = [p.grad.cpu() for p in gd.params()]
        res["means2D"] = out["viewspace_points"].grad.cpu()
        res["plan"] = dgr.last_leaf_plan
    return res


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [(20_000, 320, 240, 3), (100_000, 800, 800, 3), (30_000, 256, 192, 1),
                                 (20_000, 320, 240, 0)], ids=["small", "B", "deg1", "deg0"])
def test_model_path_equals_reference_glue(dev, cfg):
    """Forward bit for bit (the in-kernel activations are torch's), gradients of all
    six leaves and of the screen-space means within the atomics' run-to-run spread."""
    from helpers import case, random_dL

    P, W, H, deg = cfg
    cam, g = case(P, W, H, deg, seed=5, view=3)
    dL = torch.from_numpy(random_dL(H, W)).to(dev)
    ref = _run(cam, g, dev, dL, "reference")
    ref2 = _run(cam, g, dev, dL, "reference")
    got = _run(cam, g, dev, dL, "fused")
    assert torch.equal(got["radii"], ref["radii"])
    assert torch.equal(got["image"], ref["image"]), float((got["image"] - ref["image"]).abs().max())
    assert got["plan"] == ("means3D", "opacities", "rotations", "scales", "sh")
    for name, a, b, b2 in zip(NAMES, got["grads"], ref["grads"], ref2["grads"]):
        assert a.shape == b.shape and a.dtype == b.dtype, name
        if b.numel() == 0:  # degree 0: _features_rest has no coefficients
            continue
        noise = _rel(b2, b) if float(b.abs().max()) > 0 else 0.0
        assert _rel(a, b) <= max(4e-6, 4 * noise), (name, _rel(a, b), noise)
    assert _rel(got["means2D"], ref["means2D"]) <= 4e-6


@pytest.mark.gpu
def test_model_path_bit_identical_on_isolated_scene(dev):
    """Gaussians that never share a pixel: the accumulator atomics have one addend
    each, so both paths are deterministic and must agree bit for bit — the stored
    parameters' gradients through the in-kernel activations' backwards equal torch's
    exp / sigmoid / normalize / cat backwards."""
    from helpers import random_dL
    from test_leaf_grads import _isolated_scene

    cam, g = _isolated_scene()
    dL = torch.from_numpy(random_dL(cam.image_height, cam.image_width)).to(dev) * 1e4
    ref = _run(cam, g, dev, dL, "reference")
    got = _run(cam, g, dev, dL, "fused")
    assert torch.equal(got["image"], ref["image"]) and torch.equal(got["radii"], ref["radii"])
    for name, a, b in zip(NAMES, got["grads"], ref["grads"]):
        assert float(b.abs().max()) > 0, name
        if name == "rotation":  # the reference's normalize backward sums through torch's reduction
            assert float((a - b).abs().max()) <= 8 * 2.0 ** -23 * float(b.abs().max()), name
            continue
        assert torch.equal(a, b), (name, float((a - b).abs().max()))
    assert torch.equal(got["means2D"], ref["means2D"])


@pytest.mark.gpu
def test_model_path_against_oracle(dev):
    """Direct oracle check of the model path at a small size: radii exact, image within
    1e-4, dmeans2D within rel-L2 1e-4 (the oracle gets torch's activations on the CPU)."""
    import math

    from helpers import case, random_dL
    from oracle import oracle

    P, W, H = 3_000, 128, 96
    cam, g = case(P, W, H, 3, seed=11, view=1)
    dL = random_dL(H, W)
    got = _run(cam, g, dev, torch.from_numpy(dL).to(dev), "fused")
    ref = oracle.forward(g.get_xyz.numpy(), g.get_opacity.detach().numpy(), cam.world_view_transform.numpy(),
                         cam.full_proj_transform.numpy(), cam.camera_center.numpy(), np.zeros(3), H, W,
                         math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), 1.0, 3, shs=g.get_features.detach().numpy(),
                         scales=g.get_scaling.detach().numpy(), rotations=g.get_rotation.detach().numpy())
    np.testing.assert_array_equal(got["radii"].numpy(), ref["radii"])
    assert float(np.abs(got["image"].numpy() - ref["color"]).max()) <= 1e-4
    refb = oracle.backward(ref, dL.astype(np.float32))
    m2 = got["means2D"].numpy()
    assert np.linalg.norm(m2 - refb["dmeans2D"]) / np.linalg.norm(refb["dmeans2D"]) <= 1e-4


@pytest.mark.gpu
def test_model_path_forward_only_and_background(dev):
    """No-grad render (config E's shape, small) and a non-zero background: same image."""
    from helpers import case

    cam, g = case(20_000, 320, 240, 3, seed=7, view=5)
    with torch.no_grad():
        a = _run(cam, g, dev, None, "fused", bg=(0.2, 0.5, 1.0), grad=False)
        b = _run(cam, g, dev, None, "reference", bg=(0.2, 0.5, 1.0), grad=False)
    assert torch.equal(a["image"], b["image"]) and torch.equal(a["radii"], b["radii"])


@pytest.mark.gpu
def test_model_path_accumulates_into_existing_grads(dev):
    """Two renders into one backward and a pre-existing .grad: autograd accumulates
    the model path's leaf gradients like the reference glue's."""
    import train_step
    from helpers import case, random_dL

    cam, g = case(20_000, 320, 240, 3, seed=8, view=2)
    dL = torch.from_numpy(random_dL(240, 320)).to(dev)
    res = {}
    for glue in ("reference", "fused"):
        gd = g.to(dev, requires_grad=True)
        for p in gd.params():
            p.grad = torch.full_like(p, 0.25)
        render = train_step.render_fused if glue == "fused" else train_step.render
        loss = sum((render(cam.to(dev), gd, torch.zeros(3, device=dev), scaling_modifier=s)["render"] * dL).sum()
                   for s in (1.0, 1.1))
        loss.backward()
        torch.cuda.synchronize()
        res[glue] = [p.grad.cpu() for p in gd.params()]
    for name, a, b in zip(NAMES, res["fused"], res["reference"]):
        assert _rel(a, b) <= 4e-6, (name, _rel(a, b))


@pytest.mark.gpu
def test_fused_l1_loss_matches_torch(dev):
    """train_ops.l1_ssim_loss with lambda 0 (the L1-only kernel): the loss equals
    torch's abs(x - y).mean() to float rounding, the image gradient bit for bit
    (MeanBackward then AbsBackward: sign(x - y) / N), including exact ties."""
    import train_ops

    g = torch.Generator().manual_seed(3)
    x = torch.rand(3, 1080, 1920, generator=g).to(dev)
    y = torch.rand(3, 1080, 1920, generator=g).to(dev)
    y[0, :4, :] = x[0, :4, :]  # d == 0: sign 0
    xr = x.clone().requires_grad_(True)
    ref = torch.abs(xr - y).mean()
    ref.backward()
    xf = x.clone().requires_grad_(True)
    got = train_ops.l1_ssim_loss(xf, y, 0.0)
    got.backward()
    torch.cuda.synchronize()
    assert abs(float(got) - float(ref)) <= 2e-6 * float(ref)
    assert torch.equal(xf.grad, xr.grad)
    # odd length: the tail that is not a multiple of 4
    x3, y3 = x[:, :7, :5].contiguous().requires_grad_(True), y[:, :7, :5].contiguous()
    l3 = train_ops.l1_ssim_loss(x3, y3, 0.0)
    l3.backward()
    x3r = x3.detach().clone().requires_grad_(True)
    torch.abs(x3r - y3).mean().backward()
    assert torch.equal(x3.grad, x3r.grad)
    assert abs(float(l3) - float(torch.abs(x3r - y3).mean())) <= 1e-6


@pytest.mark.gpu
def test_train_step_glues_agree(dev):
    """The bench's unit with both glues: same loss (to rounding), same image."""
    import train_step
    from helpers import case

    cam, g = case(50_000, 480, 360, 3, seed=9, view=4)
    target = torch.rand(3, 360, 480, generator=torch.Generator().manual_seed(2)).to(dev)
    outs = {}
    for glue in ("reference", "fused"):
        gd = g.to(dev, requires_grad=True)
        o = train_step.train_step(cam.to(dev), gd, target, torch.zeros(3, device=dev), glue=glue)
        torch.cuda.synchronize()
        outs[glue] = (float(o["loss"]), o["render"].detach().cpu(), [p.grad.cpu() for p in gd.params()])
    assert abs(outs["fused"][0] - outs["reference"][0]) <= 1e-6 * outs["reference"][0]
    assert torch.equal(outs["fused"][1], outs["reference"][1])
    for name, a, b in zip(NAMES, outs["fused"][2], outs["reference"][2]):
        assert _rel(a, b) <= 1e-5, (name, _rel(a, b))


def _l1_run(cam, g, dev, gt, fused, extra=None):
    """render_fused -> L1 against gt (+ sum(image * extra)) -> backward; fused: the
    loss out of the rasterizer (rasterize_model(l1_target=...), the render backward
    forming the L1 pixel gradient), else train_ops' L1 kernel on the image."""
    import train_ops
    import train_step

    gd = g.to(dev, requires_grad=True)
    out = train_step.render_fused(cam.to(dev), gd, torch.zeros(3, device=dev), l1_target=gt if fused else None)
    loss = out["l1"] if fused else train_ops.l1_ssim_loss(out["render"], gt, 0.0)
    total = loss if extra is None else loss + (out["render"] * extra).sum()
    total.backward()
    torch.cuda.synchronize()
    return (loss.detach().cpu(), out["render"].detach().cpu(), [p.grad.cpu() for p in gd.params()],
            out["viewspace_points"].grad.cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("mixed", [False, True], ids=["loss_only", "image_also_used"])
def test_rasterizer_l1_seed_bit_identical_on_isolated_scene(dev, mixed):
    """The L1 loss out of the rasterizer (gsr.h GSR_FLAG_L1_SEED: the render backward
    forms (dloss / n) sign(image - gt) per pixel) against the separate L1 kernel and its
    gradient map: same loss bits, and — one atomic addend per accumulator row on this
    scene — the same gradient bits.  ``image_also_used``: the image feeds a second term
    too, so the backward adds the L1 map to that gradient instead (same bits)."""
    from helpers import random_dL
    from test_leaf_grads import _isolated_scene

    cam, g = _isolated_scene()
    H, W = cam.image_height, cam.image_width
    gt = torch.rand(3, H, W, generator=torch.Generator().manual_seed(4)).to(dev)
    extra = torch.from_numpy(random_dL(H, W)).to(dev) if mixed else None
    a = _l1_run(cam, g, dev, gt, True, extra)
    b = _l1_run(cam, g, dev, gt, False, extra)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    for name, x, y in zip(NAMES, a[2], b[2]):
        assert float(y.abs().max()) > 0, name
        assert torch.equal(x, y), (name, float((x - y).abs().max()))
    assert torch.equal(a[3], b[3])


@pytest.mark.gpu
def test_rasterizer_l1_seed_general_scene(dev):
    """The same at a shared-pixel scene: loss bits equal, gradients within the
    accumulator atomics' run-to-run spread."""
    from helpers import case

    cam, g = case(50_000, 480, 360, 3, seed=9, view=4)
    gt = torch.rand(3, 360, 480, generator=torch.Generator().manual_seed(2)).to(dev)
    a = _l1_run(cam, g, dev, gt, True)
    b = _l1_run(cam, g, dev, gt, False)
    b2 = _l1_run(cam, g, dev, gt, False)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    for name, x, y, y2 in zip(NAMES, a[2], b[2], b2[2]):
        noise = _rel(y2, y)
        assert _rel(x, y) <= max(4e-6, 4 * noise), (name, _rel(x, y), noise)


@pytest.mark.gpu
@pytest.mark.parametrize("grad", [True, False], ids=["prepared", "no_grad"])
def test_rasterizer_l1_loss_bits(dev, grad):
    """gsr_forward_render_l1's loss — its partial sums in the backward preparation's
    launch (a forward that will be differentiated) or in the L1 kernel of its own —
    equals train_ops' L1 kernel on the same image bit for bit (one block decomposition,
    gsr_l1.hpp), and an empty scene gives mean|gt| over upstream's zero image."""
    import math

    import synthetic
    import train_ops
    import train_step
    from diff_gaussian_rasterization import _C
    from helpers import case

    cam, g = case(20_000, 320, 240, 3, seed=5, view=1)
    gt = torch.rand(3, 240, 320, generator=torch.Generator().manual_seed(8)).to(dev)
    gd = g.to(dev, requires_grad=grad)
    with torch.set_grad_enabled(grad):
        out = train_step.render_fused(cam.to(dev), gd, torch.zeros(3, device=dev), l1_target=gt)
    ref = train_ops.l1_ssim_loss(out["render"].detach(), gt, 0.0)
    torch.cuda.synchronize()
    assert torch.equal(out["l1"].detach(), ref)
    vis = out["visibility_filter"]
    assert vis.dtype == torch.bool and torch.equal(vis, out["radii"] > 0) and int(vis.sum()) > 0
    cam0 = synthetic.make_camera(64, 48, view=0).to(dev)
    gt0 = gt[:, :48, :64].contiguous()
    z3, z1, z4 = (torch.zeros(0, k, device=dev) for k in (3, 1, 4))
    res = _C._rasterize(torch.zeros(3, device=dev), z3, torch.empty(0, device=dev), z1, z3, z4, 1.0,
                        torch.empty(0, device=dev), cam0.world_view_transform, cam0.full_proj_transform,
                        math.tan(cam0.FoVx * 0.5), math.tan(cam0.FoVy * 0.5), 48, 64, torch.zeros(0, 1, 3, device=dev),
                        0, cam0.camera_center, False, False, l1_target=gt0)
    assert res[0] == 0 and float(res[1].abs().max()) == 0.0
    assert torch.equal(res[7], train_ops.l1_ssim_loss(torch.zeros_like(gt0), gt0, 0.0))
