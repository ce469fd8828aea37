"""The drop-in's full autograd path on the GPU: the reference-shaped render()
(gaussian_renderer/__init__.py:20-112, restated in train_step.render) through
GaussianRasterizer -> _RasterizeGaussians.backward -> the activations (exp, sigmoid,
normalize, the SH cat; or the Python SH / cov3D branch) -> the six leaf gradients
and viewspace_points.grad, against the CPU oracle's native gradients pushed through
torch autograd of the same activations on the CPU.  Both sides run the caller's activations on the GPU, so
the rasterizer sees bit-identical inputs and its integer decisions agree exactly."""
import math

import numpy as np
import pytest
import torch

from helpers import rel_l2

pytestmark = pytest.mark.gpu

TOL = 1e-4


def _reference_grads(oracle, cam, g, dev, dL, python_branch, mt=False):
    """Leaf gradients of sum(image * dL): the reference's activations (the caller's
    torch ops, on the GPU as in the HIP run, so the rasterizer sees bit-identical
    inputs), the rasterizer forward/backward by the oracle in place of the native
    autograd Function, torch autograd through the activations for the rest."""
    import train_step

    leaves = [p.detach().to(dev).clone().requires_grad_(True) for p in g.params()]
    xyz, f_dc, f_rest, opac_l, scal_l, rot_l = leaves
    camd = cam.to(dev)
    opacity = torch.sigmoid(opac_l)
    feats = torch.cat((f_dc, f_rest), dim=1)
    kw = dict(scale_modifier=1.0, sh_degree=g.active_sh_degree, mt=mt)
    inputs, names = [xyz, opacity], ["dmeans3D", "dopacity"]
    if python_branch:
        shs_view = feats.transpose(1, 2).view(-1, 3, (g.max_sh_degree + 1) ** 2)
        dirs = xyz - camd.camera_center.repeat(feats.shape[0], 1)
        dirs = dirs / dirs.norm(dim=1, keepdim=True)
        colors = torch.clamp_min(train_step.eval_sh(g.active_sh_degree, shs_view, dirs) + 0.5, 0.0)
        cov3D = train_step.covariance(torch.exp(scal_l), 1.0, rot_l)
        kw.update(colors_precomp=colors.detach().cpu().numpy(), cov3D_precomp=cov3D.detach().cpu().numpy())
        inputs += [colors, cov3D]
        names += ["dcolors", "dcov3D"]
    else:
        scales = torch.exp(scal_l)
        rotations = torch.nn.functional.normalize(rot_l)
        kw.update(shs=feats.detach().cpu().numpy(), scales=scales.detach().cpu().numpy(),
                  rotations=rotations.detach().cpu().numpy())
        inputs += [feats, scales, rotations]
        names += ["dsh", "dscales", "drot"]
    f = oracle.forward(xyz.detach().cpu().numpy(), opacity.detach().cpu().numpy(), cam.world_view_transform.numpy(),
                       cam.full_proj_transform.numpy(), cam.camera_center.numpy(), np.zeros(3, np.float32),
                       cam.image_height, cam.image_width, math.tan(cam.FoVx * 0.5), math.tan(cam.FoVy * 0.5), **kw)
    b = oracle.backward(f, dL)
    torch.autograd.backward(inputs, [torch.from_numpy(np.ascontiguousarray(b[n])).to(dev).reshape(x.shape)
                                     for n, x in zip(names, inputs)])
    return f, [p.grad.cpu() for p in leaves], b["dmeans2D"]


def _hip_grads(cam, g, dev, dL, python_branch):
    import train_step

    gd = g.to(dev, requires_grad=True)
    out = train_step.render(cam.to(dev), gd, torch.zeros(3, device=dev), convert_SHs_python=python_branch,
                            compute_cov3D_python=python_branch)
    (out["render"] * torch.from_numpy(dL).to(dev)).sum().backward()
    torch.cuda.synchronize()
    return out, [p.grad.cpu() for p in gd.params()], out["viewspace_points"].grad.cpu().numpy()


def _check(oracle, cam, g, dev, python_branch, mt=False):
    from helpers import random_dL

    dL = random_dL(cam.image_height, cam.image_width)
    f, ref, ref_vs = _reference_grads(oracle, cam, g, dev, dL, python_branch, mt)
    out, got, got_vs = _hip_grads(cam, g, dev, dL, python_branch)
    assert np.abs(out["render"].detach().cpu().numpy() - f["color"]).max() <= 1e-4
    np.testing.assert_array_equal(out["radii"].cpu().numpy(), f["radii"])
    errs = {n: rel_l2(a.numpy(), r.numpy()) for n, a, r in
            zip(("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"), got, ref)}
    errs["viewspace_points"] = rel_l2(got_vs, ref_vs)
    assert not np.any(got_vs[:, 2]), "dmeans2D's third column is 0 upstream"
    bad = {k: v for k, v in errs.items() if not v <= TOL}
    assert not bad, f"leaf gradients off: {bad} (all {errs})"


@pytest.mark.parametrize("python_branch", [False, True], ids=["native_sh_cov", "python_sh_cov"])
def test_autograd_path_config_b(dev, oracle, python_branch):
    """Config B (100k Gaussians, 800x800, SH3) through the drop-in autograd Function."""
    from helpers import case

    cam, g = case(100_000, 800, 800, 3, seed=1, view=0)
    _check(oracle, cam, g, dev, python_branch)


@pytest.mark.slow
@pytest.mark.timeout(600)
@pytest.mark.parametrize("python_branch", [False, True], ids=["native_sh_cov", "python_sh_cov"])
def test_autograd_path_config_c(dev, oracle, python_branch):
    """Config C (1M Gaussians, 1920x1080, SH3), the headline unit's autograd path."""
    from helpers import case

    cam, g = case(1_000_000, 1920, 1080, 3, seed=0, view=0)
    _check(oracle, cam, g, dev, python_branch, mt=True)


def test_noncontiguous_inputs_match_contiguous(dev):
    """Inputs that are strided views (upstream's C++ glue calls .contiguous() on each)
    give the same image and the same gradients as contiguous copies: the forward's
    validated inputs, contiguous copies included, are what the backward reuses."""
    import math

    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from helpers import case, random_dL

    cam, g = case(10_000, 256, 256, 3, seed=3, view=2)
    camd = cam.to(dev)
    dL = torch.from_numpy(random_dL(256, 256)).to(dev)
    base = {n: t.detach().to(dev) for n, t in (("xyz", g.get_xyz), ("sh", g.get_features), ("op", g.get_opacity),
                                              ("sc", g.get_scaling), ("rot", g.get_rotation))}
    settings = GaussianRasterizationSettings(
        image_height=256, image_width=256, tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5),
        bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=camd.world_view_transform,
        projmatrix=camd.full_proj_transform, sh_degree=3, campos=camd.camera_center, prefiltered=False, debug=False)

    def run(strided):
        leaves, inputs = {}, {}
        for n, t in base.items():
            if strided:  # the same values as a view with a padded last dim (or a transposed layout for sh)
                if n == "sh":
                    wide = t.transpose(1, 2).contiguous().requires_grad_(True)
                    leaves[n], inputs[n] = wide, wide.transpose(1, 2)
                else:
                    wide = torch.cat([t, torch.zeros_like(t[:, :1])], 1).requires_grad_(True)
                    leaves[n], inputs[n] = wide, wide[:, :t.shape[1]]
            else:
                leaves[n] = inputs[n] = t.clone().requires_grad_(True)
            assert inputs[n].is_contiguous() != strided, n
        means2D = torch.zeros_like(inputs["xyz"], requires_grad=True)
        img, radii = GaussianRasterizer(settings)(means3D=inputs["xyz"], means2D=means2D, opacities=inputs["op"],
                                                  shs=inputs["sh"], scales=inputs["sc"], rotations=inputs["rot"])
        (img * dL).sum().backward()
        grads = {}
        for n, t in base.items():
            gr = leaves[n].grad
            grads[n] = (gr.transpose(1, 2) if n == "sh" else gr[:, :t.shape[1]]) if strided else gr
        return img.detach(), radii, grads, means2D.grad

    img0, r0, g0, m0 = run(False)
    img1, r1, g1, m1 = run(True)
    assert torch.equal(img0, img1) and torch.equal(r0, r1)
    for n in g0:  # accumulator atomics reorder sums run to run: rel-L2, not bits
        assert rel_l2(g1[n].cpu().numpy(), g0[n].cpu().numpy()) <= 1e-5, n
    assert rel_l2(m1.cpu().numpy(), m0.cpu().numpy()) <= 1e-5


def test_second_backward_with_retain_graph(dev):
    """Two backward passes of ONE forward (retain_graph=True) give the same gradients:
    the backward's first launch files the quadrants for render_bwd's wave order once
    per forward (bwd_prepare_kernel); the second pass finds them filed and reuses them
    (filing again would overflow the order lists)."""
    import math

    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from helpers import case, random_dL

    cam, g = case(20_000, 320, 240, 3, seed=4, view=1)
    camd = cam.to(dev)
    dL = torch.from_numpy(random_dL(240, 320)).to(dev)
    leaves = {n: t.detach().to(dev).clone().requires_grad_(True) for n, t in (
        ("xyz", g.get_xyz), ("sh", g.get_features), ("op", g.get_opacity), ("sc", g.get_scaling),
        ("rot", g.get_rotation))}
    settings = GaussianRasterizationSettings(
        image_height=240, image_width=320, tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5),
        bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=camd.world_view_transform,
        projmatrix=camd.full_proj_transform, sh_degree=3, campos=camd.camera_center, prefiltered=False, debug=False)
    means2D = torch.zeros_like(leaves["xyz"], requires_grad=True)
    img, _ = GaussianRasterizer(settings)(means3D=leaves["xyz"], means2D=means2D, opacities=leaves["op"],
                                          shs=leaves["sh"], scales=leaves["sc"], rotations=leaves["rot"])
    loss = (img * dL).sum()
    loss.backward(retain_graph=True)
    first = {n: t.grad.clone() for n, t in leaves.items()}
    for t in leaves.values():
        t.grad = None
    loss.backward()
    for n, t in leaves.items():
        assert torch.isfinite(t.grad).all(), n
        assert rel_l2(t.grad.cpu().numpy(), first[n].cpu().numpy()) <= 1e-5, n


def test_repeated_small_scene_backward(dev):
    """A one-block scene (P <= 256: the preprocess grid is a single workgroup) run
    forward + backward repeatedly gives the same gradients every time: the
    preprocess clears the backward's "filed" flag in scratch memory that the caching
    allocator hands back from the previous iteration (render_bwd sets it)."""
    import math

    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from helpers import case, random_dL

    cam, g = case(200, 64, 64, 3, seed=6, view=0)
    camd = cam.to(dev)
    dL = torch.from_numpy(random_dL(64, 64)).to(dev)
    settings = GaussianRasterizationSettings(
        image_height=64, image_width=64, tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5),
        bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=camd.world_view_transform,
        projmatrix=camd.full_proj_transform, sh_degree=3, campos=camd.camera_center, prefiltered=False, debug=False)
    runs = []
    for _ in range(3):
        leaves = {n: t.detach().to(dev).clone().requires_grad_(True) for n, t in (
            ("xyz", g.get_xyz), ("sh", g.get_features), ("op", g.get_opacity), ("sc", g.get_scaling),
            ("rot", g.get_rotation))}
        means2D = torch.zeros_like(leaves["xyz"], requires_grad=True)
        img, _ = GaussianRasterizer(settings)(means3D=leaves["xyz"], means2D=means2D, opacities=leaves["op"],
                                              shs=leaves["sh"], scales=leaves["sc"], rotations=leaves["rot"])
        (img * dL).sum().backward()
        runs.append({n: t.grad.cpu().numpy() for n, t in leaves.items()})
        del img, leaves, means2D
    assert np.abs(runs[0]["op"]).sum() > 0
    for r in runs[1:]:
        for n in r:
            assert rel_l2(r[n], runs[0][n]) <= 1e-5, n
