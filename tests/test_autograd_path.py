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
