"""Pin the oracle's analytic backward (restated from upstream backward.cu) against
float64 autograd of a dense torch restatement of the same forward.

The torch forward below is a second, independent statement of SURVEY.md
A.2-A.6 (projection, cov3D/EWA cov2D, conic, SH colour, front-to-back
compositing over the oracle's depth-sorted tile lists).  Discrete decisions
(visibility, tile membership) come from the oracle; the blend masks are
re-evaluated in float64.  Scenes are chosen away from the A.9 deviations: no
pixel saturates (T stays above 1e-4), opacities stay below the 0.99 clamp.
Upstream quirks that the comparison must respect:
  * dL/dscale is w.r.t. scale_modifier*scale (backward.cu computeCov3D) -> the
    autograd leaf is the modified scale (tested with scale_modifier = 1 and 1.5);
  * dL/drot is w.r.t. the quaternion as given (no normalisation Jacobian);
  * dL/dmeans2D is the gradient w.r.t. NDC xy (pixel gradient x W/2, H/2).
"""
import math

import numpy as np
import pytest
import torch

import synthetic
from helpers import rel_l2

torch.set_default_dtype(torch.float32)

SH_C = dict(
    C0=0.28209479177387814, C1=0.4886025119029199,
    C2=(1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396),
    C3=(-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
        1.445305721320277, -0.5900435899266435))


def sh_rgb(deg, sh, d):
    """sh [P,M,3], d [P,3] unit -> [P,3]"""
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    r = SH_C["C0"] * sh[:, 0]
    if deg > 0:
        r = r - SH_C["C1"] * y * sh[:, 1] + SH_C["C1"] * z * sh[:, 2] - SH_C["C1"] * x * sh[:, 3]
    if deg > 1:
        c = SH_C["C2"]
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        r = r + c[0] * xy * sh[:, 4] + c[1] * yz * sh[:, 5] + c[2] * (2 * zz - xx - yy) * sh[:, 6] + \
            c[3] * xz * sh[:, 7] + c[4] * (xx - yy) * sh[:, 8]
    if deg > 2:
        c = SH_C["C3"]
        r = r + c[0] * y * (3 * xx - yy) * sh[:, 9] + c[1] * xy * z * sh[:, 10] + \
            c[2] * y * (4 * zz - xx - yy) * sh[:, 11] + c[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12] + \
            c[4] * x * (4 * zz - xx - yy) * sh[:, 13] + c[5] * z * (xx - yy) * sh[:, 14] + \
            c[6] * x * (xx - 3 * yy) * sh[:, 15]
    return r


def torch_forward(leaf, cam, ref, deg, bg, mod, python_branch):
    f64 = torch.float64
    view = torch.as_tensor(cam.world_view_transform.numpy().reshape(16), dtype=f64)
    proj = torch.as_tensor(cam.full_proj_transform.numpy().reshape(16), dtype=f64)
    A = view.reshape(4, 4).T  # p_view = A [x,1] (matrices read column-major, auxiliary.h)
    Pm = proj.reshape(4, 4).T
    W, H = cam.image_width, cam.image_height
    tanx = float(np.float32(math.tan(cam.FoVx * 0.5)))
    tany = float(np.float32(math.tan(cam.FoVy * 0.5)))
    fx = float(np.float32(W) / (np.float32(2.0) * np.float32(tanx)))
    fy = float(np.float32(H) / (np.float32(2.0) * np.float32(tany)))
    m = leaf["means3D"]
    P = m.shape[0]
    hom = torch.cat([m, torch.ones(P, 1, dtype=f64)], 1)
    ph = hom @ Pm.T
    pw = 1.0 / (ph[:, 3:4] + 1e-7)
    ndc = ph[:, :2] * pw + leaf["means2D"]
    pix = torch.stack([((ndc[:, 0] + 1) * W - 1) * 0.5, ((ndc[:, 1] + 1) * H - 1) * 0.5], 1)
    t = hom @ A[:3].T
    if python_branch:
        c = leaf["cov3D"]
        Sig = torch.stack([c[:, 0], c[:, 1], c[:, 2], c[:, 1], c[:, 3], c[:, 4], c[:, 2], c[:, 4], c[:, 5]],
                          1).view(P, 3, 3)
    else:
        q = leaf["rotations"]
        r, x, y, z = q.unbind(1)
        R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                         2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                         2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], 1).view(P, 3, 3)
        L = R * leaf["scales"][:, None, :]  # scales leaf is already mod * scale
        Sig = L @ L.transpose(1, 2)
    limx, limy = 1.3 * tanx, 1.3 * tany
    tz = t[:, 2]
    tx = torch.clamp(t[:, 0] / tz, -limx, limx) * tz
    ty = torch.clamp(t[:, 1] / tz, -limy, limy) * tz
    zero = torch.zeros_like(tz)
    J = torch.stack([fx / tz, zero, -fx * tx / tz ** 2, zero, fy / tz, -fy * ty / tz ** 2], 1).view(P, 2, 3)
    Wr = A[:3, :3]
    JW = J @ Wr
    cov = JW @ Sig @ JW.transpose(1, 2)
    a = cov[:, 0, 0] + 0.3
    b = cov[:, 0, 1]
    cc = cov[:, 1, 1] + 0.3
    det = a * cc - b * b
    conic = torch.stack([cc / det, -b / det, a / det], 1)
    if python_branch:
        colors = leaf["colors"]
    else:
        campos = torch.as_tensor(cam.camera_center.numpy(), dtype=f64)
        d = m - campos
        d = d / d.norm(dim=1, keepdim=True)
        colors = torch.clamp_min(sh_rgb(deg, leaf["shs"], d) + 0.5, 0.0)
        colors.retain_grad()
        leaf["_colors"] = colors
    opac = leaf["opacities"].view(-1)
    bgt = torch.as_tensor(bg, dtype=f64)
    out = bgt[:, None, None].expand(3, H, W).clone()  # empty tiles show the background
    gx = (W + 15) // 16
    min_T = 1.0
    for tile in range(ref["ranges"].shape[0]):
        s, e = ref["ranges"][tile]
        if e <= s:
            continue
        ids = torch.as_tensor(ref["point_list"][s:e].astype(np.int64))
        tx0, ty0 = (tile % gx) * 16, (tile // gx) * 16
        yy, xx = torch.meshgrid(torch.arange(ty0, min(ty0 + 16, H)), torch.arange(tx0, min(tx0 + 16, W)),
                                indexing="ij")
        px = xx.reshape(-1).to(f64)
        py = yy.reshape(-1).to(f64)
        dx = pix[ids, 0][None, :] - px[:, None]
        dy = pix[ids, 1][None, :] - py[:, None]
        co = conic[ids]
        power = -0.5 * (co[None, :, 0] * dx * dx + co[None, :, 2] * dy * dy) - co[None, :, 1] * dx * dy
        alpha = opac[ids][None, :] * torch.exp(power)
        mask = (power <= 0) & (alpha >= 1.0 / 255.0)
        alpha = torch.where(mask, alpha, torch.zeros_like(alpha))
        one_m = 1 - alpha
        Tincl = torch.cumprod(one_m, dim=1)
        Texcl = torch.cat([torch.ones_like(Tincl[:, :1]), Tincl[:, :-1]], 1)
        min_T = min(min_T, float(Tincl[:, -1].detach().min()))
        C = (alpha * Texcl) @ colors[ids]  # [npix, 3]
        val = C + Tincl[:, -1:] * bgt[None, :]
        out[:, yy.reshape(-1), xx.reshape(-1)] = val.T
    return out, min_T


def make_leaves(g, python_branch, mod):
    f64 = torch.float64
    with torch.no_grad():
        leaf = dict(means3D=g.get_xyz.to(f64).clone(), opacities=g.get_opacity.to(f64).clone(),
                    means2D=torch.zeros(g.xyz.shape[0], 2, dtype=f64))
        if python_branch:
            from train_step import covariance

            leaf["cov3D"] = covariance(g.get_scaling.double(), mod, g.rotation.double()).clone()
            leaf["colors"] = torch.rand(g.xyz.shape[0], 3, generator=torch.Generator().manual_seed(3),
                                        dtype=f64)
        else:
            leaf["scales"] = (mod * g.get_scaling.to(f64)).clone()
            leaf["rotations"] = g.get_rotation.to(f64).clone()
            leaf["shs"] = g.get_features.to(f64).clone()
    for v in leaf.values():
        v.requires_grad_(True)
    return leaf


@pytest.mark.parametrize("python_branch,mod,deg,seed", [(False, 1.0, 3, 0), (False, 1.5, 2, 1), (True, 1.0, 0, 2),
                                                        (False, 1.0, 1, 3)])
def test_oracle_backward_matches_float64_autograd(oracle, python_branch, mod, deg, seed):
    W, H = 48, 40
    cam = synthetic.make_camera(W, H, view=seed % 8)
    g = synthetic.make_gaussians(40, deg, seed=seed, radius=1.5, scale_range=(0.1, 0.4))
    with torch.no_grad():
        g.opacity[:] = torch.logit(torch.rand(40, 1, generator=torch.Generator().manual_seed(seed)) * 0.5 + 0.1)
    bg = np.array([0.3, 0.1, 0.7], np.float32)
    leaf = make_leaves(g, python_branch, mod)
    kw = dict(scale_modifier=1.0 if python_branch else mod, sh_degree=deg)
    f32 = lambda t: t.detach().float().numpy()  # noqa: E731
    if python_branch:
        kw.update(colors_precomp=f32(leaf["colors"]), cov3D_precomp=f32(leaf["cov3D"]))
    else:
        kw.update(shs=f32(leaf["shs"]), scales=g.get_scaling.detach().numpy(), rotations=f32(leaf["rotations"]))
    ref = oracle.forward(f32(leaf["means3D"]), f32(leaf["opacities"]), cam.world_view_transform.numpy(),
                         cam.full_proj_transform.numpy(), cam.camera_center.numpy(), bg, H, W,
                         math.tan(cam.FoVx * 0.5), math.tan(cam.FoVy * 0.5), **kw)
    assert ref["num_rendered"] > 40
    out, min_T = torch_forward(leaf, cam, ref, deg, bg, mod, python_branch)
    assert min_T > 1e-3, "scene saturates; pick a sparser one"
    np.testing.assert_allclose(out.detach().numpy(), ref["color"], atol=2e-5)
    dL = np.random.default_rng(seed).standard_normal((3, H, W))
    (out * torch.as_tensor(dL)).sum().backward()
    rb = oracle.backward(ref, dL.astype(np.float32))
    vis = ref["radii"] > 0
    checks = {"dmeans3D": leaf["means3D"].grad, "dopacity": leaf["opacities"].grad,
              "dmeans2D": leaf["means2D"].grad}
    if python_branch:
        checks.update(dcov3D=leaf["cov3D"].grad, dcolors=leaf["colors"].grad)
    else:
        checks.update(dscales=leaf["scales"].grad, drot=leaf["rotations"].grad, dsh=leaf["shs"].grad,
                      dcolors=leaf["_colors"].grad)
    errs = {}
    for name, auto in checks.items():
        got = rb[name][:, :2] if name == "dmeans2D" else rb[name]
        errs[name] = rel_l2(got[vis], auto.numpy()[vis])
    assert all(v < 2e-4 for v in errs.values()), errs
