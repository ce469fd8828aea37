"""The reference's own ``gaussian_renderer.render()`` (gaussian_renderer/__init__.py:20-112),
imported unmodified from /root/reference, drives this package's
``diff_gaussian_rasterization`` surface end to end on CPU.

On CPU the native library cannot run, so ``_C``'s three entry points are replaced by
an oracle-backed shim with the same positional signatures; everything above ``_C`` —
settings NamedTuple, GaussianRasterizer argument checks, the empty-tensor convention,
the autograd Function's save/restore and its mapping of the 8 native gradients onto
the 9 inputs — is the real package.  Checked: the image, ``viewspace_points.grad``
(densification input, scene/gaussian_model.py:576-580) and every leaf gradient of the
GaussianModel storage, for both the native and the Python SH/cov3D branches.
Skipped where the reference is not mounted (the GPU box)."""
import importlib.util
import math
import sys
import types

import numpy as np
import pytest
import torch

from conftest import REFERENCE

pytestmark = pytest.mark.skipif(not (REFERENCE / "gaussian_renderer" / "__init__.py").exists(),
                                reason="reference not mounted")

NAMES = ("dmeans2D", "dcolors", "dopacity", "dmeans3D", "dcov3D", "dsh", "dscales", "drot")


class OracleC:
    """Same signatures as diff_gaussian_rasterization._C, computed by the CPU oracle."""

    def __init__(self, oracle):
        self.o = oracle
        self.states = {}
        self.calls = []

    @staticmethod
    def _np(t):
        return None if t is None or t.numel() == 0 else t.detach().cpu().numpy()

    def rasterize_gaussians(self, bg, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                            viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                            prefiltered, debug):
        self.calls.append("fwd")
        n = self._np
        f = self.o.forward(n(means3D), n(opacity), n(viewmatrix), n(projmatrix), n(campos), n(bg), image_height,
                           image_width, tan_fovx, tan_fovy, scale_modifier, degree, shs=n(sh),
                           colors_precomp=n(colors), scales=n(scales), rotations=n(rotations),
                           cov3D_precomp=n(cov3D_precomp), prefiltered=prefiltered)
        key = len(self.states)
        self.states[key] = f
        tag = torch.tensor([key])
        return f["num_rendered"], torch.from_numpy(f["color"]), torch.from_numpy(f["radii"]), tag, tag.clone(), \
            tag.clone()

    def _rasterize(self, *args, **kw):  # the autograd Function's entry: + its validated inputs (none here)
        return (*self.rasterize_gaussians(*args), None)

    def rasterize_gaussians_backward(self, bg, means3D, radii, colors, scales, rotations, scale_modifier,
                                     cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, sh,
                                     degree, campos, geomBuffer, R, binningBuffer, imageBuffer, debug,
                                     dsh_planar=False, leaf=None, opacities=None, inputs=None):
        self.calls.append("bwd")
        f = self.states[int(geomBuffer[0])]
        assert R == f["num_rendered"]
        b = self.o.backward(f, dL_dout_color.detach().cpu().numpy())
        self.last_grads = b
        out = [torch.from_numpy(b[k]) for k in NAMES]
        if dsh_planar:  # the library's coefficient-plane layout: same values, strides (3, 3P, 1)
            i = NAMES.index("dsh")
            out[i] = out[i].permute(1, 0, 2).contiguous().permute(1, 0, 2)
        self.last_leaf = None
        if leaf is not None:  # gsr_leaf_grads: the leaves' gradients written in place of dsh/dopacity/dscales/drot
            n = self._np
            lg = self.o.activation_leaf_grads(b["dsh"], b["dopacity"], b["dscales"], b["drot"],
                                              n(opacities) if opacities is not None else b["dopacity"],
                                              n(scales) if scales.numel() else b["dscales"],
                                              n(rotations) if rotations.numel() else b["drot"],
                                              n(leaf.rotation_norm) if leaf.rotation_norm is not None
                                              else np.ones(len(b["drot"]), np.float32), leaf.rotation_eps,
                                              sum_order="sequential")  # as CPU torch adds (its GPU reduction pairs)
            self.last_leaf = []
            for name, bit, idx in (("dsh_dc", 1, "dsh"), ("dsh_rest", 1, "dsh"), ("dscaling", 2, "dscales"),
                                   ("dopacity", 4, "dopacity"), ("drotation", 8, "drot")):
                t = getattr(leaf, name)
                if t is None:
                    continue
                v = torch.from_numpy(lg[name]).reshape(t.shape)
                t.copy_(t + v if leaf.accumulate & bit else v)
                out[NAMES.index(idx)] = None
                self.last_leaf.append(name)
        return tuple(out)

    def mark_visible(self, means3D, viewmatrix, projmatrix):
        return torch.from_numpy(self.o.mark_visible(self._np(means3D), self._np(viewmatrix)))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, str(path))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


class _CpuDevice:
    """The reference hard-codes device='cuda' (gaussian_renderer/__init__.py:35,
    utils/general_utils.py:73,104,120); map it to CPU while it runs here."""

    def __enter__(self):
        self.saved = {}
        for name in ("zeros", "zeros_like"):
            fn = getattr(torch, name)
            self.saved[name] = fn

            def wrap(*a, _fn=fn, **k):
                if k.get("device") == "cuda":
                    k["device"] = "cpu"
                return _fn(*a, **k)

            setattr(torch, name, wrap)

    def __exit__(self, *exc):
        for k, v in self.saved.items():
            setattr(torch, k, v)


@pytest.fixture
def reference_render(monkeypatch, oracle):
    import diff_gaussian_rasterization as dgr

    shim = OracleC(oracle)
    for fn in ("rasterize_gaussians", "_rasterize", "rasterize_gaussians_backward", "mark_visible"):
        monkeypatch.setattr(dgr._C, fn, getattr(shim, fn))
    monkeypatch.setitem(sys.modules, "diff_gaussian_rasterization", dgr)
    scene_pkg = types.ModuleType("scene")
    gm = types.ModuleType("scene.gaussian_model")
    gm.GaussianModel = object
    monkeypatch.setitem(sys.modules, "scene", scene_pkg)
    monkeypatch.setitem(sys.modules, "scene.gaussian_model", gm)
    monkeypatch.setitem(sys.modules, "utils", types.ModuleType("utils"))
    sh_utils = _load("utils.sh_utils", REFERENCE / "utils" / "sh_utils.py")
    gu = _load("ref_general_utils", REFERENCE / "utils" / "general_utils.py")
    mod = _load("ref_gaussian_renderer", REFERENCE / "gaussian_renderer" / "__init__.py")
    return mod.render, shim, gu, sh_utils


class Pipe:
    def __init__(self, sh_py, cov_py):
        self.convert_SHs_python = sh_py
        self.compute_cov3D_python = cov_py
        self.debug = False


@pytest.mark.parametrize("branch", ["native", "python"])
def test_reference_render_through_drop_in(reference_render, branch):
    import synthetic

    render, shim, gu, _ = reference_render
    cam = synthetic.make_camera(96, 64, view=1)
    pc = synthetic.make_gaussians(300, sh_degree=3, seed=7, radius=1.2, scale_range=(0.02, 0.1), active_sh_degree=2)
    for p in pc.params():
        p.requires_grad_(True)

    def get_covariance(scaling_modifier=1.0):  # GaussianModel.get_covariance (scene/gaussian_model.py:128-129)
        with _CpuDevice():
            L = gu.build_scaling_rotation(scaling_modifier * pc.get_scaling, pc.rotation)
            return gu.strip_symmetric(L @ L.transpose(1, 2))

    pc.get_covariance = get_covariance
    sh_py = cov_py = branch == "python"
    bg = torch.tensor([0.1, 0.2, 0.3])
    with _CpuDevice():
        out = render(cam, pc, Pipe(sh_py, cov_py), bg)
    img = out["render"]
    assert img.shape == (3, 64, 96) and out["radii"].dtype == torch.int32
    assert torch.equal(out["visibility_filter"], out["radii"] > 0)
    state = shim.states[len(shim.states) - 1]
    np.testing.assert_array_equal(img.detach().numpy(), state["color"])
    dL = torch.from_numpy(np.random.default_rng(0).standard_normal((3, 64, 96)).astype(np.float32))
    (img * dL).sum().backward()
    assert shim.calls == ["fwd", "bwd"]
    b = shim.last_grads
    # the reference's own graph (get_features cat, exp, sigmoid, normalize) takes the
    # fused leaf gradients (diff_gaussian_rasterization._leaf_plan)
    assert shim.last_leaf == (["dsh_dc", "dsh_rest", "dscaling", "dopacity", "drotation"] if branch == "native"
                              else ["dopacity"])
    # densification statistic input (train.py:127 -> gaussian_model.py:576-580)
    np.testing.assert_array_equal(out["viewspace_points"].grad.numpy(), b["dmeans2D"])
    vis = state["radii"] > 0
    assert vis.sum() > 50
    if branch == "native":
        np.testing.assert_allclose(pc.xyz.grad.numpy(), b["dmeans3D"], rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(pc.features_dc.grad.numpy(), b["dsh"][:, :1], rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(pc.features_rest.grad.numpy(), b["dsh"][:, 1:], rtol=1e-6, atol=1e-9)
        x = pc.opacity.detach().requires_grad_()
        (ref_op,) = torch.autograd.grad(torch.sigmoid(x), x, torch.from_numpy(b["dopacity"]))
        np.testing.assert_allclose(pc.opacity.grad.numpy(), ref_op.numpy(), rtol=1e-5, atol=1e-10)
        s = pc.scaling.detach().requires_grad_()
        (ref_s,) = torch.autograd.grad(torch.exp(s), s, torch.from_numpy(b["dscales"]))
        np.testing.assert_allclose(pc.scaling.grad.numpy(), ref_s.numpy(), rtol=1e-5, atol=1e-10)
        r = pc.rotation.detach().requires_grad_()
        (ref_r,) = torch.autograd.grad(torch.nn.functional.normalize(r), r, torch.from_numpy(b["drot"]))
        np.testing.assert_allclose(pc.rotation.grad.numpy(), ref_r.numpy(), rtol=1e-5, atol=1e-10)
    else:
        # gradients flowed through the reference's eval_sh and get_covariance
        assert b["dsh"].shape == (300, 0, 3)
        assert pc.features_rest.grad is not None and pc.scaling.grad is not None and pc.rotation.grad is not None
        xyz_total = pc.xyz.grad.numpy()
        assert np.isfinite(xyz_total).all()
        # the rasterizer's own mean gradient is part of the total
        assert np.abs(xyz_total - b["dmeans3D"]).max() < np.abs(xyz_total).max() * 10
