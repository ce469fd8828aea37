"""Pin the oracle (and the host-side helpers) to golden vectors captured from the
reference's own Python in the build container (tests/golden/make_golden.py).

* SH -> RGB: utils/sh_utils.py:57-112 eval_sh (+0.5, clamp at 0 as in
  gaussian_renderer/__init__.py:89-90) vs forward.cu computeColorFromSH restated.
* 3D covariance: scene/gaussian_model.py:27-32 + utils/general_utils.py:72-128
  vs forward.cu computeCov3D restated.
* Camera matrices: utils/graphics_utils.py:49-133 + scene/cameras.py:103-121,163-164
  vs synthetic.make_camera (must be bit-identical).
* Boundary: the 12 settings fields and the rasterizer kwargs render() produces.
* Loss: utils/loss_utils.py l1_loss / ssim vs train_step.l1_loss / ssim.
"""
import json

import numpy as np
import pytest
import torch

from conftest import ROOT, golden


def test_sh_eval_matches_reference(oracle):
    d = golden("sh_eval.npz")
    dirs, sh = d["dirs"], d["sh"]  # sh: [P, 3, 16] as eval_sh takes it
    shs = np.ascontiguousarray(np.transpose(sh, (0, 2, 1)))  # rasterizer layout [P, M, 3]
    for deg in range(4):
        ref = np.maximum(d[f"rgb_deg{deg}"] + 0.5, 0.0)
        rgb, clamped = oracle.sh_to_rgb(dirs, np.zeros(3, np.float32), shs, deg)
        np.testing.assert_allclose(rgb, ref, rtol=2e-6, atol=2e-6)
        np.testing.assert_array_equal(clamped, (d[f"rgb_deg{deg}"] + 0.5) < 0)


def test_train_step_eval_sh_matches_reference():
    from train_step import eval_sh

    d = golden("sh_eval.npz")
    for deg in range(4):
        out = eval_sh(deg, torch.from_numpy(d["sh"]), torch.from_numpy(d["dirs"])).numpy()
        np.testing.assert_allclose(out, d[f"rgb_deg{deg}"], rtol=1e-6, atol=1e-6)


def test_cov3d_matches_reference(oracle):
    from train_step import covariance

    d = golden("cov3d.npz")
    for mod in (1.0, 0.5):
        ref = d[f"cov3d_mod{mod}"]
        got = oracle.cov3d(d["scales"], mod, d["rotations"])
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-10)
        host = covariance(torch.from_numpy(d["scales"]), mod, torch.from_numpy(d["rotations"])).numpy()
        np.testing.assert_allclose(host, ref, rtol=1e-5, atol=1e-10)


def test_synthetic_cameras_match_reference_conventions():
    import synthetic

    d = golden("cameras.npz")
    for (W, H) in ((256, 256), (800, 800), (1920, 1080)):
        for view in range(8):
            key = f"{W}x{H}_v{view}"
            cam = synthetic.make_camera(W, H, view)
            np.testing.assert_array_equal(cam.world_view_transform.numpy(), d[key + "_world_view"])
            np.testing.assert_array_equal(cam.projection_matrix.numpy(), d[key + "_proj"])
            np.testing.assert_array_equal(cam.full_proj_transform.numpy(), d[key + "_full_proj"])
            np.testing.assert_array_equal(cam.camera_center.numpy(), d[key + "_center"])
            np.testing.assert_allclose([cam.FoVx, cam.FoVy], d[key + "_fov"], rtol=0, atol=0)


def test_boundary_surface_matches_reference_call():
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    import inspect

    meta = json.loads((ROOT / "tests" / "golden" / "boundary.json").read_text())
    for branch in ("native", "python"):
        assert list(GaussianRasterizationSettings._fields) == meta[branch]["settings_fields"]
        params = list(inspect.signature(GaussianRasterizer.forward).parameters)[1:]
        assert set(meta[branch]["kwargs_order"]) <= set(params)
    assert meta["native"]["kwargs"]["colors_precomp"] is None and meta["native"]["kwargs"]["cov3D_precomp"] is None
    assert meta["python"]["kwargs"]["shs"] is None and meta["python"]["kwargs"]["scales"] is None


def test_render_tiny_capture_is_what_train_step_render_builds():
    """train_step.render (used on the GPU box, where the reference is absent) hands the
    rasterizer the same tensors as the reference's render() did for the same scene."""
    import synthetic
    import train_step

    d = golden("render_tiny.npz")
    cam = synthetic.make_camera(64, 48, view=1)
    pc = synthetic.make_gaussians(40, sh_degree=3, seed=5, radius=1.0, active_sh_degree=2)
    captured = {}

    class Spy:
        def __init__(self, raster_settings):
            captured["settings"] = raster_settings

        def __call__(self, **kw):
            captured["kw"] = kw
            P = kw["means3D"].shape[0]
            return torch.zeros(3, 48, 64), torch.zeros(P, dtype=torch.int32)

    orig = train_step.GaussianRasterizer
    train_step.GaussianRasterizer = Spy
    try:
        for branch, (sh_py, cov_py) in {"native": (False, False), "python": (True, True)}.items():
            train_step.render(cam, pc, torch.zeros(3), convert_SHs_python=sh_py, compute_cov3D_python=cov_py)
            for k, v in captured["kw"].items():
                key = f"{branch}__{k}"
                if v is None:
                    assert key not in d.files, key
                else:
                    np.testing.assert_allclose(v.detach().numpy(), d[key], rtol=2e-6, atol=1e-7, err_msg=key)
            s = captured["settings"]
            for f in s._fields:
                ref = d[f"{branch}__settings__{f}"]
                val = getattr(s, f)
                val = val.numpy() if torch.is_tensor(val) else np.array(val)
                np.testing.assert_array_equal(val, ref, err_msg=f)
    finally:
        train_step.GaussianRasterizer = orig


def test_losses_match_reference():
    from train_step import l1_loss, ssim

    d = golden("loss.npz")
    a, b = torch.from_numpy(d["a"]), torch.from_numpy(d["b"])
    np.testing.assert_allclose(l1_loss(a, b).numpy(), d["l1"], rtol=1e-6)
    np.testing.assert_allclose(ssim(a, b).numpy(), d["ssim"], rtol=1e-5)
