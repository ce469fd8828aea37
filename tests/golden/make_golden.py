"""Capture golden vectors from the reference's own Python (run in the build container only).

The reference (PoplarPoplar/3dgs_study, mounted read-only at /root/reference) has no
tests and its rasterizer submodule is absent, but the pure-PyTorch pieces that define the
hot path's conventions import and run on CPU.  This script runs them on seeded inputs and
writes inputs + outputs as small .npz/.json fixtures next to itself.  Nothing from the
reference (source or bytecode) is copied; the fixtures are data only.  Re-run with

    python tests/golden/make_golden.py

Captured:
  sh_eval.npz      utils/sh_utils.py:57-112           eval_sh(deg, sh, dirs), deg 0..3
  cov3d.npz        utils/general_utils.py:72-128 +    get_covariance() path:
                   scene/gaussian_model.py:27-32      strip_symmetric(L L^T), L = R(q) S
  cameras.npz      utils/graphics_utils.py:49-133 +   world_view / projection / full_proj /
                   scene/cameras.py:95-121,163-164    camera_center of the synthetic views
  boundary.json    gaussian_renderer/__init__.py:20-112  the exact settings fields and the
                   rasterizer kwargs render() produces for both input branches
  render_tiny.npz  the same capture with its tensor values (tiny scene) for replay on GPU
  loss.npz         utils/loss_utils.py:17-108         l1_loss / ssim on small images
  ply.npz          scene/gaussian_model.py:218-318    save_ply's structured vertex array (names,
                   formats, bytes) and the parameters load_ply rebuilds, SH degrees 0/1/3
"""
from __future__ import annotations

import importlib.util
import json
import math
import sys
import types
from pathlib import Path

import numpy as np
import torch

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent
REPO = OUT.parent.parent


def _load(name: str, path: Path):
    spec = importlib.util.spec_from_file_location(name, str(path))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


class _CpuDevice:
    """Strip the reference's hard-coded device='cuda' (general_utils.py:73,104,120;
    gaussian_renderer/__init__.py:35) while a reference function runs on CPU."""

    def __enter__(self):
        self._orig = {}
        for name in ("zeros", "zeros_like", "empty", "ones", "tensor"):
            fn = getattr(torch, name)
            self._orig[name] = fn

            def wrap(*a, _fn=fn, **k):
                if k.get("device") == "cuda":
                    k["device"] = "cpu"
                return _fn(*a, **k)

            setattr(torch, name, wrap)
        return self

    def __exit__(self, *exc):
        for name, fn in self._orig.items():
            setattr(torch, name, fn)


def capture_sh():
    sh_utils = _load("ref_sh_utils", REF / "utils" / "sh_utils.py")
    g = torch.Generator().manual_seed(123)
    P = 257
    out = {}
    dirs = torch.randn(P, 3, generator=g)
    dirs = dirs / dirs.norm(dim=1, keepdim=True)
    sh = torch.randn(P, 3, 16, generator=g) * 0.5
    out["dirs"] = dirs.numpy()
    out["sh"] = sh.numpy()
    for deg in range(4):
        out[f"rgb_deg{deg}"] = sh_utils.eval_sh(deg, sh, dirs).numpy()
    np.savez_compressed(OUT / "sh_eval.npz", **out)


def capture_cov3d():
    gu = _load("ref_general_utils", REF / "utils" / "general_utils.py")
    g = torch.Generator().manual_seed(7)
    P = 257
    scales = torch.exp(math.log(0.003) + (math.log(0.03) - math.log(0.003)) * torch.rand(P, 3, generator=g))
    rots = torch.randn(P, 4, generator=g)
    rots_n = torch.nn.functional.normalize(rots)
    out = {"scales": scales.numpy(), "rotations": rots_n.numpy()}
    with _CpuDevice():
        for mod in (1.0, 0.5):
            # scene/gaussian_model.py:27-32 build_covariance_from_scaling_rotation
            L = gu.build_scaling_rotation(mod * scales, rots_n)
            cov = gu.strip_symmetric(L @ L.transpose(1, 2))
            out[f"cov3d_mod{mod}"] = cov.numpy()
    np.savez_compressed(OUT / "cov3d.npz", **out)


def capture_cameras():
    gr = _load("ref_graphics_utils", REF / "utils" / "graphics_utils.py")
    sys.modules.setdefault("utils", types.ModuleType("utils"))
    sys.modules["utils.graphics_utils"] = gr
    cams = _load("ref_cameras", REF / "scene" / "cameras.py")
    sys.path.insert(0, str(REPO / "3dgs_study_amd"))
    import synthetic  # our generator: R, T and FoV recipe

    out = {}
    for (W, H) in ((256, 256), (800, 800), (1920, 1080)):
        for view in range(8):
            fovx = math.radians(60.0)
            fovy = 2.0 * math.atan(math.tan(fovx / 2.0) * H / W)
            R = synthetic.yaw_rotation(view * math.pi / 4.0)
            T = np.array([0.0, 0.0, 6.0])
            wv = torch.tensor(gr.getWorld2View2(R, T)).transpose(0, 1)
            proj = gr.getProjectionMatrix(znear=0.01, zfar=100.0, fovX=fovx, fovY=fovy).transpose(0, 1)
            full = wv.unsqueeze(0).bmm(proj.unsqueeze(0)).squeeze(0)
            mc = cams.MiniCam(W, H, fovy, fovx, 0.01, 100.0, wv, full)
            key = f"{W}x{H}_v{view}"
            out[key + "_R"] = R
            out[key + "_T"] = T
            out[key + "_world_view"] = wv.numpy()
            out[key + "_proj"] = proj.numpy()
            out[key + "_full_proj"] = full.numpy()
            out[key + "_center"] = mc.camera_center.numpy()
            out[key + "_fov"] = np.array([fovx, fovy])
    np.savez_compressed(OUT / "cameras.npz", **out)


def capture_boundary():
    """Run the reference's render() with a recording stub in place of the absent
    diff_gaussian_rasterization module; record the settings and the kwargs."""
    calls = []

    class Settings(dict):
        def __init__(self, **kw):
            super().__init__(kw)
            calls.append({"settings_fields": list(kw.keys())})
            self.__dict__.update(kw)

    class Rasterizer:
        def __init__(self, raster_settings):
            self.s = raster_settings

        def __call__(self, **kw):
            calls[-1]["kwargs"] = {k: (None if v is None else list(v.shape)) for k, v in kw.items()}
            calls[-1]["kwargs_order"] = list(kw.keys())
            calls[-1]["values"] = {k: (None if v is None else v.detach().clone()) for k, v in kw.items()}
            calls[-1]["settings_values"] = {k: (v.detach().clone() if torch.is_tensor(v) else v)
                                            for k, v in self.s.items()}
            P = kw["means3D"].shape[0]
            return torch.zeros(3, self.s["image_height"], self.s["image_width"]), torch.zeros(P, dtype=torch.int32)

    stub = types.ModuleType("diff_gaussian_rasterization")
    stub.GaussianRasterizationSettings = Settings
    stub.GaussianRasterizer = Rasterizer
    saved = {k: sys.modules.get(k) for k in ("diff_gaussian_rasterization", "scene", "scene.gaussian_model",
                                              "utils", "utils.sh_utils")}
    sys.modules["diff_gaussian_rasterization"] = stub
    scene_pkg = types.ModuleType("scene")
    gm = types.ModuleType("scene.gaussian_model")
    gm.GaussianModel = object
    sys.modules["scene"] = scene_pkg
    sys.modules["scene.gaussian_model"] = gm
    sys.modules["utils"] = types.ModuleType("utils")
    sys.modules["utils.sh_utils"] = _load("utils.sh_utils", REF / "utils" / "sh_utils.py")
    gr_mod = _load("ref_gaussian_renderer", REF / "gaussian_renderer" / "__init__.py")

    sys.path.insert(0, str(REPO / "3dgs_study_amd"))
    import synthetic

    cam = synthetic.make_camera(64, 48, view=1)
    pc = synthetic.make_gaussians(40, sh_degree=3, seed=5, radius=1.0, active_sh_degree=2)
    pc.max_sh_degree = 3

    class Pipe:
        debug = False

    results = {}
    for branch, (sh_py, cov_py) in {"native": (False, False), "python": (True, True)}.items():
        pipe = Pipe()
        pipe.convert_SHs_python = sh_py
        pipe.compute_cov3D_python = cov_py
        # The SynthGaussians object lacks get_covariance; provide the reference formula.
        gu = _load("ref_general_utils2", REF / "utils" / "general_utils.py")

        def get_covariance(scaling_modifier=1.0, _pc=pc, _gu=gu):
            with _CpuDevice():
                L = _gu.build_scaling_rotation(scaling_modifier * _pc.get_scaling, _pc.rotation)
                return _gu.strip_symmetric(L @ L.transpose(1, 2))

        pc.get_covariance = get_covariance
        with _CpuDevice():
            gr_mod.render(cam, pc, pipe, torch.zeros(3), scaling_modifier=1.0)
        results[branch] = calls[-1]

    for k, v in saved.items():
        if v is None:
            sys.modules.pop(k, None)
        else:
            sys.modules[k] = v

    meta = {b: {"settings_fields": r["settings_fields"], "kwargs_order": r["kwargs_order"], "kwargs": r["kwargs"]}
            for b, r in results.items()}
    (OUT / "boundary.json").write_text(json.dumps(meta, indent=1) + "\n")
    arrays = {}
    for b, r in results.items():
        for k, v in r["values"].items():
            if v is not None:
                arrays[f"{b}__{k}"] = v.numpy()
        for k, v in r["settings_values"].items():
            if torch.is_tensor(v):
                arrays[f"{b}__settings__{k}"] = v.numpy()
            else:
                arrays[f"{b}__settings__{k}"] = np.array(v)
    np.savez_compressed(OUT / "render_tiny.npz", **arrays)


def capture_ply():
    """Run the reference's GaussianModel.save_ply / load_ply (scene/gaussian_model.py:
    218-318) with a recording stand-in for the absent ``plyfile`` package: ``PlyElement.
    describe`` captures the structured vertex array and element name save_ply builds,
    ``PlyData.read`` serves load_ply a captured array (also with its properties in a
    shuffled order, which load_ply's name sorts must undo).  Records the parameters
    going in, the array's field names and bytes, and the parameters load_ply rebuilt."""
    captured = {}

    class _Element:
        def __init__(self, data, name):
            self.data, self.name = data, name
            self.properties = [types.SimpleNamespace(name=n) for n in data.dtype.names]

        def __getitem__(self, key):
            return self.data[key]

    class PlyElement:
        @staticmethod
        def describe(data, name):
            captured["element"] = (np.array(data, copy=True), name)
            return _Element(data, name)

    class PlyData:
        to_read = None

        def __init__(self, elements):
            self.elements = elements

        def write(self, path):
            captured["written_to"] = path

        @classmethod
        def read(cls, path):
            return cls([_Element(cls.to_read, "vertex")])

    plyfile = types.ModuleType("plyfile")
    plyfile.PlyData, plyfile.PlyElement = PlyData, PlyElement
    knn_pkg, knn_c = types.ModuleType("simple_knn"), types.ModuleType("simple_knn._C")
    knn_c.distCUDA2 = None  # create_from_pcd only; not called here
    utils_pkg = types.ModuleType("utils")
    names = ("plyfile", "simple_knn", "simple_knn._C", "utils", "utils.general_utils", "utils.system_utils",
             "utils.sh_utils", "utils.graphics_utils")
    saved = {k: sys.modules.get(k) for k in names}
    sys.modules.update({"plyfile": plyfile, "simple_knn": knn_pkg, "simple_knn._C": knn_c, "utils": utils_pkg})
    for sub in ("general_utils", "system_utils", "sh_utils", "graphics_utils"):
        setattr(utils_pkg, sub, _load(f"utils.{sub}", REF / "utils" / f"{sub}.py"))
    gm = _load("ref_gaussian_model", REF / "scene" / "gaussian_model.py")

    sys.path.insert(0, str(REPO / "3dgs_study_amd"))
    import synthetic

    out = {}
    tmp = OUT / "_ply_tmp"
    for deg in (0, 1, 3):
        g = synthetic.make_gaussians(53, deg, seed=40 + deg)
        model = gm.GaussianModel(deg)
        model._xyz = torch.nn.Parameter(g.xyz.clone())
        model._features_dc = torch.nn.Parameter(g.features_dc.clone())
        model._features_rest = torch.nn.Parameter(g.features_rest.clone())
        model._opacity = torch.nn.Parameter(g.opacity.clone())
        model._scaling = torch.nn.Parameter(g.scaling.clone())
        model._rotation = torch.nn.Parameter(g.rotation.clone())
        captured.clear()
        model.save_ply(str(tmp / "point_cloud.ply"))
        rec, el_name = captured["element"]
        assert el_name == "vertex"
        key = f"d{deg}_"
        for n in ("xyz", "features_dc", "features_rest", "opacity", "scaling", "rotation"):
            out[key + "in_" + n] = getattr(g, n).numpy()
        out[key + "names"] = np.array(rec.dtype.names)
        out[key + "formats"] = np.array([rec.dtype.fields[n][0].str for n in rec.dtype.names])
        out[key + "body"] = np.frombuffer(rec.tobytes(), dtype=np.uint8)
        # load_ply on the captured array, and on the same columns in a shuffled order
        perm = np.random.default_rng(deg).permutation(len(rec.dtype.names))
        shuffled = np.empty(rec.shape[0], dtype=[(rec.dtype.names[i], "f4") for i in perm])
        for n in rec.dtype.names:
            shuffled[n] = rec[n]
        out[key + "shuffled_names"] = np.array(shuffled.dtype.names)
        for tag, arr in (("load_", rec), ("load_shuffled_", shuffled)):
            PlyData.to_read = arr
            back = gm.GaussianModel(deg)
            with _CpuDevice():
                back.load_ply(str(tmp / "point_cloud.ply"))
            assert back.active_sh_degree == deg
            for n in ("xyz", "features_dc", "features_rest", "opacity", "scaling", "rotation"):
                out[key + tag + n] = getattr(back, "_" + n).detach().numpy()
    if tmp.exists():
        tmp.rmdir()
    for k, v in saved.items():
        if v is None:
            sys.modules.pop(k, None)
        else:
            sys.modules[k] = v
    np.savez_compressed(OUT / "ply.npz", **out)


def capture_loss():
    lu = _load("ref_loss_utils", REF / "utils" / "loss_utils.py")
    g = torch.Generator().manual_seed(11)
    a = torch.rand(3, 37, 53, generator=g)
    b = torch.rand(3, 37, 53, generator=g)
    np.savez_compressed(OUT / "loss.npz", a=a.numpy(), b=b.numpy(), l1=lu.l1_loss(a, b).numpy(),
                        ssim=lu.ssim(a, b).numpy())


if __name__ == "__main__":
    if not REF.exists():
        sys.exit("reference not mounted; fixtures are committed, nothing to do")
    torch.set_num_threads(1)
    capture_sh()
    capture_cov3d()
    capture_cameras()
    capture_boundary()
    capture_loss()
    capture_ply()
    for p in sorted(OUT.glob("*.npz")) + sorted(OUT.glob("*.json")):
        print(p.name, p.stat().st_size)
