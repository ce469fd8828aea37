"""Where the model path's preprocess time goes (config C): the forward preprocess
stage through _C directly, alternating four input forms —
  cat      : the reference glue's inputs (activated values, the SH cat);
  split    : activated values, the SH as _features_dc + _features_rest (sh_rest);
  act      : stored parameters (activations in the kernel), the SH cat;
  model    : stored parameters and the split SH (rasterize_model's form).
usage (on the box): python tools/pre_probe.py [--reps 200] [--rounds 3]"""
import argparse
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3dgs_study_amd"), ROOT]

import synthetic  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--config", default="C")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = synthetic.CONFIGS[args.config]
    cam = synthetic.make_camera(cfg["W"], cfg["H"], view=0).to(dev)
    g = synthetic.make_gaussians(cfg["P"], cfg["sh_degree"], seed=0).to(dev)
    bg = torch.zeros(3, device=dev)
    empty = torch.empty(0, device=dev)
    act = dict(opacity=torch.sigmoid(g.opacity), scales=torch.exp(g.scaling),
               rotations=torch.nn.functional.normalize(g.rotation))
    raw = dict(opacity=g.opacity, scales=g.scaling, rotations=g.rotation)
    cat = torch.cat((g.features_dc, g.features_rest), dim=1).contiguous()
    forms = {
        "cat": (act, cat, None, 0),
        "split": (act, g.features_dc, g.features_rest, 0),
        "act": (raw, cat, None, _C.ACT_ALL),
        "model": (raw, g.features_dc, g.features_rest, _C.ACT_ALL),
    }

    def run(form):
        p, sh, rest, bits = forms[form]
        return _C._rasterize(bg, g.xyz, empty, p["opacity"], p["scales"], p["rotations"], 1.0, empty,
                             cam.world_view_transform, cam.full_proj_transform, math.tan(cam.FoVx * 0.5),
                             math.tan(cam.FoVy * 0.5), cam.image_height, cam.image_width, sh, g.active_sh_degree,
                             cam.camera_center, False, False, sh_rest=rest, activations=bits)

    ref = run("cat")
    for f in forms:  # same image from every form (the activations are torch's bit for bit)
        assert torch.equal(run(f)[1], ref[1]), f
    with torch.no_grad():
        for r in range(args.rounds):
            for f in forms:
                for _ in range(5):
                    run(f)
                torch.cuda.synchronize()
                _C.timing_enable(["preprocess", "render_fwd"])
                for _ in range(args.reps):
                    run(f)
                st = _C.timing_read()
                _C.timing_enable(False)
                print(f"{r} {f:6s} preprocess {1e3 * st['preprocess'][0] / st['preprocess'][1]:6.1f} us  "
                      f"render_fwd {1e3 * st['render_fwd'][0] / st['render_fwd'][1]:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
