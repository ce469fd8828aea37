"""Config E forward: where and why the HIP image departs from the oracle's (diagnostic)."""
import math
import sys

import numpy as np
import torch

sys.path[:0] = ["3dgs_study_amd", ".", "tests"]
from helpers import case, run_hip, run_oracle  # noqa: E402
from oracle import oracle  # noqa: E402

W, H = 3840, 2160
cam, g = case(5_000_000, W, H, 3, seed=0)
h = run_hip(cam, g, torch.device("cuda:0"))
r = run_oracle(oracle, cam, g)
err = np.abs(h["color"] - r["color"]).max(axis=0)
terr = np.abs(h["final_T"] - r["final_T"])
bad = np.argwhere(err > 1e-4)
print("pixels > 1e-4:", len(bad), "of", W * H, "max", err.max(), "final_T max", terr.max(),
      "final_T > 1e-4:", int((terr > 1e-4).sum()), flush=True)
gx = (W + 15) // 16
m2 = r["means2D"].astype(np.float64)
co = r["conic_opacity"].astype(np.float64)
for (y, x) in bad[np.argsort(-err[bad[:, 0], bad[:, 1]])][:8]:
    t = (y // 16) * gx + x // 16
    s, e = r["ranges"][t]
    ids = r["point_list"][s:e]
    dx = m2[ids, 0] - x
    dy = m2[ids, 1] - y
    pw = -0.5 * (co[ids, 0] * dx * dx + co[ids, 2] * dy * dy) - co[ids, 1] * dx * dy
    al = np.minimum(0.99, co[ids, 3] * np.exp(pw))
    near = np.abs(al * 255 - 1) < 1e-4
    Tm = np.cumprod(np.where((pw <= 0) & (al >= 1 / 255), 1 - al, 1.0))
    print(f"pixel ({x},{y}) err {err[y, x]:.3g} T_hip {h['final_T'][y, x]:.4g} T_ref {r['final_T'][y, x]:.4g} "
          f"n_contrib hip {h['n_contrib'][y, x]} ref {r['n_contrib'][y, x]} list {e - s}; "
          f"alpha within 1e-4 rel of 1/255: {np.flatnonzero(near)[:5].tolist()} "
          f"T near 1e-4 at: {np.flatnonzero(np.abs(Tm / 1e-4 - 1) < 1e-3)[:5].tolist()}", flush=True)
