"""Workload statistics of the blend stages at a BASELINE config (CPU, from the oracle).

For every tile and 8x8 quadrant (one wave64): how many list entries the forward
walks before the quadrant saturates, how many the backward replays (< wave max
n_contrib), how many of those pass the conservative alpha box, and how many have
at least one contributing pixel.  Guides the CDNA4 blend-kernel design."""
import math
import sys
import time

import numpy as np

sys.path[:0] = ["3dgs_study_amd", "."]
import synthetic  # noqa: E402
from oracle import oracle  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "B"
c = synthetic.CONFIGS[cfg]
P, W, H, deg = c["P"], c["W"], c["H"], c["sh_degree"]
cam = synthetic.make_camera(W, H, 0)
g = synthetic.make_gaussians(P, deg, seed=0)
t = time.time()
f = oracle.forward(g.get_xyz.numpy(), g.get_opacity.detach().numpy(), cam.world_view_transform.numpy(),
                   cam.full_proj_transform.numpy(), cam.camera_center.numpy(), np.zeros(3, np.float32), H, W,
                   math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), 1.0, deg, shs=g.get_features.numpy(),
                   scales=g.get_scaling.detach().numpy(), rotations=g.get_rotation.detach().numpy())
print(f"config {cfg}: oracle fwd {time.time()-t:.1f}s I={f['num_rendered']}")
m2 = f["means2D"]
co = f["conic_opacity"]
cov_det = co[:, 0] * co[:, 2] - co[:, 1] ** 2
cxx = co[:, 2] / cov_det  # Sigma_xx = conic.z / det(conic)
cyy = co[:, 0] / cov_det
lnr = np.log(np.maximum(255 * co[:, 3], 1e-30)) + 1e-3
ex = np.where(lnr > 0, np.sqrt(2 * np.maximum(lnr, 0) * cxx) * 1.01 + 0.5, -1)
ey = np.where(lnr > 0, np.sqrt(2 * np.maximum(lnr, 0) * cyy) * 1.01 + 0.5, -1)
gx = (W + 15) // 16
nc = f["n_contrib"]
stats = dict(tiles=0, list=0, fwd_walk=0, fwd_box=0, fwd_valid=0, bwd_walk=0, bwd_box=0, bwd_valid=0,
             bwd_valid_lanes=0, quads=0)
for tile in range(f["ranges"].shape[0]):
    s, e = f["ranges"][tile]
    if e <= s:
        continue
    stats["tiles"] += 1
    stats["list"] += e - s
    ids = f["point_list"][s:e]
    tx, ty = tile % gx, tile // gx
    for q in range(4):
        x0, y0 = tx * 16 + (q & 1) * 8, ty * 16 + (q >> 1) * 8
        if x0 >= W or y0 >= H:
            continue
        stats["quads"] += 1
        ncq = nc[y0:y0 + 8, x0:x0 + 8]
        wmax = int(ncq.max())
        # forward walks until every pixel is done: approx last index with any pixel still active
        # (a pixel finishes at n_contrib or later; use max n_contrib + 1 bounded by list)
        fw = min(e - s, wmax + 1)
        box = (m2[ids, 0] + ex[ids] >= x0) & (m2[ids, 0] - ex[ids] <= x0 + 7) & \
              (m2[ids, 1] + ey[ids] >= y0) & (m2[ids, 1] - ey[ids] <= y0 + 7)
        stats["fwd_walk"] += fw
        stats["fwd_box"] += int(box[:fw].sum())
        stats["bwd_walk"] += wmax
        stats["bwd_box"] += int(box[:wmax].sum())
        # valid pixels per entry (alpha >= 1/255 and k < n_contrib)
        jj = np.arange(wmax)
        if wmax:
            sel = ids[:wmax]
            ys, xs = np.mgrid[y0:y0 + 8, x0:x0 + 8]
            dx = m2[sel, 0][:, None, None] - xs[None]
            dy = m2[sel, 1][:, None, None] - ys[None]
            cc = co[sel]
            pw = -0.5 * (cc[:, 0, None, None] * dx * dx + cc[:, 2, None, None] * dy * dy) - cc[:, 1, None, None] * dx * dy
            al = np.minimum(0.99, cc[:, 3, None, None] * np.exp(pw))
            v = (pw <= 0) & (al >= 1 / 255) & (jj[:, None, None] < ncq[None])
            vl = v.reshape(wmax, -1).sum(1)
            stats["bwd_valid"] += int((vl > 0).sum())
            stats["bwd_valid_lanes"] += int(vl.sum())
            vf = (pw <= 0) & (al >= 1 / 255)
            stats["fwd_valid"] += int((vf.reshape(wmax, -1)[:fw].sum(1) > 0).sum())
for k, v in stats.items():
    print(f"{k:16s} {v:>14,d}")
q = stats["quads"]
print(f"avg list/tile {stats['list']/stats['tiles']:.0f}; per quadrant: fwd walk {stats['fwd_walk']/q:.0f} "
      f"box {stats['fwd_box']/q:.0f} valid {stats['fwd_valid']/q:.0f}; bwd walk {stats['bwd_walk']/q:.0f} "
      f"box {stats['bwd_box']/q:.0f} valid {stats['bwd_valid']/q:.0f} lanes/valid {stats['bwd_valid_lanes']/max(1,stats['bwd_valid']):.1f}")
