"""Work model for blend-kernel layouts at config C, from the CPU oracle's forward
(run in the build container; 300 random non-empty tiles, seed 0).

For each 8x8 quadrant it finds the list entries that reach a pixel with alpha >=
1/255 (the ideal quadrant cull) within the range the backward walks (up to the
quadrant's largest n_contrib), and compares layouts by replay work:
  * valid-lane fraction of the current one-wave-per-quadrant layout;
  * 4x4 sub-groups (four 16-lane Gaussian streams per wave, lockstep per
    64-entry chunk): pair iterations relative to the current layout;
  * 16x8 half-tile waves with 2 pixels per lane: lane-pixel replay work of the
    union of the two quadrants' survivors relative to the separate quadrants.
DESIGN.md §9 quotes the results (0.46, 0.83, 1.35)."""
import math
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "3dgs_study_amd"), str(ROOT / "tests"), str(ROOT)]

from helpers import case  # noqa: E402
from oracle import oracle as o  # noqa: E402

W, H, GX = 1920, 1080, 120


def quadrant_hits(f, ids, tile, qd):
    m2, co = f["means2D"].reshape(-1, 2), f["conic_opacity"].reshape(-1, 4)
    nc = f["n_contrib"].reshape(H, W)
    tx, ty = tile % GX, tile // GX
    x0, y0 = tx * 16 + (qd & 1) * 8, ty * 16 + (qd >> 1) * 8
    px, py = np.meshgrid(np.arange(x0, x0 + 8), np.arange(y0, y0 + 8))
    inside = (px < W) & (py < H)
    ncq = np.where(inside, nc[np.minimum(py, H - 1), np.minimum(px, W - 1)], 0).ravel()
    dx = m2[ids, 0][:, None] - px.ravel()[None, :]
    dy = m2[ids, 1][:, None] - py.ravel()[None, :]
    c = co[ids]
    power = -0.5 * (c[:, 0:1] * dx * dx + c[:, 2:3] * dy * dy) - c[:, 1:2] * dx * dy
    alpha = np.minimum(0.99, c[:, 3:4] * np.exp(power))
    ok = (power <= 0) & (alpha >= 1 / 255) & inside.ravel()[None, :]
    return ok, ncq


def chunked(lists, end):
    return sum(max((s[c0:c0 + 64].sum() + 1) // 2 for s in lists) for c0 in range(0, end, 64))


def main():
    cam, g = case(1_000_000, W, H, 3, seed=0, view=0)
    f = o.forward(g.get_xyz.numpy(), g.get_opacity.detach().numpy(), cam.world_view_transform.numpy(),
                  cam.full_proj_transform.numpy(), cam.camera_center.numpy(), np.zeros(3, np.float32), H, W,
                  math.tan(cam.FoVx * 0.5), math.tan(cam.FoVy * 0.5), shs=g.get_features.detach().numpy(),
                  scales=g.get_scaling.detach().numpy(), rotations=g.get_rotation.detach().numpy(), sh_degree=3,
                  mt=True)
    ranges, pl = f["ranges"], f["point_list"]
    tiles = np.random.default_rng(0).choice(np.nonzero(ranges[:, 1] > ranges[:, 0])[0], 300, replace=False)
    valid = lanes = p8 = p4 = union = sep = 0
    lx, ly = np.arange(64) % 8, np.arange(64) // 8
    for tile in tiles:
        ids = pl[ranges[tile][0]:ranges[tile][1]]
        k = np.arange(len(ids))
        per_q = [quadrant_hits(f, ids, tile, qd) for qd in range(4)]
        for ok, ncq in per_q:
            end = ncq.max()
            surv = ok.any(1) & (k < end)
            valid += (ok & (k[:, None] < ncq[None, :]))[surv].sum()
            lanes += 64 * surv.sum()
            p8 += chunked([ok[:end].any(1)], end)
            p4 += chunked([ok[:end][:, ((lx >= 4) == bool(sb & 1)) & ((ly >= 4) == bool(sb >> 1))].any(1)
                           for sb in range(4)], end)
        for half in range(2):
            (oa, na), (ob, nb) = per_q[2 * half], per_q[2 * half + 1]
            sep += (oa.any(1) & (k < na.max())).sum() + (ob.any(1) & (k < nb.max())).sum()
            union += 2 * ((oa.any(1) | ob.any(1)) & (k < max(na.max(), nb.max()))).sum()
    print(f"valid-lane fraction, one wave per 8x8 quadrant: {valid / lanes:.3f}")
    print(f"4x4 sub-group streams, pair iterations vs now:  {p4 / p8:.3f}")
    print(f"16x8 waves, 2 px/lane, replay work vs now:       {union / sep:.3f}")


if __name__ == "__main__":
    main()
