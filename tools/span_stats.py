"""Row-span statistics of the rect footprint at a BASELINE config (CPU, oracle preprocess).

Prices the row-span binning: per Gaussian the rect's rows
(one span each) and tiles (instances), the spans and instances per tile row,
the longest tile list.  Usage: python tools/span_stats.py C"""
import ctypes
import math
import sys
import time

import numpy as np

sys.path[:0] = ["3dgs_study_amd", "."]
import synthetic  # noqa: E402
from oracle import oracle  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C"
c = synthetic.CONFIGS[cfg]
P, W, H, deg = c["P"], c["W"], c["H"], c["sh_degree"]
cam = synthetic.make_camera(W, H, 0)
g = synthetic.make_gaussians(P, deg, seed=0)
lib = oracle._load(True)
f32 = lambda a: np.ascontiguousarray(np.asarray(a, np.float32))  # noqa: E731
means3D = f32(g.get_xyz.numpy())
scales = f32(g.get_scaling.detach().numpy())
rots = f32(g.get_rotation.detach().numpy())
opac = f32(g.get_opacity.detach().numpy()).reshape(P)
cols = np.zeros((P, 3), np.float32) + 0.5
radii = np.zeros(P, np.int32)
means2D = np.zeros((P, 2), np.float32)
depths = np.zeros(P, np.float32)
cov3Ds = np.zeros((P, 6), np.float32)
rgb = np.zeros((P, 3), np.float32)
conic = np.zeros((P, 4), np.float32)
tt = np.zeros(P, np.uint32)
rects = np.zeros((P, 4), np.int32)
clamped = np.zeros((P, 3), np.uint8)
p = oracle._p
t = time.time()
lib.oracle_preprocess(ctypes.c_int(P), ctypes.c_int(0), ctypes.c_int(0), p(means3D), p(scales), ctypes.c_float(1.0),
                      p(rots), p(opac), None, p(clamped), None, p(cols), p(f32(cam.world_view_transform.numpy())),
                      p(f32(cam.full_proj_transform.numpy())), p(f32(cam.camera_center.numpy())), ctypes.c_int(W),
                      ctypes.c_int(H), ctypes.c_float(math.tan(cam.FoVx / 2)), ctypes.c_float(math.tan(cam.FoVy / 2)),
                      p(radii), p(means2D), p(depths), p(cov3Ds), p(rgb), p(conic), p(tt), p(rects), ctypes.c_int(0))
print(f"config {cfg}: preprocess {time.time() - t:.1f}s")
gx, gy = (W + 15) // 16, (H + 15) // 16
x0, y0, x1, y1 = rects[:, 0], rects[:, 1], rects[:, 2], rects[:, 3]
vis = (radii > 0) & (x1 > x0) & (y1 > y0)
h = np.where(vis, y1 - y0, 0)
w = np.where(vis, x1 - x0, 0)
I = int((h * w).sum())
S = int(h.sum())
print(f"P {P} visible {int(vis.sum())} grid {gx}x{gy}  instances I={I} (tiles_touched sum {int(tt.sum())})  spans S={S}")
print(f"  per visible Gaussian: rows {h[vis].mean():.2f} cols {w[vis].mean():.2f} tiles {(h * w)[vis].mean():.2f}; "
      f"max rows {h.max()} max cols {w.max()}")
cnt = np.zeros((gy + 1, gx + 1), np.int64)
np.add.at(cnt, (y0[vis], x0[vis]), 1)
np.add.at(cnt, (y0[vis], x1[vis]), -1)
np.add.at(cnt, (y1[vis], x0[vis]), -1)
np.add.at(cnt, (y1[vis], x1[vis]), 1)
tiles = cnt.cumsum(0).cumsum(1)[:gy, :gx]
print(f"  tile lists: mean {tiles.mean():.0f} max {tiles.max()}  empty {(tiles == 0).sum()} of {gx * gy}")
rows = np.zeros(gy + 1, np.int64)
np.add.at(rows, y0[vis], 1)
np.add.at(rows, y1[vis], -1)
rows = rows.cumsum()[:gy]
print(f"  spans per tile row: mean {rows.mean():.0f} max {rows.max()}")
