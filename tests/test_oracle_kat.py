"""Analytic known-answer tests of the oracle and
integer-stage invariants (scan, duplicateWithKeys, stable sort, tile ranges)."""
import math

import numpy as np
import torch

import synthetic


def _cam(W, H, view=0):
    return synthetic.make_camera(W, H, view)


def _fwd(oracle, cam, means, opac, colors, scales, rots, bg=(0, 0, 0)):
    return oracle.forward(np.asarray(means, np.float32), np.asarray(opac, np.float32), cam.world_view_transform,
                          cam.full_proj_transform, cam.camera_center, np.asarray(bg, np.float32), cam.image_height,
                          cam.image_width, math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), 1.0, 0,
                          colors_precomp=np.asarray(colors, np.float32), scales=np.asarray(scales, np.float32),
                          rotations=np.asarray(rots, np.float32))


def _world_for_pixel(cam, px, py, depth=6.0):
    """View 0 camera sits at (0,0,-6) looking +z: world point whose projection is (px, py)."""
    W, H = cam.image_width, cam.image_height
    ndc = np.array([(2 * px + 1) / W - 1, (2 * py + 1) / H - 1])
    return [ndc[0] * depth * math.tan(cam.FoVx / 2), ndc[1] * depth * math.tan(cam.FoVy / 2), depth - 6.0]


def test_kat1_single_gaussian_on_pixel_centre(oracle):
    cam = _cam(32, 32)
    p = _world_for_pixel(cam, 10, 7)
    f = _fwd(oracle, cam, [p], [0.6], [[0.3, 0.6, 0.9]], [[0.01] * 3], [[1, 0, 0, 0]])
    assert abs(f["means2D"][0, 0] - 10) < 1e-3 and abs(f["means2D"][0, 1] - 7) < 1e-3
    np.testing.assert_allclose(f["color"][:, 7, 10], 0.6 * np.array([0.3, 0.6, 0.9]), rtol=1e-3)
    assert f["n_contrib"][7, 10] == 1
    np.testing.assert_allclose(f["final_T"][7, 10], 0.4, rtol=1e-3)


def test_kat2_behind_near_plane_is_culled(oracle):
    cam = _cam(32, 32)
    f = _fwd(oracle, cam, [[0, 0, -5.85]], [0.9], [[1, 1, 1]], [[0.1] * 3], [[1, 0, 0, 0]], bg=(0.2, 0.4, 0.6))
    assert f["radii"][0] == 0 and f["num_rendered"] == 0
    np.testing.assert_array_equal(f["color"], np.broadcast_to(np.float32([0.2, 0.4, 0.6])[:, None, None],
                                                              (3, 32, 32)))


def test_kat3_faint_gaussian_contributes_nothing(oracle):
    cam = _cam(32, 32)
    f = _fwd(oracle, cam, [[0, 0, 0]], [1.0 / 300], [[1, 1, 1]], [[0.1] * 3], [[1, 0, 0, 0]])
    assert f["num_rendered"] > 0  # binned ...
    assert not f["n_contrib"].any() and not f["color"].any()  # ... but alpha < 1/255 everywhere


def test_kat4_equal_depth_ties_blend_lower_index_first(oracle):
    cam = _cam(32, 32)
    p = _world_for_pixel(cam, 16, 16)
    f = _fwd(oracle, cam, [p, p], [0.5, 0.5], [[1, 0, 0], [0, 1, 0]], [[0.05] * 3] * 2, [[1, 0, 0, 0]] * 2)
    s, e = f["ranges"][(16 // 16) * 2 + 1]
    assert list(f["point_list"][s:e][:2]) == [0, 1]
    c = f["color"][:, 16, 16]
    assert c[0] > c[1] > 0  # red blended first with T = 1, green after with T = 1 - alpha


def test_kat5_saturation_after_five_blends(oracle):
    cam = _cam(16, 16)
    p = _world_for_pixel(cam, 8, 8)
    n = 8
    f = _fwd(oracle, cam, [p] * n, [0.8] * n, [[1, 1, 1]] * n, [[2.0] * 3] * n, [[1, 0, 0, 0]] * n)
    assert f["n_contrib"][8, 8] == 5
    np.testing.assert_allclose(f["final_T"][8, 8], 0.2 ** 5, rtol=1e-3)
    # o = 0.99 clamps alpha at 0.99: the second test_T (9.99998e-5) is already < 1e-4
    f = _fwd(oracle, cam, [p] * n, [0.9999] * n, [[1, 1, 1]] * n, [[2.0] * 3] * n, [[1, 0, 0, 0]] * n)
    assert f["n_contrib"][8, 8] == 1


def test_kat6_sh_degree0_colour(oracle):
    rng = np.random.default_rng(0)
    dc = rng.normal(0, 0.7, (50, 1, 3)).astype(np.float32)
    rgb, clamped = oracle.sh_to_rgb(rng.normal(size=(50, 3)), np.zeros(3), dc, 0)
    ref = np.float32(0.28209479177387814) * dc[:, 0] + np.float32(0.5)
    np.testing.assert_allclose(rgb, np.maximum(ref, 0), rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(clamped, ref < 0)


def test_kat7_tile_rect_edges(oracle):
    """Rect = [(int)((x - r)/16), (int)((x + r + 15)/16)) clamped to the grid; truncation toward 0."""
    cam = _cam(64, 64)
    for px in (0.0, 15.0, 16.0, 31.5, 47.9, 63.0):
        p = _world_for_pixel(cam, px, 20.0)
        f = _fwd(oracle, cam, [p], [0.5], [[1, 1, 1]], [[0.02] * 3], [[1, 0, 0, 0]])
        r = f["radii"][0]
        x = f["means2D"][0, 0]
        rect = f["rects"][0]
        exp_x0 = min(4, max(0, int((np.float32(x) - np.float32(r)) / np.float32(16))))
        exp_x1 = min(4, max(0, int((np.float32(x) + np.float32(r) + np.float32(16) - np.float32(1)) / np.float32(16))))
        assert (rect[0], rect[2]) == (exp_x0, exp_x1), (px, r, rect)
        assert f["tiles_touched"][0] == (rect[2] - rect[0]) * (rect[3] - rect[1])


def test_integer_stage_invariants(oracle):
    cam = _cam(200, 120, view=2)
    g = synthetic.make_gaussians(3000, 1, seed=4)
    f = oracle.forward(g.get_xyz.numpy(), g.get_opacity.detach().numpy(), cam.world_view_transform,
                       cam.full_proj_transform, cam.camera_center, np.zeros(3, np.float32), 120, 200,
                       math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), 1.0, 1, shs=g.get_features.numpy(),
                       scales=g.get_scaling.detach().numpy(), rotations=g.get_rotation.detach().numpy())
    I = f["num_rendered"]
    assert I == int(f["tiles_touched"].sum()) == int(f["point_offsets"][-1])
    np.testing.assert_array_equal(np.cumsum(f["tiles_touched"].astype(np.int64)), f["point_offsets"])
    keys = f["keys"]
    assert np.all(keys[1:] >= keys[:-1])  # sorted
    # stable: equal keys keep emission (index) order
    eq = keys[1:] == keys[:-1]
    assert np.all(f["point_list"][1:][eq] > f["point_list"][:-1][eq])
    lens = f["ranges"][:, 1] - f["ranges"][:, 0]
    assert lens.sum() == I
    for t in np.flatnonzero(lens):
        s, e = f["ranges"][t]
        assert np.all((keys[s:e] >> np.uint64(32)) == t)
    # every visible Gaussian appears exactly tiles_touched times
    counts = np.bincount(f["point_list"], minlength=3000)
    np.testing.assert_array_equal(counts, f["tiles_touched"])
    # mark_visible agrees with the near-plane cull
    vis = oracle.mark_visible(g.get_xyz.numpy(), cam.world_view_transform)
    assert np.all(vis[f["radii"] > 0])


def test_threaded_oracle_matches_single_threaded(oracle):
    """liboracle_mt.so (OpenMP; bench.py's CPU baseline and the full-size GPU parity
    cases) renders bit-identically to the single-threaded checker; its backward sums
    per-thread partials, so the gradients agree to float reordering."""
    import numpy as np

    from helpers import case, random_dL, run_oracle

    cam, g = case(20_000, 200, 150, 3, seed=3, view=2)
    dL = random_dL(150, 200)
    a, b = run_oracle(oracle, cam, g), run_oracle(oracle, cam, g, mt=True)
    for k in ("color", "radii", "keys", "point_list", "ranges", "n_contrib", "final_T", "means2D", "conic_opacity"):
        assert np.array_equal(a[k], b[k]), k
    ga, gb = oracle.backward(a, dL), oracle.backward(b, dL)
    for k in ga:
        den = max(float(np.linalg.norm(ga[k])), 1e-30)
        assert float(np.linalg.norm(ga[k] - gb[k])) / den < 1e-5, k
