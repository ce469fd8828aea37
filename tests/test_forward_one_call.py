"""The one-call forward (include/gsr.h gsr_forward): emit, the tile sort and the
blend are queued before the host reads num_rendered, into a binning buffer whose
capacity the binding guessed (_C._capacity_for).  Whatever the capacity — too
small by one, 1, exact, generous — and whatever depth-pass count the library
queued up front (its hint from the last forward: three passes queued for a scene
that needs four, and four for one that needs three), every output must equal the
two-call form's (gsr_forward_preprocess + gsr_forward_render) bit for bit, the
gradients to the accumulator atomics' run-to-run spread.  ("Next
round" 1: the overflow path tested on purpose.)"""
import numpy as np
import pytest
import torch

from helpers import case, random_dL, rel_l2, run_hip

pytestmark = pytest.mark.gpu

INTS = ("radii", "n_contrib", "point_list", "ranges", "depth_order", "tiles_touched")


def _run(cam, g, dev, footprint, cap):
    from diff_gaussian_rasterization import _C

    prev = _C.capacity_override
    _C.capacity_override = cap
    try:
        H, W = cam.image_height, cam.image_width
        out = run_hip(cam, g, dev, dL=random_dL(H, W), footprint=footprint)
        out["path"] = {k: _C.last_forward.get(k) for k in ("capacity", "num_rendered", "path")}
        return out
    finally:
        _C.capacity_override = prev


def _same(a, b, what):
    assert a["num_rendered"] == b["num_rendered"], what
    np.testing.assert_array_equal(a["color"], b["color"], err_msg=what)
    np.testing.assert_array_equal(a["final_T"], b["final_T"], err_msg=what)
    for k in INTS:
        np.testing.assert_array_equal(a[k], b[k], err_msg=f"{what}: {k}")
    for k, ga in a["grads"].items():
        if ga is not None and ga.size:
            assert rel_l2(ga, b["grads"][k]) <= 1e-5, (what, k)


@pytest.mark.parametrize("footprint", ["tight", "rect"])
def test_capacity_paths_match_two_calls(dev, footprint):
    cam, g = case(30_000, 320, 240, 3, seed=6, view=2)
    ref = _run(cam, g, dev, footprint, 0)
    assert ref["path"]["path"] == "two calls"
    I = ref["num_rendered"]
    assert I > 1000
    for cap, path in ((1, "regrown"), (I - 1, "regrown"), (I, "one call"), (I + 1, "one call"),
                      (2 * I, "one call")):
        got = _run(cam, g, dev, footprint, cap)
        assert got["path"] == {"capacity": cap, "num_rendered": I, "path": path}, got["path"]
        _same(got, ref, f"{footprint} capacity {cap}")


def test_depth_pass_hint_paths(dev):
    """Radius 2 needs three depth passes, radius 5.5 four.  The library queues the
    fourth pass up front when the last forward needed it: each run below follows one
    of the other kind, so both mismatches (three queued / four needed: the fourth
    pass and the rank gather run after the host's read and the binning is redone;
    four queued / three needed: the fourth pass returns at once) are exercised, with
    a capacity that fits and with one that does not."""
    cases = {r: case(30_000, 320, 240, 3, seed=6, view=2, radius=r) for r in (2.0, 5.5)}
    ref = {r: _run(*cases[r], dev, "tight", 0) for r in (2.0, 5.5)}
    for cap_of in (lambda I: 4 * I, lambda I: 1):
        for r in (2.0, 5.5, 2.0, 5.5):
            cam, g = cases[r]
            got = _run(cam, g, dev, "tight", cap_of(ref[r]["num_rendered"]))
            _same(got, ref[r], f"radius {r}, capacity {got['path']['capacity']}")
    assert ref[2.0]["dsort_ctrl"][1] == 3 and ref[5.5]["dsort_ctrl"][1] == 4


def test_model_path_one_call_with_l1(dev):
    """rasterize_model with the L1 target (the bench's headline unit): the loss, the
    visibility filter, the image and the leaf gradients of the one-call forward equal
    the two-call form's, also when the capacity is too small."""
    import train_step
    from diff_gaussian_rasterization import _C

    cam, g = case(30_000, 320, 240, 3, seed=7, view=1)
    target = torch.rand(3, 240, 320, generator=torch.Generator().manual_seed(3)).to(dev)
    cam = cam.to(dev)
    bg = torch.zeros(3, device=dev)

    def run(cap):
        prev = _C.capacity_override
        _C.capacity_override = cap
        try:
            gd = g.to(dev, requires_grad=True)
            out = train_step.train_step(cam, gd, target, bg, glue="fused")
            torch.cuda.synchronize()
            return (dict(_C.last_forward), out["loss"].item(), out["render"].detach().cpu().numpy(),
                    out["visibility_filter"].cpu().numpy(), [p.grad.cpu().numpy() for p in gd.params()])
        finally:
            _C.capacity_override = prev

    ref = run(0)
    I = ref[0]["num_rendered"]
    for cap in (I, 3, 2 * I):
        got = run(cap)
        assert got[0]["path"] == ("one call" if cap >= I else "regrown")
        assert got[1] == ref[1]
        np.testing.assert_array_equal(got[2], ref[2])
        np.testing.assert_array_equal(got[3], ref[3])
        for a, b in zip(got[4], ref[4]):
            assert rel_l2(a, b) <= 1e-5


def test_default_binding_switches_to_one_call(dev):
    """Without an override the first forward of an image size takes the two-call form
    and the next ones the one-call form (the capacity learnt from the first)."""
    from diff_gaussian_rasterization import _C

    cam, g = case(5_000, 208, 160, 3, seed=2, view=3)
    _C._capacity_level.pop((208, 160, 1), None)
    paths = [_run(cam, g, dev, "tight", None)["path"]["path"] for _ in range(3)]
    assert paths == ["two calls", "one call", "one call"]


def test_backward_with_forward_chunk_masks_bit_identical(dev):
    """render_bwd replays the forward's chunks with the forward's cull masks when the
    forward prepared the backward (GSR_FLAG_PREPARE_BACKWARD), and
    culls the same chunks itself when it did not: on the isolated scene (one atomic
    per accumulator row: a deterministic backward) every gradient is the same bits."""
    from diff_gaussian_rasterization import _C
    from test_leaf_grads import _isolated_scene

    cam, g = _isolated_scene()
    cam, g = cam.to(dev), g.to(dev)
    H, W = cam.image_height, cam.image_width
    bg = torch.zeros(3, device=dev)
    e = torch.empty(0, device=dev)
    tx, ty = float(np.tan(cam.FoVx * 0.5)), float(np.tan(cam.FoVy * 0.5))
    sh = g.get_features.contiguous()
    dL = torch.from_numpy(random_dL(H, W)).to(dev) * 1e4
    outs = []
    for prep in (True, False):
        fw = (bg, g.get_xyz, e, g.get_opacity, g.get_scaling, g.get_rotation, 1.0, e, cam.world_view_transform,
              cam.full_proj_transform, tx, ty, H, W, sh, 3, cam.camera_center, False, False)
        R, color, radii, geom, binning, img = _C.rasterize_gaussians(*fw, prepare_backward=prep)
        bw = (bg, g.get_xyz, radii, e, g.get_scaling, g.get_rotation, 1.0, e, cam.world_view_transform,
              cam.full_proj_transform, tx, ty, dL, sh, 3, cam.camera_center, geom, R, binning, img, False)
        grads = _C.rasterize_gaussians_backward(*bw)
        torch.cuda.synchronize()
        outs.append((color.cpu(), [t.cpu() if t is not None else None for t in grads]))
    (c0, g0), (c1, g1) = outs
    assert torch.equal(c0, c1)
    for i, (a, b) in enumerate(zip(g0, g1)):
        if a is None or a.numel() == 0:
            continue
        assert float(a.abs().max()) > 0 or i == 1, i
        assert torch.equal(a.view(torch.int32), b.view(torch.int32)), i

