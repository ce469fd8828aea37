"""The fused training unit captured as a CUDA (HIP) graph (train_step.CapturedUnit;
gsr.h GSR_FLAG_NO_WAIT, gsr_forward_status): replays give the eager step's image,
loss, radii and gradients — also after the parameters change in place — and a
replay whose lists outgrow the captured capacity is reported, not passed off."""
import numpy as np
import pytest
import torch

import synthetic
import train_step
from helpers import rel_l2

pytestmark = pytest.mark.gpu

P, W, H, DEG = 20_000, 320, 240, 3


def _scene(dev):
    cam = synthetic.make_camera(W, H, view=2).to(dev)
    g = synthetic.make_gaussians(P, sh_degree=DEG, seed=7).to(dev, requires_grad=True)
    target = synthetic.make_target(W, H, seed=1).to(dev)
    return cam, g, target, torch.zeros(3, device=dev)


def _eager(cam, g, target, bg):
    for p in g.params():
        p.grad = None
    out = train_step.train_step(cam, g, target, bg, glue="fused")
    torch.cuda.synchronize()
    return ({k: out[k].detach().clone() for k in ("render", "loss", "radii", "visibility_filter")},
            [p.grad.detach().clone() for p in g.params()])


def _compare(out, grads, ref_out, ref_grads):
    out = {k: v.detach() for k, v in out.items() if isinstance(v, torch.Tensor)}
    np.testing.assert_array_equal(out["render"].cpu().numpy(), ref_out["render"].cpu().numpy())
    np.testing.assert_array_equal(out["radii"].cpu().numpy(), ref_out["radii"].cpu().numpy())
    np.testing.assert_array_equal(out["visibility_filter"].cpu().numpy(), ref_out["visibility_filter"].cpu().numpy())
    assert float(out["loss"]) == float(ref_out["loss"])
    for a, b in zip(grads, ref_grads):  # float atomics: the order may differ
        assert rel_l2(a.cpu().numpy(), b.cpu().numpy()) <= 1e-6


def test_captured_unit_matches_eager(dev):
    from diff_gaussian_rasterization import _C

    cam, g, target, bg = _scene(dev)
    ref_out, ref_grads = _eager(cam, g, target, bg)
    n_ref = _C.last_forward["num_rendered"]
    unit = train_step.CapturedUnit(cam, g, target, bg)
    for _ in range(3):
        out = unit.replay()
    torch.cuda.synchronize()
    assert unit.check() == n_ref
    _compare(out, [p.grad for p in g.params()], ref_out, ref_grads)
    # parameters changed in place: the replay renders the new values
    with torch.no_grad():
        g.xyz.add_(0.01)
        g.opacity.mul_(0.9)
    out = unit.replay()
    torch.cuda.synchronize()
    got = ({k: out[k].detach().clone() for k in ("render", "loss", "radii", "visibility_filter")},
           [p.grad.detach().clone() for p in g.params()])
    unit.check()
    ref_out2, ref_grads2 = _eager(cam, g, target, bg)
    assert not torch.equal(ref_out2["render"], ref_out["render"])
    _compare(got[0], got[1], ref_out2, ref_grads2)


def test_captured_unit_reports_overflow(dev):
    from diff_gaussian_rasterization import _C

    cam, g, target, bg = _scene(dev)
    _eager(cam, g, target, bg)
    prev = _C.capacity_override
    _C.capacity_override = 1_000  # far below the scene's num_rendered
    try:
        unit = train_step.CapturedUnit(cam, g, target, bg, warmup=1)
        unit.replay()
        torch.cuda.synchronize()
        with pytest.raises(RuntimeError, match="capacity"):
            unit.check()
    finally:
        _C.capacity_override = prev
