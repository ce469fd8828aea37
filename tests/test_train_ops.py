"""§8f "next" rows 1-2: fused L1 + D-SSIM (loss and gradient in one HIP pass), Adam
over the six parameter groups and the densification statistics, against the
reference's torch formulas (utils/loss_utils.py, torch.optim.Adam,
scene/gaussian_model.py:565-581) and the golden loss captured from the reference.

CPU tests: argument validation through the C ABI.  GPU tests: numerics."""
import ctypes

import numpy as np
import pytest
import torch

from conftest import golden


# ------------------------------------------------------------------ CPU: validation
@pytest.fixture(scope="module")
def lib():
    from diff_gaussian_rasterization import _C

    return _C.load_library()


def test_train_ops_reject_bad_arguments(lib):
    from diff_gaussian_rasterization import _C

    assert lib.gsr_l1_ssim(None, None, 0, 8, 8, 0.2, None, None, None, None) != 0
    assert "empty image" in lib.gsr_last_error().decode()
    assert lib.gsr_l1_ssim(1, 1, 3, 8, 8, 0.2, None, 1, 1, None) != 0
    assert "NULL" in lib.gsr_last_error().decode()
    segs = (_C.GsrAdamSegment * 9)()
    assert lib.gsr_adam_step(segs, 9, 1, 0.9, 0.999, 1e-15, None) != 0
    assert "segments" in lib.gsr_last_error().decode()
    assert lib.gsr_adam_step(segs, 1, 0, 0.9, 0.999, 1e-15, None) != 0
    assert "step" in lib.gsr_last_error().decode()
    assert lib.gsr_densify_stats(4, None, None, 1, None, None, None, None) != 0
    assert "stride" in lib.gsr_last_error().decode()
    assert lib.gsr_l1_ssim_scratch_bytes(3, 1080, 1920) >= 2 * 4 * 3 * -(-1080 // 32) * (1920 // 32)  # 32x32 tiles
    # nothing to do is not an error
    assert lib.gsr_adam_step(segs, 0, 1, 0.9, 0.999, 1e-15, None) == 0
    assert lib.gsr_densify_stats(0, None, None, 3, None, None, None, None) == 0


# ------------------------------------------------------------------ GPU: numerics
def _torch_loss(img, gt, lam):
    from train_step import l1_loss, ssim

    return (1.0 - lam) * l1_loss(img, gt) + lam * (1.0 - ssim(img, gt))


@pytest.mark.gpu
def test_l1_ssim_matches_reference_golden(dev):
    """Pinned by the reference's own l1_loss / ssim on the golden images."""
    import train_ops

    d = golden("loss.npz")
    a = torch.from_numpy(d["a"]).to(dev)
    b = torch.from_numpy(d["b"]).to(dev)
    for lam in (0.0, 0.2, 1.0):
        loss = train_ops.l1_ssim_loss(a, b, lam)
        want = (1 - lam) * float(d["l1"]) + lam * (1 - float(d["ssim"]))
        np.testing.assert_allclose(loss.item(), want, rtol=2e-6, atol=2e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(3, 37, 53), (3, 64, 96), (3, 131, 250), (1, 17, 5)])
def test_l1_ssim_gradient_matches_torch_autograd(dev, shape):
    """Loss and d loss / d image against autograd of the torch restatement (float64)."""
    import train_ops

    g = torch.Generator().manual_seed(hash(shape) % 1000)
    img = torch.rand(shape, generator=g)
    gt = torch.rand(shape, generator=g)
    x = img.to(dev).requires_grad_(True)
    loss = train_ops.l1_ssim_loss(x, gt.to(dev), 0.2)
    loss.backward()
    xr = img.double().requires_grad_(True)
    ref = _torch_loss(xr, gt.double(), 0.2)
    ref.backward()
    np.testing.assert_allclose(loss.item(), ref.item(), rtol=1e-5)
    gh, gr = x.grad.double().cpu(), xr.grad
    rel = (gh - gr).norm() / gr.norm()
    assert rel < 1e-5, f"gradient rel-L2 {rel:.3e}"


@pytest.mark.gpu
def test_l1_ssim_full_hd_against_torch(dev):
    """1080p, the headline image size: fused vs the torch float32 path."""
    import train_ops

    g = torch.Generator().manual_seed(5)
    img = torch.rand(3, 1080, 1920, generator=g).to(dev)
    gt = torch.rand(3, 1080, 1920, generator=g).to(dev)
    x = img.clone().requires_grad_(True)
    loss = train_ops.l1_ssim_loss(x, gt, 0.2)
    loss.backward()
    xr = img.clone().requires_grad_(True)
    ref = _torch_loss(xr, gt, 0.2)
    ref.backward()
    np.testing.assert_allclose(loss.item(), ref.item(), rtol=1e-5)
    rel = ((x.grad - xr.grad).norm() / xr.grad.norm()).item()
    assert rel < 1e-4, f"gradient rel-L2 {rel:.3e}"


def _groups(params, lrs):
    names = ["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"]
    return [{"params": [p], "lr": lr, "name": n} for p, lr, n in zip(params, lrs, names)]


@pytest.mark.gpu
def test_fused_adam_matches_torch_adam(dev):
    import train_ops

    g = torch.Generator().manual_seed(3)
    shapes = [(1000, 3), (1000, 1, 3), (1000, 15, 3), (1000, 1), (1000, 3), (1001, 4)]
    lrs = [0.00016 * 6.6, 0.0025, 0.0025 / 20, 0.05, 0.005, 0.001]
    base = [torch.randn(s, generator=g) for s in shapes]
    pa = [b.clone().to(dev).requires_grad_(True) for b in base]
    pb = [b.clone().to(dev).requires_grad_(True) for b in base]
    fa = train_ops.FusedAdam(_groups(pa, lrs), lr=0.0, eps=1e-15)
    ta = torch.optim.Adam(_groups(pb, lrs), lr=0.0, eps=1e-15)
    for _ in range(4):
        grads = [torch.randn(s, generator=g).to(dev) for s in shapes]
        for p, q, gr in zip(pa, pb, grads):
            p.grad = gr.clone()
            q.grad = gr.clone()
        fa.step()
        ta.step()
    for p, q in zip(pa, pb):
        np.testing.assert_allclose(p.detach().cpu().numpy(), q.detach().cpu().numpy(), rtol=1e-6, atol=1e-7)
        st, sq = fa.state[p], ta.state[q]
        np.testing.assert_allclose(st["exp_avg"].cpu().numpy(), sq["exp_avg"].cpu().numpy(), rtol=1e-6, atol=2e-7)
        np.testing.assert_allclose(st["exp_avg_sq"].cpu().numpy(), sq["exp_avg_sq"].cpu().numpy(), rtol=1e-6,
                                   atol=1e-12)


@pytest.mark.gpu
def test_densify_stats_match_reference_formula(dev):
    import train_ops

    g = torch.Generator().manual_seed(4)
    P = 5000
    radii = torch.randint(-2, 9, (P,), generator=g, dtype=torch.int32).clamp_min(0).to(dev)
    vgrad = torch.randn(P, 3, generator=g).to(dev)
    mr = torch.rand(P, generator=g).mul(5).to(dev)
    acc = torch.rand(P, 1, generator=g).to(dev)
    den = torch.randint(0, 5, (P, 1), generator=g).float().to(dev)
    mr2, acc2, den2 = mr.clone(), acc.clone(), den.clone()
    train_ops.densify_stats(radii, vgrad, mr, acc, den)
    vis = radii > 0
    mr2[vis] = torch.max(mr2[vis], radii[vis])
    acc2[vis] += torch.norm(vgrad[vis, :2], dim=-1, keepdim=True)
    den2[vis] += 1
    torch.testing.assert_close(mr, mr2, rtol=0, atol=0)
    torch.testing.assert_close(den, den2, rtol=0, atol=0)
    torch.testing.assert_close(acc, acc2, rtol=1e-6, atol=1e-7)


@pytest.mark.gpu
def test_full_train_step_fused_matches_torch(dev):
    """One iteration of train.py's loop (config A-sized scene): fused loss/Adam/statistics
    vs the reference's torch ops give the same loss, parameters and statistics."""
    import synthetic
    import train_step

    cam = synthetic.make_camera(256, 192, 0).to(dev)
    target = synthetic.make_target(256, 192, seed=1).to(dev)
    bg = torch.zeros(3, device=dev)
    out = {}
    for fused in (False, True):
        g = synthetic.make_gaussians(20_000, 3, seed=0).to(dev, requires_grad=True)
        st = train_step.TrainState(g, spatial_lr_scale=6.6, fused=fused)
        losses = [train_step.full_train_step(it, cam, g, st, target, bg).item() for it in (1, 2)]
        out[fused] = (losses, [p.detach().clone() for p in g.params()], st)
    np.testing.assert_allclose(out[True][0], out[False][0], rtol=1e-5)
    # Adam divides by sqrt(v) (eps 1e-15): an entry whose gradient is ~0 moves by up to
    # ~lr per step on a last-ulp difference of that gradient (here the fused loss's
    # dL/dpix vs torch's, and the atomics' summation order), even flipping sign.  So:
    # nearly every entry within 2e-5, the rare rest within the 2 steps' 2 lr bound.
    lrs = [g["lr"] for g in out[False][2].optimizer.param_groups]
    for a, b, lr in zip(out[True][1], out[False][1], lrs):
        d = (a - b).abs()
        assert float((d > 2e-5 + 1e-4 * b.abs()).float().mean()) < 1e-3, float((d > 2e-5).float().mean())
        assert float(d.max()) <= 2 * 2 * lr + 1e-6, (float(d.max()), lr)
    for n in ("max_radii2D", "denom"):
        torch.testing.assert_close(getattr(out[True][2], n), getattr(out[False][2], n), rtol=0, atol=0)
    # the second step's statistics inherit those few entries' moves (and their
    # neighbours' through the blend): all but ~1 % agree to 1e-4
    a, b = out[True][2].xyz_gradient_accum, out[False][2].xyz_gradient_accum
    off = (a - b).abs() > 1e-4 * b.abs() + 1e-9
    assert float(off.float().mean()) < 0.01, float(off.float().mean())
