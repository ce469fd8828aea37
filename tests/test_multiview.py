"""View-parallel gradient exchange on the CPU with gloo, world size 2,
and on one GPU with two processes (gloo) against the single-process sum of views."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    for p in (str(PKG), str(ROOT), str(ROOT / "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _cpu_worker(rank, world, port, out):
    _init(rank, world, port)
    from multiview import GradAllReduce, views_for_rank

    torch.manual_seed(0)
    shapes = [(5, 3), (5, 1, 3), (5, 15, 3), (5, 1), (5, 3), (5, 4)]
    params = [torch.zeros(s, requires_grad=True) for s in shapes]
    for i, p in enumerate(params):
        p.grad = torch.full(s if (s := p.shape) else (), float(rank + 1) * (i + 1))
    ar = GradAllReduce(params)
    flat = ar()
    out[rank] = (flat.clone(), [p.grad.clone() for p in params], views_for_rank(rank, world, 8), ar.nbytes)
    dist.destroy_process_group()


def test_grad_all_reduce_gloo_world2():
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_cpu_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    f0, g0, v0, nb = res[0]
    f1, g1, v1, _ = res[1]
    assert torch.equal(f0, f1)
    for i, (a, b) in enumerate(zip(g0, g1)):
        assert torch.equal(a, b)
        assert torch.all(a == 3.0 * (i + 1))  # (1 + 2) * (i + 1)
    assert v0 == [0, 2, 4, 6] and v1 == [1, 3, 5, 7]
    assert nb == 5 * (3 + 3 + 45 + 1 + 3 + 4) * 4


def _cpu_overlap_worker(rank, world, port, out):
    _init(rank, world, port)
    from multiview import GradAllReduce

    torch.manual_seed(0)
    shapes = [(5, 3), (5, 1, 3), (5, 15, 3), (5, 1), (5, 3), (5, 4)]
    params = [torch.randn(s, requires_grad=True) for s in shapes]
    ar = GradAllReduce(params)  # the bucket's all-reduce starts when the backward ends
    w = float(rank + 1)
    loss = sum((w * (i + 1) * p * p).sum() for i, p in enumerate(params))
    loss.backward()
    pending = ar.pending
    ar()
    out[rank] = ([p.detach().clone() for p in params], [p.grad.clone() for p in params], pending)
    ar.remove_hooks()
    dist.destroy_process_group()


def test_grad_all_reduce_overlapped_gloo_world2():
    """Overlapped mode: the bucket's one all-reduce launches from the end-of-backward
    callback the parameters' hooks queue; after the wait every rank holds the sum of
    the ranks' gradients, as views of one flat bucket."""
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_cpu_overlap_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    p0, g0, n0 = res[0]
    p1, g1, n1 = res[1]
    assert n0 == n1 == 1  # one async all-reduce of the bucket, launched at the end of backward
    for i, (a, b, p) in enumerate(zip(g0, g1, p0)):
        assert torch.equal(a, b)
        # d/dp sum_r (r+1)(i+1) p^2 = 2 p (i+1) (1 + 2)
        torch.testing.assert_close(a, 2 * p * (i + 1) * 3.0)


def _records_rebuild(oracle_mod, P, M):
    """CPU stand-in for the HIP rebuild kernel (tests only): parse the gathered
    records and sum the views' SH gradients with the C oracle."""
    def rebuild(xyz, recs, nviews, dc, rest):
        from diff_gaussian_rasterization import _C
        stride = _C.sh_record_floats(P)
        r = recs.reshape(nviews, stride).numpy()
        dsh = oracle_mod.sh_grad_sum(xyz.numpy(), r[:, 0:3], r[:, 3].astype(np.int32), r[:, 4:4 + 3 * P], M)
        dc.copy_(torch.from_numpy(dsh[:, :1]))
        rest.copy_(torch.from_numpy(dsh[:, 1:]))
    return rebuild


def _sh_view(rank, P):
    g = torch.Generator().manual_seed(100 + rank)
    drgb = torch.randn(P, 3, generator=g)
    drgb[::7] = 0.0  # culled / clamped entries
    campos = torch.tensor([6.0 * np.cos(rank), 0.5 * rank, 6.0 * np.sin(rank)], dtype=torch.float32)
    return drgb, campos


def _cpu_sh_worker(rank, world, port, out):
    _init(rank, world, port)
    from multiview import GradAllReduce
    from oracle import oracle as orc

    P, M = 37, 16
    torch.manual_seed(0)
    shapes = [(P, 3), (P, 1, 3), (P, M - 1, 3), (P, 1), (P, 3), (P, 4)]
    params = [torch.randn(s, requires_grad=True) for s in shapes]
    ar = GradAllReduce(params, sh=(params[0], params[1], params[2]), rebuild=_records_rebuild(orc, P, M))
    for i in (0, 3, 4, 5):  # the all-reduced gradients, assigned by hand (flat mode)
        params[i].grad = torch.full(shapes[i], float(rank + 1) * (i + 1))
    drgb, campos = _sh_view(rank, P)
    sh = torch.empty(P, M, 3)
    assert ar.sh_exchange and ar.accepts(sh, params[0])
    rec = ar.record(P)
    rec[4:4 + 3 * P] = drgb.reshape(-1)  # what the rasterizer's backward writes
    ar.push(rec, campos, 3)
    ar()
    out[rank] = ([p.grad.clone() for p in params], params[0].detach().clone(), ar.nbytes)
    ar.remove_hooks()
    dist.destroy_process_group()


def test_sh_colour_exchange_gloo_world2(oracle):
    """SH exchange: ranks gather (campos, colour gradient) records; every rank's
    f_dc / f_rest gradients equal the oracle's sum over both views' SH gradients."""
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_cpu_sh_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    (g0, xyz, nb), (g1, _, _) = res[0], res[1]
    P, M = 37, 16
    for a, b in zip(g0, g1):
        assert torch.equal(a, b)
    for i in (0, 3, 4, 5):
        assert torch.all(g0[i] == 3.0 * (i + 1))
    views = [_sh_view(r, P) for r in (0, 1)]
    ref = oracle.sh_grad_sum(xyz.numpy(), np.stack([v[1].numpy() for v in views]), [3, 3],
                             np.stack([v[0].numpy() for v in views]), M)
    assert np.array_equal(g0[1].numpy(), ref[:, :1]) and np.array_equal(g0[2].numpy(), ref[:, 1:])
    assert np.abs(ref).sum() > 0
    stride = 4 + ((3 * P + 3) // 4) * 4
    assert nb == P * (3 + 1 + 3 + 4) * 4 + stride * 4


def test_oracle_sh_grad_sum_matches_preprocess_backward(oracle):
    """The oracle's per-view SH gradient sum equals upstream's SH backward run view by view."""
    rng = np.random.default_rng(5)
    P, M = 50, 16
    means = rng.normal(size=(P, 3)).astype(np.float32)
    campos = rng.normal(size=(2, 3)).astype(np.float32) * 5
    drgb = rng.normal(size=(2, P, 3)).astype(np.float32)
    got = oracle.sh_grad_sum(means, campos, [3, 1], drgb, M)
    # degree 1 leaves coefficients 4..15 of that view untouched
    one = [oracle.sh_grad_sum(means, campos[v:v + 1], [d], drgb[v:v + 1], M) for v, d in ((0, 3), (1, 1))]
    assert np.array_equal(got, one[0] + one[1])
    assert np.all(one[1][:, 4:] == 0)
    # basis(dir) . dRGB contracted with sh = d(rgb)/d(sh) . dRGB: check via eval_sh linearity
    shs = rng.normal(size=(P, M, 3)).astype(np.float32)
    rgb0, cl = oracle.sh_to_rgb(means, campos[0], shs, 3)
    lin = (one[0] * shs).sum(axis=1)  # sum_k basis_k sh[k][c] * drgb[c]
    expect = (rgb0 - 0.5) * drgb[0]
    ok = ~cl  # unclamped channels: rgb = basis . sh + 0.5
    assert np.allclose(lin[ok], expect[ok], atol=1e-4)


def _gpu_worker(rank, world, port, out, sh_exchange=False):
    _init(rank, world, port)
    import synthetic
    import train_step
    from multiview import GradAllReduce

    dev = torch.device("cuda:0")
    cam = synthetic.make_camera(160, 120, view=rank).to(dev)
    g = synthetic.make_gaussians(20_000, 3, seed=0).to(dev, requires_grad=True)
    target = synthetic.make_target(160, 120).to(dev)
    params = g.params()
    # overlapped: the all-reduces (and the SH record gather) start inside backward
    reducer = GradAllReduce(params, sh=(params[0], params[1], params[2]) if sh_exchange else None)
    train_step.train_step(cam, g, target, torch.zeros(3, device=dev))
    assert reducer.pending == 1 and reducer.launched_in_backward
    # the SH records' gather was consumed inside backward: the rebuild is queued on
    # the exchange's stream right behind it (GradAllReduce._rebuild_beside), and the
    # SH gradients reach the leaves when the reducer is called
    assert not reducer._gathers
    if sh_exchange:
        assert reducer._sh_out is not None
        assert params[1].grad is None and params[2].grad is None
    reducer()
    if sh_exchange:
        assert reducer._sh_out is None
        assert params[1].grad is not None and params[2].grad is not None
    out[rank] = [p.grad.detach().cpu() for p in g.params()]
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("sh_exchange", [False, True], ids=["allreduce", "sh_colour_exchange"])
def test_view_parallel_grads_equal_sum_of_views(dev, sh_exchange):
    import synthetic
    import train_step

    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_gpu_worker, args=(2, port, out, sh_exchange), nprocs=2, join=True)
        res = dict(out)
    # single process: sum of the two views' gradients
    g = synthetic.make_gaussians(20_000, 3, seed=0).to(dev, requires_grad=True)
    target = synthetic.make_target(160, 120).to(dev)
    total = None
    for view in (0, 1):
        for p in g.params():
            p.grad = None
        cam = synthetic.make_camera(160, 120, view=view).to(dev)
        train_step.train_step(cam, g, target, torch.zeros(3, device=dev))
        grads = [p.grad.detach().cpu().clone() for p in g.params()]
        total = grads if total is None else [a + b for a, b in zip(total, grads)]
    for a, b, ref in zip(res[0], res[1], total):
        assert torch.equal(a, b)  # replicas receive identical gradients
        rel = (a - ref).norm() / ref.norm().clamp_min(1e-30)
        assert rel < 1e-5, float(rel)


@pytest.mark.gpu
def test_sh_rebuild_bit_identical_to_preprocess_backward(dev):
    """One native backward: rebuilding dsh from that call's colour gradient (masked by
    the forward's clamp bits) through the HIP kernel gives preprocess_bwd's dsh bit
    for bit (shared sh_basis products, no fp contraction)."""
    import synthetic
    from diff_gaussian_rasterization import _C

    W, H, P = 200, 150, 30_000
    cam = synthetic.make_camera(W, H, view=3).to(dev)
    g = synthetic.make_gaussians(P, 3, seed=4).to(dev)
    bg = torch.zeros(3, device=dev)
    e = torch.empty(0, device=dev)
    sh = g.get_features.contiguous()
    tx, ty = float(np.tan(cam.FoVx * 0.5)), float(np.tan(cam.FoVy * 0.5))
    fw = (bg, g.get_xyz, e, g.get_opacity, g.get_scaling, g.get_rotation, 1.0, e, cam.world_view_transform,
          cam.full_proj_transform, tx, ty, H, W, sh, 3, cam.camera_center, False, False)
    R, color, radii, geom, binning, img = _C.rasterize_gaussians(*fw)
    dpix = torch.randn(3, H, W, device=dev, generator=torch.Generator(device=dev).manual_seed(2)) * 1e-3
    bw = (bg, g.get_xyz, radii, e, g.get_scaling, g.get_rotation, 1.0, e, cam.world_view_transform,
          cam.full_proj_transform, tx, ty, dpix, sh, 3, cam.camera_center, geom, R, binning, img,
          False)
    out = _C.rasterize_gaussians_backward(*bw)
    dcolors, dsh = out[1], out[5]
    off = _C.layouts(P, W, H, R)[0]["clamped"]
    cl = geom[off:off + P].to(torch.int32)
    bits = torch.stack([(cl >> c) & 1 for c in range(3)], dim=1)
    drgb = dcolors * (1 - bits).to(torch.float32)
    rec = torch.zeros(_C.sh_record_floats(P), device=dev)
    rec[0:3] = cam.camera_center
    rec[3] = 3
    rec[4:4 + 3 * P] = drgb.reshape(-1)
    dc = torch.empty(P, 1, 3, device=dev)
    rest = torch.empty(P, 15, 3, device=dev)
    _C.sh_grad_from_colors(g.get_xyz, rec, 1, dc, rest)
    assert torch.equal(torch.cat([dc, rest], dim=1), dsh)
    assert dsh.abs().sum() > 0
    # the colours-only backward writes that same masked colour gradient
    rec2 = torch.zeros_like(rec)
    out2 = _C.rasterize_gaussians_backward(*bw, drgb_out=rec2[4:])
    assert out2[5] is None
    got = rec2[4:4 + 3 * P].view(P, 3)
    rel = (got - drgb).norm() / drgb.norm()  # atomics order differs between the two backward calls
    assert rel < 1e-5, float(rel)
    assert torch.equal(got == 0, drgb == 0) or rel < 1e-6


@pytest.mark.gpu
def test_sh_exchange_single_rank_matches_plain_step(dev):
    """One rank, exchange forced on, through autograd: no SH gradient flows through
    autograd, and after the exchange every gradient matches the plain step (to the
    atomics-order tolerance)."""
    import synthetic
    import train_step
    from multiview import GradAllReduce

    cam = synthetic.make_camera(200, 150, view=3).to(dev)
    target = synthetic.make_target(200, 150).to(dev)
    res = []
    for force in (False, True):
        g = synthetic.make_gaussians(30_000, 3, seed=4).to(dev, requires_grad=True)
        params = g.params()
        ar = GradAllReduce(params, sh=(params[0], params[1], params[2]), sh_force=force)
        assert ar.sh_exchange == force
        train_step.train_step(cam, g, target, torch.zeros(3, device=dev))
        if force:
            assert params[1].grad is None and params[2].grad is None  # no dsh through autograd
        ar()
        ar.remove_hooks()
        res.append([p.grad.detach().cpu().clone() for p in params])
    for i, (a, b) in enumerate(zip(*res)):
        rel = (a - b).norm() / b.norm().clamp_min(1e-30)
        assert rel < 1e-5, (i, float(rel))
    assert res[0][2].abs().sum() > 0


@pytest.mark.gpu
def test_sh_grad_from_colors_kernel_vs_oracle(dev, oracle):
    """The rebuild kernel over 5 records (mixed SH degrees, zero rows) against the
    C oracle's view-ordered sum."""
    from diff_gaussian_rasterization import _C

    rng = np.random.default_rng(9)
    P, V = 4_099, 5
    for M in (16, 9, 4, 1):
        means = rng.normal(size=(P, 3)).astype(np.float32)
        campos = (rng.normal(size=(V, 3)) * 6).astype(np.float32)
        degs = [min(d, int(np.sqrt(M)) - 1) for d in (3, 2, 0, 1, 3)]
        drgb = rng.normal(size=(V, P, 3)).astype(np.float32)
        drgb[:, ::11] = 0
        stride = _C.sh_record_floats(P)
        rec = np.zeros((V, stride), np.float32)
        rec[:, :3], rec[:, 3], rec[:, 4:4 + 3 * P] = campos, degs, drgb.reshape(V, -1)
        dc = torch.empty(P, 1, 3, device=dev)
        rest = torch.empty(P, M - 1, 3, device=dev) if M > 1 else None
        _C.sh_grad_from_colors(torch.from_numpy(means).to(dev), torch.from_numpy(rec).to(dev), V, dc, rest)
        ref = oracle.sh_grad_sum(means, campos, degs, drgb, M)
        got = dc.cpu().numpy() if rest is None else np.concatenate([dc.cpu().numpy(), rest.cpu().numpy()], axis=1)
        err = np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-30)
        assert err <= 1e-6, (M, err)


@pytest.mark.gpu
def test_sh_grad_from_colors_one_view_form_bit_identical(dev):
    """One record takes the one-view kernel (products formed at write-out); the
    same record followed by an all-zero one takes the general kernel (the zero
    view is skipped).  The two agree bit for bit — signed zeros included — for
    every degree, ragged sizes, zero and signed-zero rows, and a Gaussian at the
    camera centre."""
    from diff_gaussian_rasterization import _C

    rng = np.random.default_rng(21)
    for P in (1, 7, 256, 4_099):
        for deg in (3, 2, 1, 0):
            means = rng.normal(size=(P, 3)).astype(np.float32)
            campos = (rng.normal(size=3) * 6).astype(np.float32)
            means[P // 2] = campos  # zero-length direction
            drgb = rng.normal(size=(P, 3)).astype(np.float32)
            drgb[::5] = 0
            drgb[P // 2] = 0
            drgb[1::7, 1] = -0.0
            stride = _C.sh_record_floats(P)
            rec = np.zeros((2, stride), np.float32)
            rec[:, :3], rec[:, 3], rec[0, 4:4 + 3 * P] = campos, deg, drgb.reshape(-1)
            m = torch.from_numpy(means).to(dev)
            r = torch.from_numpy(rec).to(dev)
            out = []
            for V in (1, 2):
                dc = torch.full((P, 1, 3), 7.0, device=dev)
                rest = torch.full((P, 15, 3), 7.0, device=dev)
                _C.sh_grad_from_colors(m, r, V, dc, rest)
                out.append(torch.cat([dc, rest], dim=1).cpu())
            a, b = out
            assert torch.equal(a.view(torch.int32), b.view(torch.int32)), (P, deg)
            assert not torch.isnan(a).any()
            if deg < 3:
                assert (a[:, (deg + 1) ** 2:] == 0).all()


# ---------------------------------------------------------------- several views per rank, re-binding, training
def _loss(params, view):
    """A stand-in for one view's render -> loss: view-dependent weights per parameter."""
    g = torch.Generator().manual_seed(1000 + view)
    return sum((torch.randn(p.shape, generator=g) * p * p).sum() for p in params)


def _shapes(P=6):
    return [(P, 3), (P, 1, 3), (P, 15, 3), (P, 1), (P, 3), (P, 4)]


def _views_worker(rank, world, port, out):
    _init(rank, world, port)
    from multiview import GradAllReduce, views_for_rank

    torch.manual_seed(0)
    params = [torch.randn(s, requires_grad=True) for s in _shapes()]
    views = views_for_rank(rank, world, 4)
    ar = GradAllReduce(params, views_per_step=len(views))
    for v in views:  # two backwards per rank: the all-reduces start on the second
        _loss(params, v).backward()
    pending = ar.pending
    ar()
    out[rank] = ([p.grad.clone() for p in params], pending)
    ar.remove_hooks()
    dist.destroy_process_group()


def test_two_views_per_rank_overlapped_gloo_world2():
    """with several backwards per step the bucket's all-reduce starts at the
    end of the step's last backward only; every rank ends with the sum over all 4 views."""
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_views_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    torch.manual_seed(0)
    params = [torch.randn(s, requires_grad=True) for s in _shapes()]
    for v in range(4):
        _loss(params, v).backward()
    (g0, n0), (g1, n1) = res[0], res[1]
    assert n0 == n1 == 1
    for a, b, p in zip(g0, g1, params):
        assert torch.equal(a, b)
        torch.testing.assert_close(a, p.grad, rtol=1e-6, atol=1e-6)


def _rebind_worker(rank, world, port, out):
    _init(rank, world, port)
    from multiview import GradAllReduce

    torch.manual_seed(0)
    model = {"params": [torch.randn(s, requires_grad=True) for s in _shapes()]}
    ar = GradAllReduce(lambda: model["params"])
    res = []
    for step in range(3):
        if step == 1:  # densify: every parameter replaced by a longer one (cat_tensors_to_optimizer)
            model["params"] = [torch.cat([p.detach(), p.detach()[:2] * 0.5]).requires_grad_(True)
                               for p in model["params"]]
        _loss(model["params"], 10 * step + rank).backward()
        hooked = ar.pending
        ar()
        res.append(([p.grad.clone() for p in model["params"]], hooked))
        for p in model["params"]:
            p.grad = None
    out[rank] = res
    ar.remove_hooks()
    dist.destroy_process_group()


def test_exchange_follows_replaced_parameters_gloo_world2():
    """after a densify step replaces every parameter, the exchange keeps
    summing over the ranks (flat bucket on the step of the swap, hooks re-bound for
    the next) instead of reducing the stale tensors."""
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_rebind_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    torch.manual_seed(0)
    params = [torch.randn(s, requires_grad=True) for s in _shapes()]
    for step in range(3):
        if step == 1:
            params = [torch.cat([p.detach(), p.detach()[:2] * 0.5]).requires_grad_(True) for p in params]
        for r in (0, 1):
            _loss(params, 10 * step + r).backward()
        (g0, h0), (g1, h1) = res[0][step], res[1][step]
        assert h0 == h1 == (0 if step == 1 else 1), (step, h0)  # no hooks on the fresh tensors yet
        for a, b, p in zip(g0, g1, params):
            assert torch.equal(a, b) and a.shape == p.shape
            torch.testing.assert_close(a, p.grad, rtol=1e-6, atol=1e-6)
        for p in params:
            p.grad = None


def _train_worker(rank, world, port, out):
    _init(rank, world, port)
    from multiview import GradAllReduce

    torch.manual_seed(0)
    params = [torch.randn(s, requires_grad=True) for s in _shapes()]
    opt = torch.optim.Adam([{"params": [p], "lr": 0.01 * (i + 1)} for i, p in enumerate(params)], eps=1e-15)
    ar = GradAllReduce(params)
    for step in range(4):
        _loss(params, 2 * step + rank).backward()
        ar()  # exchange before the optimizer step (train_step.full_train_step's order)
        opt.step()
        opt.zero_grad(set_to_none=True)
    out[rank] = [p.detach().clone() for p in params]
    ar.remove_hooks()
    dist.destroy_process_group()


def test_view_parallel_training_keeps_replicas_identical_gloo_world2():
    """N > 1 training: exchange then Adam on every rank; after 4 steps the replicas are
    bit-identical and equal a single process stepping on the summed gradients."""
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_train_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    torch.manual_seed(0)
    params = [torch.randn(s, requires_grad=True) for s in _shapes()]
    opt = torch.optim.Adam([{"params": [p], "lr": 0.01 * (i + 1)} for i, p in enumerate(params)], eps=1e-15)
    for step in range(4):
        grads = []
        for r in (0, 1):
            _loss(params, 2 * step + r).backward()
            grads.append([p.grad.clone() for p in params])
            for p in params:
                p.grad = None
        for p, a, b in zip(params, *grads):
            p.grad = a + b
        opt.step()
        opt.zero_grad(set_to_none=True)
    for a, b, p in zip(res[0], res[1], params):
        assert torch.equal(a, b)
        assert torch.equal(a, p.detach())


def _stats_worker(rank, world, port, out):
    _init(rank, world, port)
    from multiview import reduce_densification_stats

    P = 7
    g = torch.Generator().manual_seed(rank)
    acc = torch.rand(P, 1, generator=g)
    den = torch.randint(0, 3, (P, 1), generator=g).float()
    mx = torch.rand(P, generator=g) * 10
    loc = (acc.clone(), den.clone(), mx.clone())
    red = reduce_densification_stats(acc, den, mx)
    # copies: the per-rank accumulators are untouched, so a second call gives the same
    assert all(torch.equal(a, b) for a, b in zip((acc, den, mx), loc))
    again = reduce_densification_stats(acc, den, mx)
    assert all(torch.equal(a, b) for a, b in zip(red, again))
    out[rank] = red
    dist.destroy_process_group()


def test_densification_stats_reduce_sum_sum_max_gloo_world2():
    """scene/gaussian_model.py:565-581 statistics combined over the ranks before a
    densify step: SUM, SUM, MAX — identical on every rank."""
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_stats_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    loc = []
    for r in (0, 1):
        g = torch.Generator().manual_seed(r)
        loc.append((torch.rand(7, 1, generator=g), torch.randint(0, 3, (7, 1), generator=g).float(),
                    torch.rand(7, generator=g) * 10))
    for r in (0, 1):
        acc, den, mx = res[r]
        assert torch.equal(acc, loc[0][0] + loc[1][0])
        assert torch.equal(den, loc[0][1] + loc[1][1])
        assert torch.equal(mx, torch.maximum(loc[0][2], loc[1][2]))


def _foreign_worker(rank, world, port, out):
    _init(rank, world, port)
    from multiview import GradAllReduce

    P, M = 9, 16
    params = [torch.randn(s, requires_grad=True) for s in _shapes(P)]
    ar = GradAllReduce(params, sh=(params[0], params[1], params[2]), rebuild=lambda *a: None)
    try:
        ar.accepts(torch.empty(P + 1, M, 3), torch.empty(P + 1, 3))
        out[rank] = "accepted"
    except RuntimeError as e:
        out[rank] = str(e)
    ar.remove_hooks()
    dist.destroy_process_group()


def test_sh_sink_refuses_a_foreign_model_with_several_ranks():
    """with more than one rank, a backward whose SH input is not the bound
    model raises instead of silently keeping a local dsh."""
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_foreign_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    for r in (0, 1):
        assert "not the bound model" in res[r], res[r]


# ---------------------------------------------------------------- on the GPU: training steps, config D
def _gpu_train_worker(rank, world, port, out, sh_exchange):
    _init(rank, world, port)
    import synthetic
    import train_step
    from multiview import GradAllReduce

    dev = torch.device("cuda:0")
    cam = synthetic.make_camera(160, 120, view=rank).to(dev)
    g = synthetic.make_gaussians(20_000, 3, seed=0).to(dev, requires_grad=True)
    target = synthetic.make_target(160, 120).to(dev)
    st = train_step.TrainState(g, spatial_lr_scale=6.6, fused=True)
    reducer = GradAllReduce(g.params, sh=(lambda: g.params()[:3]) if sh_exchange else None)
    for it in range(1, 4):
        train_step.full_train_step(it, cam, g, st, target, torch.zeros(3, device=dev), reducer=reducer)
    torch.cuda.synchronize()
    out[rank] = [p.detach().cpu() for p in g.params()]
    reducer.remove_hooks()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("sh_exchange", [False, True], ids=["allreduce", "sh_colour_exchange"])
def test_view_parallel_full_train_step_keeps_replicas_identical(dev, sh_exchange):
    """Two ranks (gloo, sharing cuda:0) run three reference training iterations
    (train.py:86-141: render, L1 + D-SSIM, backward, exchange, fused Adam) on views 0
    and 1: the replicas stay bit-identical and match one process that steps on the sum
    of the two views' gradients."""
    import synthetic
    import train_step

    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_gpu_train_worker, args=(2, port, out, sh_exchange), nprocs=2, join=True)
        res = dict(out)
    g = synthetic.make_gaussians(20_000, 3, seed=0).to(dev, requires_grad=True)
    p0 = [p.detach().cpu().clone() for p in g.params()]
    target = synthetic.make_target(160, 120).to(dev)
    st = train_step.TrainState(g, spatial_lr_scale=6.6, fused=True)
    cams = [synthetic.make_camera(160, 120, view=v).to(dev) for v in (0, 1)]
    for it in range(1, 4):
        st.update_learning_rate(it)
        grads = []
        for cam in cams:
            for p in g.params():
                p.grad = None
            out_ = train_step.render(cam, g, torch.zeros(3, device=dev))
            import train_ops
            train_ops.l1_ssim_loss(out_["render"], target, 0.2).backward()
            grads.append([p.grad.clone() for p in g.params()])
        with torch.no_grad():
            for p, a, b in zip(g.params(), *grads):
                p.grad = a + b
            st.optimizer.step()
            st.optimizer.zero_grad(set_to_none=True)
    ref = [p.detach().cpu() for p in g.params()]
    for a, b, r, q in zip(res[0], res[1], ref, p0):
        assert torch.equal(a, b)  # replicas identical
        rel = ((a - q) - (r - q)).norm() / (r - q).norm().clamp_min(1e-30)
        assert rel < 1e-4, float(rel)


def _config_d_worker(rank, world, port, out, sh_exchange, path):
    _init(rank, world, port)
    import hashlib

    import synthetic
    import train_step
    from multiview import GradAllReduce

    dev = torch.device("cuda:0")
    cfg = synthetic.CONFIGS["C"]
    cam = synthetic.make_camera(cfg["W"], cfg["H"], view=rank).to(dev)
    g = synthetic.make_gaussians(cfg["P"], cfg["sh_degree"], seed=0).to(dev, requires_grad=True)
    target = synthetic.make_target(cfg["W"], cfg["H"], seed=1).to(dev)
    params = g.params()
    reducer = GradAllReduce(params, sh=(params[0], params[1], params[2]) if sh_exchange else None)
    train_step.train_step(cam, g, target, torch.zeros(3, device=dev))
    reducer()
    grads = [p.grad.detach().cpu().contiguous() for p in params]
    h = hashlib.sha256()
    for x in grads:
        h.update(x.numpy().tobytes())
    out[rank] = h.hexdigest()
    if rank == 0:
        torch.save(grads, path)
    reducer.remove_hooks()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.timeout(900)
@pytest.mark.parametrize("sh_exchange", [False, True], ids=["allreduce", "sh_colour_exchange"])
def test_config_d_eight_ranks_on_one_gpu(dev, sh_exchange, tmp_path):
    """Config D's workload (1M Gaussians, 1920x1080, views 0-7, one per rank) with 8
    ranks over gloo sharing cuda:0 — the exchange code path of the RCCL run, which the
    1-GPU box cannot measure: every rank ends with bit-identical leaf gradients, and
    they match the sequential sum of the 8 single-view gradients (rel-L2 1e-5)."""
    import synthetic
    import train_step

    port = _free_port()
    path = tmp_path / "rank0_grads.pt"
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_config_d_worker, args=(8, port, out, sh_exchange, str(path)), nprocs=8, join=True)
        res = dict(out)
    assert len(set(res.values())) == 1, "ranks disagree"
    got = torch.load(path, weights_only=True)
    cfg = synthetic.CONFIGS["C"]
    g = synthetic.make_gaussians(cfg["P"], cfg["sh_degree"], seed=0).to(dev, requires_grad=True)
    target = synthetic.make_target(cfg["W"], cfg["H"], seed=1).to(dev)
    total = None
    for view in range(8):
        for p in g.params():
            p.grad = None
        cam = synthetic.make_camera(cfg["W"], cfg["H"], view=view).to(dev)
        train_step.train_step(cam, g, target, torch.zeros(3, device=dev))
        grads = [p.grad.detach().clone() for p in g.params()]
        total = grads if total is None else [a + b for a, b in zip(total, grads)]
    for a, ref in zip(got, total):
        ref = ref.cpu()
        rel = (a - ref).norm() / ref.norm().clamp_min(1e-30)
        assert rel < 1e-5, float(rel)


def _rccl_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    for p in (str(PKG), str(ROOT), str(ROOT / "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    import synthetic
    import train_step
    from multiview import GradAllReduce, reduce_densification_stats

    cam = synthetic.make_camera(200, 150, view=2).to(dev)
    target = synthetic.make_target(200, 150).to(dev)
    res = {}
    for mode in ("plain", "allreduce", "sh_colour", "plain_fused", "allreduce_fused", "sh_colour_fused"):
        glue = "fused" if mode.endswith("_fused") else "reference"
        g = synthetic.make_gaussians(30_000, 3, seed=4).to(dev, requires_grad=True)
        params = g.params()
        ar = None
        if not mode.startswith("plain"):
            ar = GradAllReduce(params, sh=(params[0], params[1], params[2]) if mode.startswith("sh_colour") else None,
                               comm_force=True)
        train_step.train_step(cam, g, target, torch.zeros(3, device=dev), glue=glue)
        import diff_gaussian_rasterization as dgr
        plan = dgr.last_leaf_plan
        launched = ar is not None and ar.launched_in_backward
        if ar is not None:
            ar()
            ar.remove_hooks()
        stats = [torch.rand(30_000, 1, device=dev), torch.rand(30_000, 1, device=dev), torch.rand(30_000, device=dev)]
        red = reduce_densification_stats(*stats, force=True)
        torch.cuda.synchronize()
        res[mode] = ([p.grad.detach().cpu().clone() for p in params],
                     all(torch.equal(a, b) for a, b in zip(stats, red)), plan, launched)
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_collectives_one_rank(dev):
    """The exchange's RCCL calls on the real backend ("nccl" = RCCL), which the
    one-GPU box can only run as a one-rank group: the overlapped all-reduces from the
    post-accumulate-grad hooks, the all-gather of the SH colour records, and the
    densification statistics' SUM / MAX all-reduces, forced on.  With one rank every
    collective is the identity, so the gradients must equal the plain step's and the
    statistics must come back unchanged."""
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_rccl_worker, args=(1, port, out), nprocs=1, join=True)
        res = dict(out)[0]
    plain = res["plain"][0]
    assert res["plain"][2] == ("opacities", "rotations", "scales", "sh")
    # the fused leaf gradients survive the exchange — the rasterizer
    # writes xyz / opacity / scaling / rotation (and the SH leaves without the SH
    # exchange) into the bucket, whose one all-reduce starts at the end of backward
    assert res["sh_colour"][2] == ("means3D", "opacities", "rotations", "scales")
    assert res["allreduce"][2] == ("means3D", "opacities", "rotations", "scales", "sh")
    for mode in ("allreduce", "sh_colour"):
        grads, stats_same, _, launched = res[mode]
        assert stats_same and launched, mode
        for i, (a, b) in enumerate(zip(grads, plain)):
            rel = (a - b).norm() / b.norm().clamp_min(1e-30)
            assert rel < 1e-5, (mode, i, float(rel))
    # the model path (rasterize_model: stored parameters in, their gradients out)
    # under the same exchanges: every leaf the library writes lands in the bucket
    every = ("means3D", "opacities", "rotations", "scales", "sh")
    assert res["plain_fused"][2] == every
    assert res["sh_colour_fused"][2] == ("means3D", "opacities", "rotations", "scales")
    assert res["allreduce_fused"][2] == every
    for mode in ("plain_fused", "allreduce_fused", "sh_colour_fused"):
        grads, stats_same, _, launched = res[mode]
        assert stats_same and (launched or mode == "plain_fused"), mode
        for i, (a, b) in enumerate(zip(grads, plain)):
            rel = (a - b).norm() / b.norm().clamp_min(1e-30)
            assert rel < 1e-5, (mode, i, float(rel))


# ---------------------------------------------------------------- the bucket protocol with fused writers (CPU)
class _FusedWriter(torch.autograd.Function):
    """Stands in for the rasterizer's fused leaf gradients: its backward asks the
    installed exchange for bucket views of the leaves it writes (xyz and opacity
    here), writes (or, when the view is already the leaf's .grad, adds) their
    gradients itself and returns None for them; the other inputs get theirs through
    autograd, as unfusable ones do."""

    @staticmethod
    def forward(ctx, xyz, opacity, rest, w):
        ctx.save_for_backward(xyz, opacity, rest)
        ctx.w = w
        return (w * (xyz * xyz).sum() + w * (opacity * opacity).sum() + w * (rest * rest).sum()).reshape(())

    @staticmethod
    def backward(ctx, g):
        import diff_gaussian_rasterization as dgr

        xyz, opacity, rest = ctx.saved_tensors
        ex = dgr._exchange
        views = ex.leaf_bucket({"xyz": (xyz,), "opacity": (opacity,)}) if ex is not None else {}
        out = []
        for name, leaf in (("xyz", xyz), ("opacity", opacity)):
            v = views.get(name)
            val = 2 * ctx.w * leaf.detach() * g
            if v is None:
                out.append(val)
                continue
            if leaf.grad is None:
                v[0].copy_(val)
                leaf.grad = v[0]
            else:
                v[0].add_(val)
            out.append(None)
        return out[0], out[1], 2 * ctx.w * rest.detach() * g, None


def _fused_worker(rank, world, port, out, views_per_step):
    _init(rank, world, port)
    from multiview import GradAllReduce

    torch.manual_seed(0)
    xyz, opacity, rest = (torch.randn(s, requires_grad=True) for s in ((7, 3), (7, 1), (7, 4)))
    ar = GradAllReduce([xyz, rest, opacity], views_per_step=views_per_step)
    for v in range(views_per_step):
        w = float(rank + 1) * (v + 1)
        _FusedWriter.apply(xyz, opacity, rest, w).backward()
    launched, pending = ar.launched_in_backward, ar.pending
    flat = ar()
    grads = [p.grad.clone() for p in (xyz, opacity, rest)]
    views_ok = all(p.grad.data_ptr() >= flat.data_ptr() and
                   p.grad.data_ptr() < flat.data_ptr() + flat.numel() * 4 for p in (xyz, opacity, rest))
    out[rank] = (grads, [p.detach().clone() for p in (xyz, opacity, rest)], launched, pending, views_ok)
    ar.remove_hooks()
    dist.destroy_process_group()


@pytest.mark.parametrize("views_per_step", [1, 2])
def test_bucket_with_fused_writers_gloo_world2(views_per_step):
    """leaves whose gradients a fused backward writes straight into the
    exchange's bucket (the first backward writes, a later one of the step adds) and a
    leaf that goes through autograd share ONE bucket; its single all-reduce starts at
    the end of the step's last backward, and every rank ends with the sum of both
    ranks' views, every .grad a view of the bucket."""
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_fused_worker, args=(2, port, out, views_per_step), nprocs=2, join=True)
        res = dict(out)
    (g0, p, l0, n0, v0), (g1, _, l1, n1, v1) = res[0], res[1]
    assert l0 and l1 and n0 == n1 == 1 and v0 and v1
    wsum = sum(float(r + 1) * (v + 1) for r in (0, 1) for v in range(views_per_step))
    for a, b, x in zip(g0, g1, p):
        assert torch.equal(a, b)
        torch.testing.assert_close(a, 2 * wsum * x, rtol=1e-6, atol=1e-6)


class _AllWriter(torch.autograd.Function):
    """The rasterizer at N > 1 with every reduced leaf fused: its backward writes all
    of them into the exchange's bucket views and tells the exchange
    (``rasterizer_done``), which starts the bucket's all-reduce right there on the
    step's last backward instead of in the end-of-backward callback."""

    @staticmethod
    def forward(ctx, xyz, opacity, w):
        ctx.save_for_backward(xyz, opacity)
        ctx.w = w
        return (w * (xyz * xyz).sum() + w * (opacity * opacity).sum()).reshape(())

    @staticmethod
    def backward(ctx, g):
        import diff_gaussian_rasterization as dgr

        xyz, opacity = ctx.saved_tensors
        ex = dgr._exchange
        views = ex.leaf_bucket({"xyz": (xyz,), "opacity": (opacity,)})
        for name, leaf in (("xyz", xyz), ("opacity", opacity)):
            v = views[name][0]
            val = 2 * ctx.w * leaf.detach() * g
            if leaf.grad is None:
                v.copy_(val)
                leaf.grad = v
            else:
                v.add_(val)
        started_before = ex.pending
        ex.rasterizer_done(views)
        ctx.started = (started_before, ex.pending)
        _AllWriter.started.append(ctx.started)
        return None, None, None

    started = []


def _all_writer_worker(rank, world, port, out, views_per_step):
    _init(rank, world, port)
    from multiview import GradAllReduce

    torch.manual_seed(0)
    xyz, opacity = (torch.randn(s, requires_grad=True) for s in ((7, 3), (7, 1)))
    ar = GradAllReduce([xyz, opacity], views_per_step=views_per_step)
    probe = []
    for step in range(2):  # the first step probes the loss graph (no early start)
        for p in (xyz, opacity):
            p.grad = None
        _AllWriter.started = []
        for v in range(views_per_step):
            _AllWriter.apply(xyz, opacity, float(rank + 1) * (v + 1)).backward()
        started = list(_AllWriter.started)
        probe.append(ar._mode)
        ar()
    started = (started, probe)
    out[rank] = ([p.grad.clone() for p in (xyz, opacity)], [p.detach().clone() for p in (xyz, opacity)], started)
    ar.remove_hooks()
    dist.destroy_process_group()


@pytest.mark.parametrize("views_per_step", [1, 2])
def test_bucket_started_by_the_rasterizer_gloo_world2(views_per_step):
    """Every reduced leaf written by the fused backward: the all-reduce starts inside
    the step's last backward (not on an earlier one), and the sums are right."""
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_all_writer_worker, args=(2, port, out, views_per_step), nprocs=2, join=True)
        res = dict(out)
    (g0, p, s0), (g1, _, s1) = res[0], res[1]
    expect = [(0, 0)] * (views_per_step - 1) + [(0, 1)]
    assert s0 == s1 == (expect, ["probe", "early"])
    wsum = sum(float(r + 1) * (v + 1) for r in (0, 1) for v in range(views_per_step))
    for a, b, x in zip(g0, g1, p):
        assert torch.equal(a, b)
        torch.testing.assert_close(a, 2 * wsum * x, rtol=1e-6, atol=1e-6)


def _late_path_worker(rank, world, port, out, views_per_step, only_rank0):
    _init(rank, world, port)
    from multiview import GradAllReduce

    torch.manual_seed(0)
    xyz, opacity = (torch.randn(s, requires_grad=True) for s in ((7, 3), (7, 1)))
    ar = GradAllReduce([xyz, opacity], views_per_step=views_per_step)
    c = 0.5 * (rank + 1)
    res = []
    for step in range(3):
        for p in (xyz, opacity):
            p.grad = None
        _AllWriter.started = []
        for v in range(views_per_step):
            w = _AllWriter.apply(xyz, opacity, float(rank + 1) * (v + 1))
            if only_rank0 and rank != 0:
                w.backward()
                continue
            # a regulariser on a reduced leaf, formed before the render: AccumulateGrad(opacity)
            # waits for both paths, so it runs AFTER the writer's backward
            (c * (opacity * opacity).sum() + w).backward()
        mode = ar._mode
        ar()
        res.append((mode, list(_AllWriter.started), [p.grad.clone() for p in (xyz, opacity)]))
    out[rank] = (res, [p.detach().clone() for p in (xyz, opacity)])
    ar.remove_hooks()
    dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("views_per_step", [1, 2])
@pytest.mark.parametrize("only_rank0", [False, True])
def test_late_gradient_path_gloo_world2(views_per_step, only_rank0):
    """VERDICT r5 #6 / ADVICE r4-r5: another loss term on a reduced leaf, whose
    gradient reaches it after the rasterizer's backward — on both ranks, or on rank 0
    only.  The first step probes the graph (no early start); its summed flags put
    every rank in "late" mode, so no all-reduce starts before the backward is done,
    every rank issues the same collectives, and every step's gradients are the full
    sums, bit-identical on both ranks."""
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_late_path_worker, args=(2, port, out, views_per_step, only_rank0), nprocs=2, join=True)
        res = dict(out)
    (r0, p), (r1, _) = res[0], res[1]
    wsum = sum(float(r + 1) * (v + 1) for r in (0, 1) for v in range(views_per_step))
    creg = 2 * views_per_step * (0.5 if only_rank0 else 0.5 + 1.0)
    for step in range(3):
        (m0, s0, g0), (m1, s1, g1) = r0[step], r1[step]
        assert m0 == m1 == ("probe" if step == 0 else "late")
        assert all(b == 0 for _, b in s0 + s1)  # no early start, on any step
        for a, b in zip(g0, g1):
            assert torch.equal(a, b)
        torch.testing.assert_close(g0[0], 2 * wsum * p[0], rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(g0[1], (2 * wsum + creg) * p[1], rtol=1e-6, atol=1e-6)


def _graph_change_worker(rank, world, port, out):
    _init(rank, world, port)
    from multiview import GradAllReduce

    torch.manual_seed(0)
    xyz, opacity = (torch.randn(s, requires_grad=True) for s in ((7, 3), (7, 1)))
    ar = GradAllReduce([xyz, opacity])
    grads, raised = [], None
    for step in range(40):
        for p in (xyz, opacity):
            p.grad = None
        try:
            w = _AllWriter.apply(xyz, opacity, float(rank + 1))
            if rank == 0 and step >= 3:  # the loss graph changes on one rank after early starts began
                w = w + (opacity * opacity).sum()
            w.backward()
            ar()
        except RuntimeError as e:
            raised = (step, str(e))
            break
        grads.append([p.grad.clone() for p in (xyz, opacity)])
    out[rank] = (grads, raised)
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_late_gradient_after_early_start_raises_on_every_rank_gloo_world2():
    """A gradient path that appears on one rank only after early starts began: it is
    left out on that rank (the replicas stay bit-identical), and every rank raises the
    same RuntimeError at the same step — no rank issues a collective the other does
    not, so nothing hangs (the spawn runs under a timeout)."""
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_graph_change_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    (g0, e0), (g1, e1) = res[0], res[1]
    assert e0 is not None and e1 is not None and e0[0] == e1[0], (e0, e1)
    assert "after the bucket's all-reduce had started" in e0[1]
    assert len(g0) == len(g1) == e0[0]
    for a, b in zip(g0, g1):
        for x, y in zip(a, b):
            assert torch.equal(x, y)


class _MaybeWriter(torch.autograd.Function):
    """The rasterizer's contract in full: leaves it gets bucket views for are written
    there (and reported with rasterizer_done); the others get their gradients back
    through autograd."""

    @staticmethod
    def forward(ctx, xyz, opacity, w):
        ctx.save_for_backward(xyz, opacity)
        ctx.w = w
        return (w * (xyz * xyz).sum() + w * (opacity * opacity).sum()).reshape(())

    @staticmethod
    def backward(ctx, g):
        import diff_gaussian_rasterization as dgr

        xyz, opacity = ctx.saved_tensors
        ex = dgr._exchange
        views = ex.leaf_bucket({"xyz": (xyz,), "opacity": (opacity,)})
        back = []
        for name, leaf in (("xyz", xyz), ("opacity", opacity)):
            val = 2 * ctx.w * leaf.detach() * g
            if name not in views:
                back.append(val)
                continue
            v = views[name][0]
            if leaf.grad is None:
                v.copy_(val)
                leaf.grad = v
            else:
                v.add_(val)
            back.append(None)
        if views:
            ex.rasterizer_done(views)
        return back[0], back[1], None


def _two_calls_worker(rank, world, port, out):
    _init(rank, world, port)
    from multiview import GradAllReduce

    torch.manual_seed(0)
    xyz, opacity = (torch.randn(s, requires_grad=True) for s in ((7, 3), (7, 1)))
    ar = GradAllReduce([xyz, opacity])
    res = []
    for step in range(3):
        for p in (xyz, opacity):
            p.grad = None
        # two rasterizer calls in one backward: the second finds no bucket
        # once the first started the all-reduce, so the graph probe keeps early starts off
        (_MaybeWriter.apply(xyz, opacity, float(rank + 1)) + _MaybeWriter.apply(xyz, opacity, 2.0)).backward()
        mode = ar._mode
        ar()
        res.append((mode, [p.grad.clone() for p in (xyz, opacity)]))
    out[rank] = (res, [p.detach().clone() for p in (xyz, opacity)])
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_two_rasterizer_calls_in_one_backward_gloo_world2():
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_two_calls_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    (r0, p), (r1, _) = res[0], res[1]
    wsum = (1.0 + 2.0) + 2 * 2.0
    assert [r[0] for r in r0] == [r[0] for r in r1] == ["probe", "late", "late"]
    for step in range(3):
        for a, b, x in zip(r0[step][1], r1[step][1], p):
            assert torch.equal(a, b)
            torch.testing.assert_close(a, 2 * wsum * x, rtol=1e-6, atol=1e-6)


def _reuse_worker(rank, world, port, out):
    _init(rank, world, port)
    from multiview import GradAllReduce

    torch.manual_seed(0)
    xyz, opacity = (torch.randn(s, requires_grad=True) for s in ((7, 3), (7, 1)))
    ar = GradAllReduce([xyz, opacity])
    res = []
    for step in range(3):
        _AllWriter.apply(xyz, opacity, float(rank + 1) * (step + 1)).backward()
        bucket = ar()
        res.append((bucket.data_ptr(), [p.grad.clone() for p in (xyz, opacity)]))
        if step == 0:
            for p in (xyz, opacity):
                p.grad = None               # released: step 1 reuses the bucket
        elif step == 1:
            for p in (xyz, opacity):
                p.grad.zero_()              # still the views (zero_grad(set_to_none=False)): reused
    # a tensor of the caller's own in one leaf: the next bucket is a fresh one
    xyz.grad = xyz.grad.clone()
    opacity.grad = None
    ar.leaf_bucket({"opacity": (opacity,)})
    fresh = ar._bucket.data_ptr()
    ar()
    out[rank] = (res, [p.detach().clone() for p in (xyz, opacity)], fresh)
    ar.remove_hooks()
    dist.destroy_process_group()


def test_bucket_reused_only_when_released_gloo_world2():
    """The all-reduce bucket is reused step to step when every reduced leaf's .grad
    was set to None or is still its bucket view (as DDP's gradient_as_bucket_view),
    and not when the caller installed a tensor of its own; the reduced gradients are
    the ranks' sums either way (a kept view accumulates, as autograd would)."""
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_reuse_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    (r0, prm, fresh), (r1, _, _) = res[0], res[1]
    b = [x[0] for x in r0]
    assert b[1] == b[0] and b[2] == b[0] and fresh != b[0], (b, fresh)
    for step in range(3):
        for a, c in zip(r0[step][1], r1[step][1]):
            assert torch.equal(a, c)
    for step in (0, 1, 2):
        wsum = sum(float(r + 1) * (step + 1) for r in (0, 1))
        for g, x in zip(r0[step][1], prm):
            torch.testing.assert_close(g, 2 * wsum * x, rtol=1e-6, atol=1e-6)
