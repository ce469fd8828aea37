"""Fused leaf gradients (diff_gaussian_rasterization._leaf_plan): the backward writes
the gradients of GaussianModel's leaves itself when the caller's activations are
exactly the reference's (scene/gaussian_model.py:106-126: cat, exp, sigmoid,
F.normalize) and nothing else observes them; every other graph keeps upstream's
activation gradients.

CPU: the graph matching and gating rules, driven by a stand-in autograd Function
whose backward runs the same planner.  GPU: the fused leaf gradients against the
plain path (set_fused_leaf_grads(False)) bit for bit at configs B and C, with
fresh and accumulating .grad, two views per backward, and the Python branches."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import diff_gaussian_rasterization as dgr


def _leaves(P=6, M=16, requires=True):
    g = torch.Generator().manual_seed(0)
    mk = lambda *s: torch.randn(*s, generator=g).requires_grad_(requires)  # noqa: E731
    return dict(xyz=mk(P, 3), f_dc=mk(P, 1, 3), f_rest=mk(P, M - 1, 3), opacity=mk(P, 1), scaling=mk(P, 3),
                rotation=mk(P, 4))


class _Probe(torch.autograd.Function):
    """Stands in for _RasterizeGaussians: its backward records the planner's answer."""
    seen = []

    exchange = None  # an exchange stand-in (owns_hooks / leaf_bucket), as multiview.GradAllReduce

    @staticmethod
    def forward(ctx, means3D, sh, opacities, scales, rotations):
        ctx.save_for_backward(means3D, sh, opacities, scales, rotations)
        return means3D.sum() + sh.sum() + opacities.sum() + scales.sum() + rotations.sum()

    @staticmethod
    def backward(ctx, g):
        means3D, sh, opacities, scales, rotations = ctx.saved_tensors
        n = ctx.needs_input_grad
        needs = (n[0], False, n[1], False, n[2], n[3], n[4])
        plan = dgr._leaf_plan(ctx, needs, sh, torch.empty(0), opacities, scales, rotations, means3D, False,
                              _Probe.exchange)
        _Probe.seen.append({k: (v[1] if v[3] is None else (v[1], "bucket")) for k, v in plan.items()})
        return tuple(torch.zeros_like(x) for x in (means3D, sh, opacities, scales, rotations))


def _activations(L, normalize=None):
    sh = torch.cat((L["f_dc"], L["f_rest"]), dim=1)  # get_features
    rot = F.normalize(L["rotation"]) if normalize is None else normalize(L["rotation"])
    return L["xyz"], sh, torch.sigmoid(L["opacity"]), torch.exp(L["scaling"]), rot


def _plan(L, run=lambda out: out.backward(), **kw):
    _Probe.seen.clear()
    acts = _activations(L, **kw)
    out = _Probe.apply(*acts)
    run(out)
    return _Probe.seen[-1] if _Probe.seen else None


ALL = {"sh": 0, "scales": 0, "opacities": 0, "rotations": 0}


def test_reference_graph_is_fused():
    assert _plan(_leaves()) == ALL
    assert _plan(_leaves(M=1)) == ALL  # SH degree 0: an empty f_rest leaf


def test_existing_grad_accumulates():
    L = _leaves()
    for k in L:
        L[k].grad = torch.ones_like(L[k])
    assert _plan(L) == {k: 1 for k in ALL}
    L["f_rest"].grad = None  # the two SH leaves must agree
    assert "sh" not in _plan(L)
    L["scaling"].grad = torch.ones(6, 3).t().contiguous().t()  # not contiguous
    assert "scales" not in _plan(L)


def test_hooks_and_observers_keep_upstream_path():
    L = _leaves()
    L["scaling"].register_post_accumulate_grad_hook(lambda p: None)  # the exchange's all-reduce hooks
    L["f_dc"].register_hook(lambda g: g)
    assert _plan(L) == {"opacities": 0, "rotations": 0}
    L = _leaves()
    _Probe.seen.clear()
    acts = list(_activations(L))
    acts[2].retain_grad()
    _Probe.apply(*acts).backward()
    assert "opacities" not in _Probe.seen[-1]


def test_other_graphs_keep_upstream_path():
    hand = lambda r: r / r.norm(dim=1, keepdim=True)  # noqa: E731
    assert "rotations" not in _plan(_leaves(), normalize=hand)
    L = _leaves()
    L["f_dc"].requires_grad_(False)
    assert "sh" not in _plan(L)
    L = _leaves()
    assert _plan(L, run=lambda out: out.backward(inputs=[L["xyz"]])) == {}
    assert _plan(L, run=lambda out: torch.autograd.grad(out, [L["rotation"]])) == {}
    assert _plan(L, run=lambda out: out.backward(create_graph=True)) == {}


def test_oracle_leaf_formulas_equal_torch_autograd():
    """oracle.activation_leaf_grads (the arithmetic gsr_leaf_grads asks the library
    for) equals torch's own CPU autograd of cat / exp / sigmoid / F.normalize bit for
    bit."""
    from oracle import oracle as o

    P, g = 50_000, torch.Generator().manual_seed(0)
    L = {k: v.detach().requires_grad_() for k, v in _leaves(P).items()}
    L["rotation"].data[:7] *= 1e-3  # short quaternions
    _, sh, op, sc, rot = _activations(L)
    norm = rot.grad_fn.next_functions[1][0].next_functions[0][0].next_functions[0][0]._saved_result.detach().clone()
    d = [torch.randn(t.shape, generator=g) for t in (sh, op, sc, rot)]
    torch.autograd.backward([sh, op, sc, rot], d)
    lg = o.activation_leaf_grads(d[0].numpy(), d[1].numpy(), d[2].numpy(), d[3].numpy(), op.detach().numpy(),
                                 sc.detach().numpy(), rot.detach().numpy(), norm.numpy(),
                                 sum_order="sequential")  # torch's CPU reduction (its GPU one pairs: the library's)
    for name, leaf in (("dsh_dc", "f_dc"), ("dsh_rest", "f_rest"), ("dscaling", "scaling"), ("dopacity", "opacity"),
                       ("drotation", "rotation")):
        np.testing.assert_array_equal(lg[name], L[leaf].grad.numpy(), err_msg=name)


def test_switch():
    prev = dgr.set_fused_leaf_grads(False)
    try:
        assert dgr._fused_leaf_grads is False and not dgr._fusion_on(None)
        dgr.set_fused_leaf_grads(None)
        assert dgr._fusion_on(None)  # no process group: automatic = on
    finally:
        dgr.set_fused_leaf_grads(prev)


class _Exchange:
    """The interface multiview.GradAllReduce offers the plan: its own hooks on the
    reduced leaves, and bucket views for them."""

    def __init__(self, L, reduced=("xyz", "opacity", "scaling", "rotation")):
        self.reduced = [L[k] for k in reduced]
        self.bucket = torch.zeros(sum(p.numel() for p in self.reduced))
        self.views, self.ids, off = [], set(), 0
        for p in self.reduced:
            self.views.append(self.bucket[off:off + p.numel()].view_as(p))
            off += p.numel()
            self.ids.add(p.register_post_accumulate_grad_hook(lambda p: None).id)

    def owns_hooks(self, leaf):
        return set(getattr(leaf, "_post_accumulate_grad_hooks", None) or {}) <= self.ids

    def leaf_bucket(self, leaves):
        out = {}
        for name, ls in leaves.items():
            idx = [next((i for i, p in enumerate(self.reduced) if p is x), -1) for x in ls]
            if all(i >= 0 for i in idx):
                out[name] = tuple(self.views[i] for i in idx)
        return out


def test_exchange_bucket_plan():
    """With an exchange installed, leaves carrying only ITS hooks stay fusable, the
    xyz leaf (means3D itself) joins the plan, and the reduced leaves get bucket
    views; the SH leaves, not in this exchange's bucket, are written as usual."""
    L = _leaves()
    _Probe.exchange = _Exchange(L)
    try:
        assert _plan(L) == {"means3D": (0, "bucket"), "opacities": (0, "bucket"), "scales": (0, "bucket"),
                            "rotations": (0, "bucket"), "sh": 0}
        L2 = _leaves()
        L2["opacity"].register_post_accumulate_grad_hook(lambda p: None)  # a hook of someone else's
        _Probe.exchange = _Exchange(L2)
        assert "opacities" not in _plan(L2)
    finally:
        _Probe.exchange = None
    # without an exchange the xyz leaf is left to autograd (it steals the tensor anyway)
    assert "means3D" not in _plan(_leaves())


def _ddp_gate_worker(rank, world, port, out):
    import os

    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    import diff_gaussian_rasterization as d

    prev = d.set_fused_leaf_grads(None)
    res = [d._fusion_on(None), d._fusion_on(object())]
    d.set_fused_leaf_grads(True)
    res.append(d._fusion_on(None))
    d.set_fused_leaf_grads(prev)
    out[rank] = res
    dist.destroy_process_group()


def test_fusion_off_in_multi_rank_group_without_exchange():
    """a DDP-wrapped model's reducer hooks AccumulateGrad nodes from C++,
    invisible to the plan; in a process group of more than one rank the fused path
    turns itself off unless our exchange is installed (or it is forced on)."""
    import torch.multiprocessing as mp

    from test_multiview import _free_port

    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_ddp_gate_worker, args=(2, _free_port(), out), nprocs=2, join=True)
        res = dict(out)
    assert res[0] == res[1] == [False, True, True]


# ---------------------------------------------------------------- GPU: fused == plain
def _isolated_scene(W=256, H=192, per_quadrant=3, seed=0):
    """Small Gaussians (0.55 px after the 0.3 low-pass) whose means sit within 0.5 px
    of an 8x8 quadrant's centre: each reaches one quadrant only, so its accumulator
    row gets exactly one atomic and the backward is deterministic run to run (in
    general the atomics' order varies and gradients differ in the last bits)."""
    import synthetic

    cam = synthetic.make_camera(W, H, view=1)
    rng = np.random.default_rng(seed)
    qx, qy = np.meshgrid(np.arange(W // 8), np.arange(H // 8))
    q = np.stack([qx.ravel(), qy.ravel()], 1).repeat(per_quadrant, 0)
    pix = q * 8 + 3.5 + rng.uniform(-0.5, 0.5, q.shape)
    z = rng.uniform(4.0, 8.0, len(pix))
    fx = W / (2 * np.tan(cam.FoVx / 2))
    fy = H / (2 * np.tan(cam.FoVy / 2))
    pc = np.stack([(pix[:, 0] - (W - 1) / 2) / fx * z, (pix[:, 1] - (H - 1) / 2) / fy * z, z, np.ones_like(z)], 1)
    c2w = torch.linalg.inv(cam.world_view_transform.T.double()).numpy()
    xyz = (pc @ c2w.T)[:, :3].astype(np.float32)
    g = synthetic.make_gaussians(len(xyz), 3, seed=seed, scale_range=(0.0005, 0.001))
    g.xyz = torch.from_numpy(xyz)
    return cam, g


def _run(cam, g, dev, dL, fused, views=1, pre_grad=False, python_branch=False):
    import train_step

    gd = g.to(dev, requires_grad=True)
    if pre_grad:
        for p in gd.params():
            p.grad = torch.full_like(p, 0.25)
    prev = dgr.set_fused_leaf_grads(fused)
    try:
        loss = 0
        for v in range(views):
            out = train_step.render(cam.to(dev), gd, torch.zeros(3, device=dev), scaling_modifier=1.0 + 0.1 * v,
                                    convert_SHs_python=python_branch, compute_cov3D_python=python_branch)
            loss = loss + (out["render"] * dL).sum()
        loss.backward()
        plan = dgr.last_leaf_plan
    finally:
        dgr.set_fused_leaf_grads(prev)
    torch.cuda.synchronize()
    return [p.grad.cpu() for p in gd.params()], out["viewspace_points"].grad.cpu(), plan


NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")
FUSED = ("opacities", "rotations", "scales", "sh")


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [{}, {"pre_grad": True}, {"views": 2}, {"python_branch": True}],
                         ids=["fresh", "accumulate", "two_views", "python_branch"])
def test_fused_leaf_grads_bit_identical(dev, kw):
    """Deterministic scene: the fused leaf gradients equal the plain path's (torch's
    cat / exp / sigmoid / normalize backwards + AccumulateGrad) bit for bit, for a
    fresh .grad, an existing one, two views into one backward, and the Python branch
    (only the opacity is a sigmoid leaf there)."""
    from helpers import random_dL

    cam, g = _isolated_scene()
    dL = torch.from_numpy(random_dL(cam.image_height, cam.image_width)).to(dev) * 1e4
    ref, ref_vs, plan0 = _run(cam, g, dev, dL, False, **kw)
    ref2, _, _ = _run(cam, g, dev, dL, False, **kw)
    got, got_vs, plan = _run(cam, g, dev, dL, True, **kw)
    assert plan0 == () and plan == (("opacities",) if kw.get("python_branch") else FUSED)
    from helpers import rel_l2

    for name, a, b, b2 in zip(NAMES, got, ref, ref2):
        np.testing.assert_array_equal(b.numpy(), b2.numpy(), err_msg=f"{name}: plain path not deterministic")
        assert a.shape == b.shape and a.is_contiguous(), name
        assert float(b.abs().max()) > 0, name
        if name == "rotation":
            # the normalize backward's 4-term sum is paired like torch's GPU reduction
            # ((a0 + a1) + (a2 + a3)), an implementation detail of torch's reduce kernel
            # that may change across versions, and with two renders autograd sums the
            # terms into the leaf in its own engine order: held to a few ulp here
            # (ADVICE r3), every other leaf bit for bit
            scale = float(b.abs().max())
            assert float((a - b).abs().max()) <= 8 * 2.0 ** -23 * scale, name
            assert rel_l2(a.numpy(), b.numpy()) <= 1e-6
            continue
        np.testing.assert_array_equal(a.numpy(), b.numpy(), err_msg=name)
    np.testing.assert_array_equal(got_vs.numpy(), ref_vs.numpy())


def _compare_tol(W, H, P, dev):
    """Full-size scenes: the accumulator atomics reorder each Gaussian's sums run to
    run, so the plain path does not repeat itself bit for bit either.  Fused vs plain
    is held to that noise floor: rel-L2 within 4e-6 or 4x what two plain runs differ
    by (measured ~1e-6 at config C for the rotation, whose normalize backward removes
    the radial component and so cancels most of each gradient)."""
    from helpers import case, random_dL, rel_l2

    cam, g = case(P, W, H, 3, seed=2, view=1)
    dL = torch.from_numpy(random_dL(H, W)).to(dev)
    got, got_vs, plan = _run(cam, g, dev, dL, True)
    ref, ref_vs, plan0 = _run(cam, g, dev, dL, False)
    ref2, _, _ = _run(cam, g, dev, dL, False)
    assert plan0 == () and plan == FUSED
    for name, a, b, b2 in zip(NAMES, got, ref, ref2):
        assert a.shape == b.shape and a.is_contiguous(), name
        noise = rel_l2(b2.numpy(), b.numpy())
        assert noise <= 4e-6, name
        assert rel_l2(a.numpy(), b.numpy()) <= max(4e-6, 4 * noise), name
    assert rel_l2(got_vs.numpy(), ref_vs.numpy()) <= 4e-6


@pytest.mark.gpu
def test_fused_leaf_grads_config_b(dev):
    _compare_tol(800, 800, 100_000, dev)


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.timeout(600)
def test_fused_leaf_grads_config_c(dev):
    _compare_tol(1920, 1080, 1_000_000, dev)
