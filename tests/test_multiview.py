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
    ar = GradAllReduce(params)  # hooks: each gradient's all-reduce starts inside backward
    w = float(rank + 1)
    loss = sum((w * (i + 1) * p * p).sum() for i, p in enumerate(params))
    loss.backward()
    pending = len(ar._works)
    ar()
    out[rank] = ([p.detach().clone() for p in params], [p.grad.clone() for p in params], pending)
    ar.remove_hooks()
    dist.destroy_process_group()


def test_grad_all_reduce_overlapped_gloo_world2():
    """Overlapped mode: the all-reduces launch from post-accumulate-grad hooks during
    backward; after the wait every rank holds the sum of the ranks' gradients."""
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_cpu_overlap_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    p0, g0, n0 = res[0]
    p1, g1, n1 = res[1]
    assert n0 == n1 == 6  # one async all-reduce per parameter, launched during backward
    for i, (a, b, p) in enumerate(zip(g0, g1, p0)):
        assert torch.equal(a, b)
        # d/dp sum_r (r+1)(i+1) p^2 = 2 p (i+1) (1 + 2)
        torch.testing.assert_close(a, 2 * p * (i + 1) * 3.0)


def _gpu_worker(rank, world, port, out):
    _init(rank, world, port)
    import synthetic
    import train_step
    from multiview import GradAllReduce

    dev = torch.device("cuda:0")
    cam = synthetic.make_camera(160, 120, view=rank).to(dev)
    g = synthetic.make_gaussians(20_000, 3, seed=0).to(dev, requires_grad=True)
    target = synthetic.make_target(160, 120).to(dev)
    reducer = GradAllReduce(g.params())  # overlapped: the all-reduces start inside backward
    train_step.train_step(cam, g, target, torch.zeros(3, device=dev))
    assert len(reducer._works) == 6
    reducer()
    out[rank] = [p.grad.detach().cpu() for p in g.params()]
    dist.destroy_process_group()


@pytest.mark.gpu
def test_view_parallel_grads_equal_sum_of_views(dev):
    import synthetic
    import train_step

    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_gpu_worker, args=(2, port, out), nprocs=2, join=True)
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
