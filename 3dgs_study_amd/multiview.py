"""View-parallel training across the GPUs of one node.

The reference trains one view per iteration on one GPU (train.py:86-98).  Views are
independent given the Gaussians, so N ranks (one process per MI355X) each render
view ``rank`` (or ``rank::world``) of a fully replicated model, and the only exchange
is a SUM all-reduce of the leaf gradients per step — `torch.distributed` with the
"nccl" backend, which is RCCL over xGMI on ROCm.  The six leaf gradients of the
GaussianModel storage are xyz 3, f_dc 3, f_rest 3(M-1), opacity 1, scaling 3,
rotation 4 = 59 floats per Gaussian at SH3, 236 MB at 1M.  Identical reduced
gradients then drive identical optimizer steps, so the replicas stay equal.

Two modes:
  * overlapped (``overlap=True``, default): a post-accumulate-grad hook on every
    parameter starts that gradient's all-reduce (async, on RCCL's stream) the
    moment autograd has written it — xyz straight out of the rasterizer's
    backward, f_dc / f_rest after the SH ``cat`` backward, opacity / scaling /
    rotation after their activation backwards — so the exchange of the big
    f_rest block (76 % of the bytes) runs under the remaining backward kernels,
    and no flat copy of the gradients is made.  ``__call__`` waits for them.
  * flat (no pending hooks, e.g. gradients assigned by hand): the six gradients
    are packed into ONE fp32 bucket and reduced with one call.
"""
from __future__ import annotations

from typing import Sequence

import torch
import torch.distributed as dist


def views_for_rank(rank: int, world: int, num_views: int) -> list:
    """Round-robin view assignment: rank r renders views r, r+world, ..."""
    return list(range(rank, num_views, world))


class GradAllReduce:
    """Sum the gradients of `params` over the process group."""

    def __init__(self, params: Sequence[torch.Tensor], group=None, overlap: bool = True):
        self.params = list(params)
        self.group = group
        self.numel = sum(p.numel() for p in self.params)
        self._works = []
        self._hooks = []
        if overlap:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._launch))

    @property
    def nbytes(self) -> int:
        return self.numel * 4

    def _active(self) -> bool:
        return dist.is_initialized() and dist.get_world_size(self.group) > 1

    def _launch(self, p: torch.Tensor) -> None:
        if self._active():
            self._works.append(dist.all_reduce(p.grad, op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []

    def __call__(self):
        """Finish this step's exchange: wait for the overlapped all-reduces, or (none
        pending) reduce the current gradients as one flat bucket."""
        if self._works:
            for w in self._works:
                w.wait()
            self._works = []
            return None
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in self.params]
        flat = torch.cat([g.reshape(-1) for g in grads])
        if self._active():
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
        off = 0
        for p in self.params:
            n = p.numel()
            p.grad = flat[off:off + n].view_as(p)
            off += n
        return flat
