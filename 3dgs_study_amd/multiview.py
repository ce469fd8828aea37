"""View-parallel training across the GPUs of one node.

The reference trains one view per iteration on one GPU (train.py:86-98).  Views are
independent given the Gaussians, so N ranks (one process per MI355X) each render
view ``rank`` (or ``rank::world``) of a fully replicated model, and the only exchange
is one SUM all-reduce of the leaf gradients per step — `torch.distributed` with the
"nccl" backend, which is RCCL over xGMI on ROCm.  The six leaf gradients of the
GaussianModel storage (xyz 3, f_dc 3, f_rest 3(M-1), opacity 1, scaling 3,
rotation 4 = 59 floats per Gaussian at SH3, 236 MB at 1M) are packed into ONE flat
fp32 bucket: a single large message keeps every xGMI link busy instead of paying
per-tensor launch and ring-setup latency six times.  Identical reduced gradients
then drive identical optimizer steps, so the replicas stay equal.
"""
from __future__ import annotations

from typing import Sequence

import torch
import torch.distributed as dist


def views_for_rank(rank: int, world: int, num_views: int) -> list:
    """Round-robin view assignment: rank r renders views r, r+world, ..."""
    return list(range(rank, num_views, world))


class GradAllReduce:
    """Sum the gradients of `params` over the process group with one all-reduce."""

    def __init__(self, params: Sequence[torch.Tensor], group=None):
        self.params = list(params)
        self.group = group
        self.numel = sum(p.numel() for p in self.params)

    @property
    def nbytes(self) -> int:
        return self.numel * 4

    def __call__(self) -> torch.Tensor:
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in self.params]
        flat = torch.cat([g.reshape(-1) for g in grads])
        if dist.is_initialized() and dist.get_world_size(self.group) > 1:
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
        off = 0
        for p in self.params:
            n = p.numel()
            p.grad = flat[off:off + n].view_as(p)
            off += n
        return flat
