"""View-parallel training across the GPUs of one node.

The reference trains one view per iteration on one GPU (train.py:86-98).  Views are
independent given the Gaussians, so N ranks (one process per MI355X) each render
view ``rank`` (or ``rank::world``) of a fully replicated model, and the only exchange
is a SUM all-reduce of the leaf gradients per step — `torch.distributed` with the
"nccl" backend, which is RCCL over xGMI on ROCm.  The six leaf gradients of the
GaussianModel storage are xyz 3, f_dc 3, f_rest 3(M-1), opacity 1, scaling 3,
rotation 4 = 59 floats per Gaussian at SH3, 236 MB at 1M.  Identical reduced
gradients then drive identical optimizer steps, so the replicas stay equal.

SH gradient as colour gradients (``sh=(xyz, f_dc, f_rest)``).  Per view, upstream's SH
backward makes dL/dsh the outer product basis(dir_v) (x) dL/dRGB_v (backward.cu
computeColorFromSH), so the 48 SH floats per Gaussian — 76 % of the bucket — need not
be all-reduced: while the exchange is installed as the rasterizer's SH sink
(``diff_gaussian_rasterization.set_sh_grad_sink``), each rank's backward writes the
12-byte clamp-masked colour gradient of its view into a record (with the camera
centre and SH degree), the records are all-gathered (async, launched inside the
backward), and every rank rebuilds f_dc.grad / f_rest.grad = sum over views in view
order with one HIP kernel (``_C.sh_grad_from_colors``): identical on every rank, and
equal to the sum of the single-view gradients.  Per GPU and step at 1M Gaussians and
8 ranks the ring traffic drops from 2·(7/8)·236 MB = 413 MB to 2·(7/8)·44 MB
(xyz, opacity, scaling, rotation all-reduced) + 7·12 MB (records received) = 161 MB.
It also skips the 192 MB dsh write and the SH ``cat`` backward on every rank.

Two modes for the all-reduced gradients:
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
    """Sum the gradients of `params` over the process group.

    ``sh=(xyz, f_dc, f_rest)`` (three of `params`) exchanges the SH gradient as
    per-view colour gradients instead (module docstring); it engages when the group
    has more than one rank, or always with ``sh_force=True`` (tests).  ``rebuild``
    replaces the HIP kernel that turns gathered records into the SH gradients (CPU
    tests only)."""

    def __init__(self, params: Sequence[torch.Tensor], group=None, overlap: bool = True, sh=None,
                 sh_force: bool = False, rebuild=None):
        self.params = list(params)
        self.group = group
        self.numel = sum(p.numel() for p in self.params)
        self._works = []
        self._hooks = []
        self._gathers = []
        self._sh = None
        self._prev_sink = None
        if sh is not None and (sh_force or self._active()):
            xyz, f_dc, f_rest = sh
            if not any(f_dc is p for p in self.params) or not any(f_rest is p for p in self.params):
                raise ValueError("sh=(xyz, f_dc, f_rest) must be among params")
            self._sh = (xyz, f_dc, f_rest)
            self._rebuild = rebuild
            from diff_gaussian_rasterization import set_sh_grad_sink
            self._prev_sink = set_sh_grad_sink(self)
        self._reduced = [p for p in self.params if self._sh is None or not any(p is q for q in self._sh[1:])]
        if overlap:
            for p in self._reduced:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._launch))

    @property
    def nbytes(self) -> int:
        """Bytes each rank contributes per step: the all-reduced gradients, plus one
        SH record per view when the SH exchange is on."""
        n = sum(p.numel() for p in self._reduced) * 4
        if self._sh is not None:
            from diff_gaussian_rasterization import _C
            n += _C.sh_record_floats(self._sh[0].size(0)) * 4
        return n

    @property
    def sh_exchange(self) -> bool:
        return self._sh is not None

    def _active(self) -> bool:
        return dist.is_initialized() and dist.get_world_size(self.group) > 1

    # ---- the rasterizer's SH sink (diff_gaussian_rasterization.set_sh_grad_sink)
    def accepts(self, sh: torch.Tensor, means3D: torch.Tensor) -> bool:
        xyz, f_dc, f_rest = self._sh
        return (means3D.data_ptr() == xyz.data_ptr() and sh.size(0) == xyz.size(0)
                and sh.size(1) == f_dc.size(1) + f_rest.size(1))

    def record(self, P: int) -> torch.Tensor:
        from diff_gaussian_rasterization import _C
        return torch.empty(_C.sh_record_floats(P), dtype=torch.float32, device=self._sh[0].device)

    def push(self, rec: torch.Tensor, campos: torch.Tensor, sh_degree: int) -> None:
        rec[0:3].copy_(campos.reshape(-1)[:3])
        rec[3:4].fill_(float(sh_degree))
        if self._active():
            world = dist.get_world_size(self.group)
            out = torch.empty(world * rec.numel(), dtype=rec.dtype, device=rec.device)
            work = dist.all_gather_into_tensor(out, rec, group=self.group, async_op=True)
            self._gathers.append((out, world, work))
        else:
            self._gathers.append((rec, 1, None))

    def _finish_sh(self) -> None:
        xyz, f_dc, f_rest = self._sh
        if not self._gathers:
            return
        for _, _, w in self._gathers:
            if w is not None:
                w.wait()
        recs = torch.cat([o for o, _, _ in self._gathers]) if len(self._gathers) > 1 else self._gathers[0][0]
        nviews = sum(n for _, n, _ in self._gathers)
        self._gathers = []
        dc = torch.empty_like(f_dc)
        rest = torch.empty_like(f_rest)
        if self._rebuild is not None:
            self._rebuild(xyz.detach(), recs, nviews, dc, rest)
        else:
            from diff_gaussian_rasterization import _C
            _C.sh_grad_from_colors(xyz.detach(), recs, nviews, dc, rest if rest.numel() else None)
        for p, g in ((f_dc, dc), (f_rest, rest)):
            if p.grad is None:
                p.grad = g
            else:
                p.grad.add_(g)

    def _launch(self, p: torch.Tensor) -> None:
        if self._active():
            self._works.append(dist.all_reduce(p.grad, op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
        if self._sh is not None:
            from diff_gaussian_rasterization import set_sh_grad_sink
            set_sh_grad_sink(self._prev_sink)
            self._sh = None

    def __call__(self):
        """Finish this step's exchange: wait for the overlapped all-reduces, or (none
        pending) reduce the current gradients as one flat bucket; then rebuild the SH
        gradients from the gathered colour gradients (SH exchange on)."""
        if self._works:
            for w in self._works:
                w.wait()
            self._works = []
            if self._sh is not None:
                self._finish_sh()
            return None
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in self._reduced]
        flat = torch.cat([g.reshape(-1) for g in grads])
        if self._active():
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
        off = 0
        for p in self._reduced:
            n = p.numel()
            p.grad = flat[off:off + n].view_as(p)
            off += n
        if self._sh is not None:
            self._finish_sh()
        return flat
