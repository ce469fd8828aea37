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
    parameter counts the backwards that accumulate into it and, on the step's last
    one (``views_per_step`` backwards per rank and step), starts that gradient's
    all-reduce (async, on RCCL's stream) — xyz straight out of the rasterizer's
    backward, f_dc / f_rest after the SH ``cat`` backward, opacity / scaling /
    rotation after their activation backwards — so the exchange runs under the
    remaining backward kernels and no flat copy is made.  ``__call__`` waits.
  * flat: every gradient whose all-reduce did not start from a hook (no hook on a
    replaced tensor, gradients assigned by hand, fewer backwards than announced) is
    packed into ONE fp32 bucket and reduced with one call in ``__call__``.

Parameters may be given as a zero-argument callable returning the current tensors
(and ``sh`` likewise): the reference's densify / prune replaces every parameter with
a new ``nn.Parameter`` (scene/gaussian_model.py cat_tensors_to_optimizer /
_prune_optimizer), and ``__call__`` re-binds its hooks to whatever the callable
returns, so the exchange follows the model instead of going stale.
"""
from __future__ import annotations

from typing import Callable, Sequence, Union

import torch
import torch.distributed as dist

ParamSource = Union[Sequence[torch.Tensor], Callable[[], Sequence[torch.Tensor]]]


def views_for_rank(rank: int, world: int, num_views: int) -> list:
    """Round-robin view assignment: rank r renders views r, r+world, ..."""
    return list(range(rank, num_views, world))


class GradAllReduce:
    """Sum the gradients of `params` over the process group.

    ``sh=(xyz, f_dc, f_rest)`` (three of `params`, or a callable returning them)
    exchanges the SH gradient as per-view colour gradients instead (module
    docstring); it engages when the group has more than one rank, or always with
    ``sh_force=True`` (tests).  ``views_per_step``: backwards each rank runs per step
    (the overlapped all-reduces start on the last one).  ``rebuild`` replaces the HIP
    kernel that turns gathered records into the SH gradients (CPU tests only).
    ``comm_force=True`` runs every collective even in a one-rank group (tests: the
    RCCL calls on a one-GPU box)."""

    def __init__(self, params: ParamSource, group=None, overlap: bool = True, sh=None, sh_force: bool = False,
                 rebuild=None, views_per_step: int = 1, comm_force: bool = False):
        if views_per_step < 1:
            raise ValueError("views_per_step must be >= 1")
        self._params_src = params
        self._sh_src = sh
        self.group = group
        self.overlap = overlap
        self.views_per_step = views_per_step
        self._comm_force = comm_force  # run the collectives even in a one-rank group (RCCL smoke tests)
        self._rebuild = rebuild
        self._works = []       # (param, work) of the all-reduces started from hooks
        self._hooks = []
        self._counts = {}      # id(param) -> backwards accumulated into it this step
        self._gathers = []
        self._sh = None
        self._prev_sink = None
        self._sink_installed = False
        self._sh_on = sh is not None and (sh_force or self._active())
        self._bind()
        if self._sh_on:
            from diff_gaussian_rasterization import set_sh_grad_sink
            self._prev_sink = set_sh_grad_sink(self)
            self._sink_installed = True

    # ---- binding to the current parameter tensors
    def _resolve(self):
        params = list(self._params_src() if callable(self._params_src) else self._params_src)
        sh = None
        if self._sh_on:
            sh = tuple(self._sh_src() if callable(self._sh_src) else self._sh_src)
            xyz, f_dc, f_rest = sh
            if not any(f_dc is p for p in params) or not any(f_rest is p for p in params):
                raise ValueError("sh=(xyz, f_dc, f_rest) must be among params")
        return params, sh

    def _bind(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self.params, self._sh = self._resolve()
        self.numel = sum(p.numel() for p in self.params)
        self._reduced = [p for p in self.params if self._sh is None or not any(p is q for q in self._sh[1:])]
        self._counts = {id(p): 0 for p in self._reduced}
        # hooks only while there is something to exchange: with one rank the
        # rasterizer may then write the leaves' gradients itself (diff_gaussian_
        # rasterization's fused leaf gradients skip leaves that carry hooks)
        if self.overlap and self._active():
            for p in self._reduced:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._launch))

    def _stale(self) -> bool:
        params, sh = self._resolve()
        return (len(params) != len(self.params) or any(a is not b for a, b in zip(params, self.params))
                or (sh is not None and any(a is not b for a, b in zip(sh, self._sh))))

    @property
    def nbytes(self) -> int:
        """Bytes each rank contributes per step: the all-reduced gradients, plus one
        SH record per view when the SH exchange is on."""
        n = sum(p.numel() for p in self._reduced) * 4
        if self._sh is not None:
            from diff_gaussian_rasterization import _C
            n += _C.sh_record_floats(self._sh[0].size(0)) * 4 * self.views_per_step
        return n

    @property
    def sh_exchange(self) -> bool:
        return self._sh is not None

    def _active(self) -> bool:
        return dist.is_initialized() and (dist.get_world_size(self.group) > 1 or self._comm_force)

    # ---- the rasterizer's SH sink (diff_gaussian_rasterization.set_sh_grad_sink)
    def accepts(self, sh: torch.Tensor, means3D: torch.Tensor) -> bool:
        """True when this backward's SH input is the bound model's.  With more than
        one rank a mismatch raises: a silent local dsh would leave this rank's SH
        gradient out of the exchange and the replicas would drift apart."""
        if self._stale():  # the model's tensors were replaced (densify / prune): follow them
            self._bind()
        xyz, f_dc, f_rest = self._sh
        ok = (means3D.data_ptr() == xyz.data_ptr() and sh.size(0) == xyz.size(0)
              and sh.size(1) == f_dc.size(1) + f_rest.size(1))
        if not ok and self._active():
            raise RuntimeError("GradAllReduce: the rasterizer's SH input is not the bound model's "
                               f"(means3D {tuple(means3D.shape)} vs xyz {tuple(xyz.shape)}); pass params/sh as "
                               "callables that return the current tensors")
        return ok

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
        # gathered buffers hold [rank 0 .. world-1] per push; with several views per
        # rank the sum runs push by push (identical order on every rank)
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
        k = id(p)
        if k not in self._counts or not self._active():  # one rank: nothing to exchange
            return
        self._counts[k] += 1
        if self._counts[k] > self.views_per_step:
            raise RuntimeError(f"GradAllReduce: {self._counts[k]} backwards accumulated into a parameter in one step "
                               f"(views_per_step={self.views_per_step}); its all-reduce already started")
        if self._counts[k] == self.views_per_step and self._active():
            self._works.append((p, dist.all_reduce(p.grad, op=dist.ReduceOp.SUM, group=self.group, async_op=True)))

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
        if self._sink_installed:
            from diff_gaussian_rasterization import set_sh_grad_sink
            set_sh_grad_sink(self._prev_sink)
            self._sink_installed = False
            self._sh = None
            self._sh_on = False

    def __call__(self):
        """Finish this step's exchange: wait for the overlapped all-reduces, reduce
        every other gradient as one flat bucket, then rebuild the SH gradients from
        the gathered colour gradients (SH exchange on).  Returns the flat bucket (or
        None when every gradient went through a hook)."""
        done = set()
        for p, w in self._works:
            w.wait()
            done.add(id(p))
        self._works = []
        if self._stale():
            # the model's tensors were replaced since the hooks were bound (densify /
            # prune): their gradients go through the flat bucket this step, and the
            # hooks move to them for the next
            self._bind()
        rest = [p for p in self._reduced if id(p) not in done]
        flat = None
        if rest:
            grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in rest]
            flat = torch.cat([g.reshape(-1) for g in grads])
            if self._active():
                dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            off = 0
            for p in rest:
                n = p.numel()
                p.grad = flat[off:off + n].view_as(p)
                off += n
        if self._sh is not None:
            self._finish_sh()
        for k in self._counts:
            self._counts[k] = 0
        return flat


@torch.no_grad()
def reduce_densification_stats(xyz_gradient_accum: torch.Tensor, denom: torch.Tensor, max_radii2D: torch.Tensor,
                               group=None, force: bool = False):
    """The ranks' densification statistics combined for a densify step: SUM of the
    accumulated screen-space gradient norms and of the visibility counts, MAX of the
    largest screen radii (scene/gaussian_model.py:565-581 accumulates them per view;
    train.py:126-127 and :130-136 use them), so every rank densifies and prunes the
    same Gaussians and the replicas stay identical.  Returns reduced copies
    (xyz_gradient_accum, denom, max_radii2D) and leaves the per-rank accumulators
    as they are, so calling it again (another caller, a non-densify iteration)
    cannot count a rank's views twice; densify_and_prune reads the copies and the
    accumulators are reset as upstream resets them (densification_postfix)."""
    if not (dist.is_initialized() and (dist.get_world_size(group) > 1 or force)):
        return xyz_gradient_accum.clone(), denom.clone(), max_radii2D.clone()
    both = torch.cat([xyz_gradient_accum.reshape(-1), denom.reshape(-1)])
    mx = max_radii2D.clone()
    w1 = dist.all_reduce(both, op=dist.ReduceOp.SUM, group=group, async_op=True)
    w2 = dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group, async_op=True)
    w1.wait()
    w2.wait()
    n = xyz_gradient_accum.numel()
    return both[:n].view_as(xyz_gradient_accum), both[n:].view_as(denom), mx
