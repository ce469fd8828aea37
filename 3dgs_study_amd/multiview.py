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

One bucket for the all-reduced gradients.  Every gradient the exchange sums
(xyz, opacity, scaling, rotation — and f_dc / f_rest without the SH exchange) lives
in ONE flat fp32 bucket per step, reduced by ONE all-reduce:
  * overlapped (``overlap=True``, default): the rasterizer's fused leaf gradients
    (diff_gaussian_rasterization, ``_leaf_plan``) are written by its backward
    kernel straight into bucket views that become the leaves' ``.grad`` — the xyz
    gradient included — so no activation backward, AccumulateGrad copy or pack
    copy runs; a post-accumulate-grad hook on every parameter queues a callback at
    the end of the autograd pass, which (on the step's last backward,
    ``views_per_step``) copies any gradient that is not in the bucket yet (another
    graph, an unfusable input) into it and starts the bucket's all-reduce, async
    on RCCL's stream.  ``__call__`` makes the compute stream wait for it.
  * flat (``overlap=False``): nothing starts during the backward; ``__call__``
    packs every gradient into the bucket and reduces it.
At 1M Gaussians the bucket is 44 MB with the SH exchange (one all-reduce instead of
four per-parameter ones), and each rank's backward runs no torch kernel after the
rasterizer's own at any N.

Parameters may be given as a zero-argument callable returning the current tensors
(and ``sh`` likewise): the reference's densify / prune replaces every parameter with
a new ``nn.Parameter`` (scene/gaussian_model.py cat_tensors_to_optimizer /
_prune_optimizer), and ``__call__`` re-binds its hooks to whatever the callable
returns, so the exchange follows the model instead of going stale.
"""
from __future__ import annotations

import os
import time
from typing import Callable, Sequence, Union

import torch
import torch.distributed as dist

ParamSource = Union[Sequence[torch.Tensor], Callable[[], Sequence[torch.Tensor]]]


class _Queued:
    """A collective queued in line on the compute stream: nothing left to wait for."""

    @staticmethod
    def wait():
        return True


_QUEUED = _Queued()


def views_for_rank(rank: int, world: int, num_views: int) -> list:
    """Round-robin view assignment: rank r renders views r, r+world, ..."""
    return list(range(rank, num_views, world))


class GradAllReduce:
    """Sum the gradients of `params` over the process group.

    ``sh=(xyz, f_dc, f_rest)`` (three of `params`, or a callable returning them)
    exchanges the SH gradient as per-view colour gradients instead (module
    docstring); it engages when the group has more than one rank, or always with
    ``sh_force=True`` (tests).  ``views_per_step``: backwards each rank runs per step
    (the bucket's all-reduce starts at the end of the last one).  ``rebuild``
    replaces the HIP kernel that turns gathered records into the SH gradients (CPU
    tests only).  ``comm_force=True`` runs every collective even in a one-rank
    group (tests and the bench's forced one-rank exchange: the RCCL calls on a
    one-GPU box).  ``timing=True`` records, per ``__call__``, how long the compute
    stream waits for the exchange and how long the SH rebuild takes (``stats()``).

    The leaves' ``.grad`` are views of one flat bucket, and the bucket is reused the
    next step when the caller let go of them (``.grad = None``) or left the views in
    place — DDP's ``gradient_as_bucket_view``: a reference kept to last step's
    ``.grad`` tensor is overwritten by the next step's gradients (clone it to keep it).

    Early start and the loss graph (DDP's ``static_graph``).  The bucket's
    all-reduce starts inside the rasterizer's backward (``rasterizer_done``) once the
    first step after (re)binding has shown, on every rank, that no other gradient path
    reaches a reduced leaf after the rasterizer's.  That probe step starts it at the
    end of the backward instead, and each rank flags whether such a late gradient came
    (a reduced leaf's accumulate hook after the rasterizer's backward); the flags are
    summed in one spare float of the bucket, so every rank reads the same answer one
    step later: none -> early starts from then on; any -> never (the late gradients are
    packed into the bucket at the end of each backward, so the sums stay right).  If a
    late gradient appears after early starts began (the loss graph changed), it is
    left out on its rank (the replicas stay identical), the flag rides in the next
    buckets, and every rank raises the same RuntimeError at the check after it (every
    ``FLAG_EVERY`` steps) — no rank issues a collective the others do not."""

    def __init__(self, params: ParamSource, group=None, overlap: bool = True, sh=None, sh_force: bool = False,
                 rebuild=None, views_per_step: int = 1, comm_force: bool = False, timing: bool = False):
        if views_per_step < 1:
            raise ValueError("views_per_step must be >= 1")
        self._params_src = params
        self._sh_src = sh
        self.group = group
        self.overlap = overlap
        self.views_per_step = views_per_step
        self._comm_force = comm_force  # run the collectives even in a one-rank group (RCCL smoke tests)
        self._rebuild = rebuild
        self._hooks = []
        self._gathers = []
        self._sh = None
        self._bucket = None     # this step's flat fp32 bucket over self._reduced
        self._views = None      # its per-parameter views
        self._work = None       # the bucket's async all-reduce
        self._early = False     # ... started by the rasterizer (rasterizer_done): the leaves' .grad are cleared
        self._backwards = 0     # backwards finished this step
        self._pushes = 0        # SH records pushed this step (views_per_step of them)
        # early start (class docstring): "probe" until every rank's first step has shown
        # no late gradient path, then "early"; "late" when one has
        self._mode = "probe"
        self._rast_seen = False  # this step's rasterizer backward has run (late = hooks after it)
        self._view_ver = {}      # the bucket views' versions at the rasterizer's backward
        self._late_local = False  # a late gradient reached a reduced leaf on this rank (sticky in "early")
        self._flag_read = None   # (pinned float, event, mode when sent): the summed flag slot of a bucket
        self._flag_send = None   # the mode of this step's flag, to be copied to the host in __call__
        self._slot_fresh = True  # the bucket's flag slot holds garbage (a new bucket)
        self._cb_queued = False
        self.launched_in_backward = False  # the bucket's all-reduce started from the end-of-backward callback
        self._timing = timing
        self.timing_every = 4   # regions recorded on every 4th step (each event pair idles the device ~4 us)
        self._tstats = {"exchange_wait_ms": 0.0, "sh_rebuild_ms": 0.0, "calls": 0, "timed_calls": 0}
        self._prev_ex = None
        self._hdr = None        # the record header's cached 4-float source
        self._recs = []         # per view slot of a step: [record, header key] (reused step to step)
        self._gouts = []        # per view slot: the all-gather's output (reused step to step)
        self._sh_out = None     # (dc, rest, event): the SH rebuild queued beside the backward
        self._gather_done = None  # event after this step's in-stream record gathers
        self._nccl = None       # the group's backend is RCCL (collectives in stream order, below)
        self._installed = False
        self._sh_on = sh is not None and (sh_force or self._active())
        self._bind()
        if self._sh_on or (overlap and self._active()):
            from diff_gaussian_rasterization import set_grad_exchange
            self._prev_ex = set_grad_exchange(self)
            self._installed = True

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
        self._index = {id(p): i for i, p in enumerate(self._reduced)}  # (strong refs: ids are unique)
        self._bucket = self._views = None
        self._bucket_cache = None
        self._mode, self._late_local, self._flag_read, self._flag_send = "probe", False, None, None
        # hooks only while there is something to exchange: with one rank the leaves
        # carry none, and the rasterizer's fused leaf gradients apply as without us
        if self.overlap and self._active():
            for p in self._reduced:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_accumulate))
        self._hook_ids = {h.id for h in self._hooks}

    def _stale(self) -> bool:
        if not callable(self._params_src) and not callable(self._sh_src):
            return False  # fixed tensors: bound once (the host path runs this several times a step)
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

    @property
    def pending(self) -> int:
        """Collectives in flight for this step (the bucket's all-reduce)."""
        return int(self._work is not None)

    def _active(self) -> bool:
        return dist.is_initialized() and (dist.get_world_size(self.group) > 1 or self._comm_force)

    # ---- the bucket
    def _ensure_bucket(self):
        if self._bucket is None and self._bucket_cache is not None:
            # last step's bucket again when the caller let go of its views (.grad set
            # to None, or still the view itself: zero_grad(set_to_none=False)) — as
            # DDP's gradient_as_bucket_view; its allocation and views cost the step's
            # critical host path ~15 us
            b, vs = self._bucket_cache
            if all(p.grad is None or self._is_view(p.grad, v) for p, v in zip(self._reduced, vs)):
                self._bucket, self._views = b, vs
        if self._bucket is None:
            ref = self._reduced[0]
            # + one spare float: the ranks' late-gradient flags, summed with the gradients
            n = sum(p.numel() for p in self._reduced)
            self._bucket = torch.empty(n + 1, dtype=torch.float32, device=ref.device)
            parts = self._bucket[:n].split([p.numel() for p in self._reduced])
            self._views = [v.view(p.shape) for v, p in zip(parts, self._reduced)]
            self._slot_fresh = True
        return self._bucket

    # ---- the late-gradient flag (class docstring)
    FLAG_EVERY = 16  # in "early" mode the summed flag is read back every FLAG_EVERY steps

    def _set_flag_slot(self, bucket: torch.Tensor) -> None:
        """This rank's flag into the bucket's spare float before its all-reduce: only
        when it is not 0 already (a fresh bucket, or a raised flag)."""
        flag = 1.0 if (self._late_local and self._mode != "late") else 0.0
        if self._slot_fresh or flag:
            bucket[-1:].fill_(flag)
            self._slot_fresh = False

    def _send_flag(self, bucket: torch.Tensor) -> None:
        """The bucket's all-reduce is queued: its summed flag is copied to the host in
        __call__, after the wait (probe steps, and every FLAG_EVERY-th step in "early"
        mode)."""
        if self._mode == "late" or self._flag_read is not None:
            return
        if self._mode == "early" and self._tstats["calls"] % self.FLAG_EVERY:
            return
        self._flag_send = self._mode

    def _copy_flag(self) -> None:
        mode, self._flag_send = self._flag_send, None
        if mode is None or self._bucket is None:
            return
        b = self._bucket
        if b.is_cuda:  # behind the collective on the compute stream (__call__ waited for it)
            host = torch.empty(1, dtype=torch.float32, pin_memory=True)
            host.copy_(b[-1:], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(b.device))
        else:
            host, ev = b[-1:].clone(), None
        self._flag_read = (host, ev, mode)

    def _check_flag(self) -> None:
        """The summed flag of an earlier step's bucket (every rank reads the same value
        at the same step): decides the probe, or raises on a late gradient.  By the
        next step's backward the device is past that all-reduce (the forward's
        num_rendered read-back waited for a later kernel), so the wait costs nothing."""
        if self._flag_read is None:
            return
        host, ev, mode = self._flag_read
        self._flag_read = None
        if ev is not None:
            ev.synchronize()
        n = float(host.item())
        if mode == "probe":
            self._mode = "early" if n == 0 else "late"
        elif n:
            raise RuntimeError(
                f"GradAllReduce: a gradient reached a reduced parameter after the bucket's all-reduce had started "
                f"({int(n)} rank(s), within the last {self.FLAG_EVERY} steps): the loss graph changed after the "
                f"first step (another term on a parameter the rasterizer writes), and that gradient was left out on "
                f"every rank.  Re-create the exchange (its first step detects such paths) or call reset_graph() "
                f"after changing the loss.")

    def reset_graph(self) -> None:
        """Probe the loss graph again at the next step (call it on every rank after
        changing the loss terms): the next step starts its all-reduce at the end of the
        backward and re-decides whether early starts are safe."""
        self._mode, self._late_local, self._flag_read, self._flag_send = "probe", False, None, None

    @staticmethod
    def _is_view(g, v) -> bool:
        return g is not None and g.data_ptr() == v.data_ptr() and g.shape == v.shape and g.dtype == v.dtype

    def _pack(self) -> torch.Tensor:
        """Every reduced parameter's .grad into its bucket view (zeros where a
        parameter got none), the views installed as .grad."""
        self._ensure_bucket()
        for p, v in zip(self._reduced, self._views):
            g = p.grad
            if self._is_view(g, v):
                continue
            if g is None:
                v.zero_()
            else:
                v.copy_(g)
            p.grad = v
        return self._bucket

    # ---- what the rasterizer asks (diff_gaussian_rasterization.set_grad_exchange)
    def owns_hooks(self, leaf) -> bool:
        """True when the leaf's post-accumulate hooks are this exchange's (the fused
        path may then write its gradient: the hook still fires and the bucket is
        packed at the end of the backward)."""
        hooks = getattr(leaf, "_post_accumulate_grad_hooks", None) or {}
        return bool(self._hooks) and set(hooks) <= self._hook_ids

    def leaf_bucket(self, leaves: dict) -> dict:
        """Bucket views for the rasterizer's fused leaf gradients: {name: views} for
        each name whose leaves are all reduced here and have no gradient yet or
        already hold their bucket view (a later backward of the step accumulates)."""
        if not (self.overlap and self._active()) or not self._reduced or self._stale():
            return {}
        if self._rast_seen:  # a second rasterizer after the first one's early-start point
            self._late_local = True
        if self._work is not None or self._early:
            # the bucket's all-reduce has started: a later writer gets no view
            # — its gradients reach the leaves through autograd (a late gradient)
            return {}
        self._check_flag()
        self._ensure_bucket()
        self._queue_callback()
        out = {}
        for name, ls in leaves.items():
            idx = [self._index.get(id(leaf), -1) for leaf in ls]
            if all(i >= 0 and (ls[j].grad is None or self._is_view(ls[j].grad, self._views[i]))
                   for j, i in enumerate(idx)):
                out[name] = tuple(self._views[i] for i in idx)
        return out

    def rasterizer_done(self, views: dict) -> bool:
        """Called by the rasterizer's backward right after its kernels are queued, with
        the bucket views it wrote (``leaf_bucket``'s answer), before it installs them
        as the leaves' ``.grad``.  On the step's last backward, when those views cover
        every reduced parameter, the bucket is complete already: its all-reduce
        starts here, the SH rebuild is queued behind the backward's last kernel, and
        True tells the rasterizer to leave the leaves' ``.grad`` unset (below).  Done
        from the end-of-backward callback instead, the host's round trip through the
        autograd engine left the device idle for ~65 us per step
        (``tools/exchange_profile.py`` traces)."""
        self._rast_seen = self._backwards + 1 == self.views_per_step  # (the early start's point)
        if self._views is not None:  # the views as the rasterizer left them (late-gradient test)
            self._view_ver = {i: v._version for i, v in enumerate(self._views)}
        if self._work is not None or self._bucket is None or self._backwards + 1 != self.views_per_step:
            return False
        if self._mode != "early":  # the probe step (or a graph with late paths): start at the end
            return False
        covered = {id(v) for vs in views.values() for v in vs if v is not None}
        if any(id(v) not in covered for v in self._views):
            return False
        # The all-reduce is launched first, on the compute stream as it stands (RCCL's
        # stream waits for the backward's kernels queued so far, not for what
        # follows), then the SH rebuild.  The device is still a render or more behind
        # the host here, so the launch order costs it nothing; what the exchange path
        # costs is host time (each event / stream switch ~5-10 us on the step's
        # critical host path, which the device waited for: exchange_profile traces).
        self._set_flag_slot(self._bucket)
        self._work = self._reduce(self._bucket)
        self._send_flag(self._bucket)
        self._sh_rebuild()
        self.launched_in_backward = True
        # The bucket now belongs to the collective.  Another gradient path into a
        # reduced leaf (an extra loss term, a regulariser on _scaling ...) reaches
        # its AccumulateGrad after this backward — and would add in place into the
        # .grad it finds, i.e. into the bucket RCCL is reading, never to be reduced
        # (ADVICE r4).  So the leaves hold no .grad until __call__: such a
        # contribution lands in a fresh tensor (flagged by the accumulate hook, left
        # out on every rank alike: class docstring), and __call__ installs the views.
        self._early = True
        for p in self._reduced:
            if p.grad is not None:  # a view installed by an earlier backward of the step
                p.grad = None
        return True

    def _in_stream(self, t: torch.Tensor) -> bool:
        """RCCL on device tensors: collectives are issued as non-async ops, which
        torch (>= 2.7) runs on the caller's current stream — no event recorded on
        the compute stream for RCCL's own stream to wait on, and no wait back (each
        such cross-queue step idled the compute stream 5-7 us, two hops ~21 us:
        exchange_profile traces); the host is not blocked (tools/pg_stream_probe.py).
        gloo keeps async work objects."""
        if not t.is_cuda:
            return False
        if self._nccl is None:
            self._nccl = dist.get_backend(self.group) == "nccl"
        return self._nccl

    def _pg(self):
        g = getattr(self, "_pg_obj", None)
        if g is None:
            g = self._pg_obj = self.group or dist.distributed_c10d._get_default_group()
        return g

    def _gather_now(self, out: torch.Tensor, rec: torch.Tensor) -> None:
        """all_gather_into_tensor as a non-async op on the current stream, straight
        through the process group (torch's Python wrapper costs ~15 us of host time
        per call, on the step's critical host path in this exchange)."""
        try:
            opts = dist.distributed_c10d.AllgatherOptions()
            opts.asyncOp = False
            work = self._pg()._allgather_base(out, rec, opts)
        except (AttributeError, TypeError):  # another torch: the public call
            dist.all_gather_into_tensor(out, rec, group=self.group)
            return
        if work is not None:
            work.wait()

    def _all_reduce_now(self, t: torch.Tensor) -> None:
        try:
            opts = dist.distributed_c10d.AllreduceOptions()
            opts.reduceOp = dist.ReduceOp.SUM
            opts.asyncOp = False
            work = self._pg().allreduce([t], opts)
        except (AttributeError, TypeError):
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            return
        if work is not None:
            work.wait()

    def _reduce(self, bucket: torch.Tensor):
        """The bucket's all-reduce, started now (behind everything queued on the
        compute stream).  In stream order it runs on the compute stream itself,
        after the records' gather on the exchange stream has completed (one
        collective of a communicator at a time)."""
        if self._in_stream(bucket):
            if self._gather_done is not None:
                torch.cuda.current_stream(bucket.device).wait_event(self._gather_done)
            self._all_reduce_now(bucket)
            return _QUEUED
        return dist.all_reduce(bucket, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    # ---- the end of each backward: start the bucket's all-reduce on the step's last
    def _queue_callback(self):
        if not self._cb_queued:
            try:
                torch.autograd.Variable._execution_engine.queue_callback(self._on_backward_end)
                self._cb_queued = True
            except RuntimeError:  # not inside a backward: __call__ packs and reduces
                pass

    def _on_accumulate(self, p: torch.Tensor) -> None:
        if self._active():
            if (self._rast_seen or self._early) and p.grad is not None:
                # after the rasterizer's backward: a gradient arrived through autograd if
                # .grad is not its bucket view as the rasterizer left it (the hook also
                # runs when no gradient came: then .grad is that view, unchanged)
                i = self._index.get(id(p))
                v = self._views[i] if (self._views is not None and i is not None) else None
                if v is None or not self._is_view(p.grad, v) or p.grad._version != self._view_ver.get(i):
                    self._late_local = True
            self._queue_callback()

    def _on_backward_end(self) -> None:
        self._cb_queued = False
        self._rast_seen = False
        self._backwards += 1
        if self._backwards > self.views_per_step:
            raise RuntimeError(f"GradAllReduce: {self._backwards} backwards in one step (views_per_step="
                               f"{self.views_per_step}); the bucket's all-reduce already started")
        if self._early and self._backwards == self.views_per_step:
            # late gradients after the early start are left out on this rank (flagged:
            # every rank raises at the next read of the flags); no collective of its own
            for p in self._reduced:
                p.grad = None
            return
        if self._backwards == self.views_per_step and self._work is None and not self._stale():
            bucket = self._pack()
            # the bucket's all-reduce behind the pack; the SH rebuild (it needs only the
            # gathered records) queued here too, behind the backward's last kernel,
            # instead of after the host has returned from backward() into the caller's
            # __call__ (a host round trip the device spent idle: 60-90 us per step)
            self._set_flag_slot(bucket)
            self._work = self._reduce(bucket)
            self._send_flag(bucket)
            self._sh_rebuild()
            self.launched_in_backward = True

    # ---- the rasterizer's SH sink
    def accepts(self, sh, means3D: torch.Tensor) -> bool:
        """True when this backward's SH input is the bound model's (and the SH
        exchange is on): the cat [P,M,3], or the (f_dc, f_rest) leaves themselves
        (diff_gaussian_rasterization.rasterize_model).  With more than one rank a mismatch raises: a silent local
        dsh would leave this rank's SH gradient out of the exchange and the replicas
        would drift apart."""
        if not self._sh_on:
            return False
        if self._stale():  # the model's tensors were replaced (densify / prune): follow them
            self._bind()
        xyz, f_dc, f_rest = self._sh
        if isinstance(sh, tuple):  # rasterize_model: GaussianModel's two SH leaves themselves
            ok = means3D.data_ptr() == xyz.data_ptr() and sh[0] is f_dc and sh[1] is f_rest
        else:
            ok = (means3D.data_ptr() == xyz.data_ptr() and sh.size(0) == xyz.size(0)
                  and sh.size(1) == f_dc.size(1) + f_rest.size(1))
        if not ok and self._active():
            raise RuntimeError("GradAllReduce: the rasterizer's SH input is not the bound model's "
                               f"(means3D {tuple(means3D.shape)} vs xyz {tuple(xyz.shape)}); pass params/sh as "
                               "callables that return the current tensors")
        return ok

    def _header(self, slot: list, campos: torch.Tensor, sh_degree: int) -> None:
        """The record's header [campos, degree], written when it differs from what the
        slot's record holds: one copy from a cached 4-float tensor (the view's camera
        is usually the same tensor step after step, and then nothing is queued)."""
        key = (campos, campos._version, int(sh_degree))
        if slot[1] is not None and slot[1][0] is campos and slot[1][1:] == key[1:]:
            return
        h = self._hdr
        if h is None or h[0] is not campos or h[1:3] != key[1:]:
            h = self._hdr = key + (torch.cat([campos.reshape(-1)[:3].float(),
                                              torch.full((1,), float(sh_degree), device=slot[0].device)]),)
        slot[0][0:4].copy_(h[3])
        slot[1] = key

    def _slot(self, P: int) -> list:
        # the record of this step's next view; a slot's record is reused the next step
        # (stream order makes that safe: its gather and its rebuild are done before
        # the next step's backward writes it, and the compute stream waited for both)
        from diff_gaussian_rasterization import _C
        i, n, dev = self._pushes, _C.sh_record_floats(P), self._sh[0].device
        while len(self._recs) <= i:
            self._recs.append(None)
        slot = self._recs[i]
        if slot is None or slot[0].numel() != n or slot[0].device != dev:
            if dev.type == "cuda" and self._active() and dist.get_backend(self.group) == "nccl":
                # RCCL: the record is this rank's slice of the all-gather's output, so
                # the gather runs in place (no local copy; at one rank no kernel at all)
                world, rank = dist.get_world_size(self.group), dist.get_rank(self.group)
                while len(self._gouts) <= i:
                    self._gouts.append(None)
                out = self._gouts[i] = torch.empty(world * n, dtype=torch.float32, device=dev)
                slot = self._recs[i] = [out.narrow(0, rank * n, n), None]
            else:
                slot = self._recs[i] = [torch.empty(n, dtype=torch.float32, device=dev), None]
        return slot

    def record(self, P: int, campos: torch.Tensor = None, sh_degree: int = None) -> torch.Tensor:
        """A view's record; with the camera given its header is written now (when it
        changed), on the compute stream ahead of the backward's kernels."""
        slot = self._slot(P)
        if campos is not None:
            self._header(slot, campos, sh_degree)
        else:
            slot[1] = None
        return slot[0]

    def _side(self, device) -> "torch.cuda.Stream":
        if not self.exchange_stream:  # everything in line on the compute stream
            return torch.cuda.current_stream(device)
        st = getattr(self, "_side_stream", None)
        if st is None or st.device != device:
            st = self._side_stream = torch.cuda.Stream(device=device)
        return st

    def _launch(self, ready, fn):
        """fn() (a collective, async) ordered after `ready` (an event on the compute
        stream: started from a stream of its own that waits for it), or with None
        after everything queued so far."""
        if ready is None:
            return fn()
        st = self._side(ready.device if hasattr(ready, "device") and ready.device is not None
                        else torch.cuda.current_device())
        with torch.cuda.stream(st):
            st.wait_event(ready)
            return fn()

    # the rasterizer hands over the colour kernel itself (push's `write`): with RCCL
    # it runs on the exchange stream, beside the per-Gaussian backward
    colours_apart = True
    # the SH rebuild on the exchange stream right behind the gather (beside
    # preprocess_bwd), or (False) on the compute stream after preprocess_bwd
    rebuild_on_side = True
    # the colour kernel, the record gather and the SH rebuild on a stream of their
    # own beside the per-Gaussian backward (True), or in line on the compute stream
    # (False: no second hardware queue, no cross-queue waits)
    exchange_stream = os.environ.get("GSR_EXCHANGE_STREAM", "1") != "0"

    def push(self, rec: torch.Tensor, campos: torch.Tensor, sh_degree: int, ready=None, write=None) -> None:
        """Exchange a view's record (from ``record``): the all-gather starts behind
        everything queued on the compute stream so far (the rasterizer calls this
        right after the kernels that write the colour gradient), or behind `ready`,
        an event after which it is written.  `write` (``colours_apart``): a function
        that queues the colour gradient's kernel on the current stream — called here
        first, on the exchange stream when the collectives run in stream order (the
        render backward is what the compute stream holds so far), else in line."""
        i = self._pushes
        if i >= self.views_per_step:
            # the step's SH rebuild is already queued over views_per_step records (ADVICE
            # r5): another record would start a second rebuild that overwrites the first
            raise RuntimeError(f"GradAllReduce: SH record {i + 1} in one step with views_per_step="
                               f"{self.views_per_step} (a second rasterizer call in one backward?); construct "
                               f"the exchange with views_per_step equal to the rasterizer calls per step")
        self._pushes += 1
        slot = self._recs[i] if i < len(self._recs) else None
        if slot is None or slot[0] is not rec:  # a record not made by record(): header now, gather behind it
            if slot is not None:
                slot[1] = None  # the gather may overwrite the slot's record (in place: a slice of its output)
            slot = [rec, None]
            ready = None
        if slot[1] is None:
            self._header(slot, campos, sh_degree)
        if self._active():
            world = dist.get_world_size(self.group)
            while len(self._gouts) <= i:
                self._gouts.append(None)
            out = self._gouts[i]
            if out is None or out.numel() != world * rec.numel() or out.device != rec.device:
                out = self._gouts[i] = torch.empty(world * rec.numel(), dtype=rec.dtype, device=rec.device)
            if self._in_stream(rec):
                # in stream order on the exchange stream, behind the colour gradient
                # (or `ready`); the SH rebuild follows it there, and the bucket's
                # all-reduce waits for this event
                side = self._side(rec.device)
                if ready is None:
                    side.wait_stream(torch.cuda.current_stream(rec.device))
                else:
                    side.wait_event(ready)
                last = self._pushes == self.views_per_step and self.rebuild_on_side
                if last:  # the rebuild's outputs from the compute stream's pool (see _rebuild_beside)
                    _, f_dc, f_rest = self._sh
                    dc, rest = torch.empty_like(f_dc), torch.empty_like(f_rest)
                with torch.cuda.stream(side):
                    if write is not None:
                        write()
                    self._gather_now(out, rec)
                    self._gather_done = torch.cuda.Event()
                    self._gather_done.record(side)
                    self._gathers.append((out, world, None))
                    if last:
                        self._rebuild_on_side(side, dc, rest)
                return
            else:
                if write is not None:
                    write()
                    ready = None
                work = self._launch(ready, lambda: dist.all_gather_into_tensor(out, rec, group=self.group,
                                                                               async_op=True))
            self._gathers.append((out, world, work))
            if self._pushes == self.views_per_step and rec.is_cuda:
                self._rebuild_beside()
        else:
            if write is not None:
                write()
            self._gathers.append((rec, 1, None))

    def _rebuild_on_side(self, side, dc: torch.Tensor, rest: torch.Tensor) -> None:
        """The SH rebuild on the exchange stream (current), right behind the gathers:
        _rebuild_beside's work inside push's stream block."""
        self._begin("sh_rebuild")
        self._rebuild_into(dc, rest)
        self._end("sh_rebuild")
        done = torch.cuda.Event()
        done.record(side)
        dc.record_stream(side)
        rest.record_stream(side)
        self._sh_out = (dc, rest, done)

    def _rebuild_beside(self) -> None:
        """The step's last record is out: the SH rebuild goes on the exchange's own
        stream right behind the gathers, beside the compute stream's per-Gaussian
        backward (both HBM-bound, but the rebuild no longer waits for preprocess_bwd
        and the compute stream no longer waits for the gathers).  ``__call__`` makes
        the compute stream wait for it and installs the gradients.  The outputs come
        from the compute stream's pool: their block was last used by compute-stream
        work ordered before this step's colour gradient, which the gathers (and so
        the rebuild) follow; record_stream keeps a later reuse behind the rebuild."""
        xyz, f_dc, f_rest = self._sh
        dc, rest = torch.empty_like(f_dc), torch.empty_like(f_rest)
        side = self._side(xyz.device)
        with torch.cuda.stream(side):
            for _, _, w in self._gathers:
                if w is not None:
                    w.wait()
            self._begin("sh_rebuild")
            self._rebuild_into(dc, rest)
            self._end("sh_rebuild")
            done = torch.cuda.Event()
            done.record(side)
        dc.record_stream(side)
        rest.record_stream(side)
        self._sh_out = (dc, rest, done)

    def _sh_rebuild(self) -> None:
        """The compute stream waits for the records' all-gather, then rebuilds the SH
        leaf gradients (no-op when there is nothing gathered)."""
        if self._sh is None or not self._gathers:
            return
        self._begin("exchange_wait")
        for _, _, w in self._gathers:
            if w is not None:
                w.wait()
        self._end("exchange_wait")
        self._begin("sh_rebuild")
        self._finish_sh()
        self._end("sh_rebuild")

    def _rebuild_into(self, dc: torch.Tensor, rest: torch.Tensor) -> None:
        # gathered buffers hold [rank 0 .. world-1] per push; with several views per
        # rank the sum runs push by push (identical order on every rank)
        xyz = self._sh[0]
        recs = torch.cat([o for o, _, _ in self._gathers]) if len(self._gathers) > 1 else self._gathers[0][0]
        nviews = sum(n for _, n, _ in self._gathers)
        self._gathers = []
        if self._rebuild is not None:
            self._rebuild(xyz.detach(), recs, nviews, dc, rest)
        else:
            from diff_gaussian_rasterization import _C
            _C.sh_grad_from_colors(xyz.detach(), recs, nviews, dc, rest if rest.numel() else None)

    def _install_sh(self, dc: torch.Tensor, rest: torch.Tensor) -> None:
        for p, g in ((self._sh[1], dc), (self._sh[2], rest)):
            if p.grad is None:
                p.grad = g
            else:
                p.grad.add_(g)

    def _finish_sh(self) -> None:
        if not self._gathers:
            return
        for _, _, w in self._gathers:
            if w is not None:
                w.wait()
        if self._gather_done is not None:  # gathered in stream order on the exchange stream
            torch.cuda.current_stream(self._sh[0].device).wait_event(self._gather_done)
        dc, rest = torch.empty_like(self._sh[1]), torch.empty_like(self._sh[2])
        self._rebuild_into(dc, rest)
        self._install_sh(dc, rest)

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self._hook_ids = set()
        if self._installed:
            from diff_gaussian_rasterization import set_grad_exchange
            set_grad_exchange(self._prev_ex)
            self._installed = False
            self._sh = None
            self._sh_on = False

    # ---- timing (bench.py's N > 1 line): on a GPU the regions are the library's
    # fence-free stage events (stages "exchange_wait" / "sh_rebuild", recorded while
    # _C.timing_enable has them on, read with _C.timing_read); on the CPU host clocks
    def _timed_now(self) -> bool:
        return self._timing and self._tstats["calls"] % self.timing_every == 0

    def _begin(self, name):
        if not self._timed_now():
            return
        if self._reduced and self._reduced[0].is_cuda:
            from diff_gaussian_rasterization import _C
            _C.timing_begin(name, self._reduced[0].device)
        else:
            self._t0 = time.perf_counter()

    def _end(self, name):
        if not self._timed_now():
            return
        if self._reduced and self._reduced[0].is_cuda:
            from diff_gaussian_rasterization import _C
            _C.timing_end(name, self._reduced[0].device)
        else:
            self._tstats[name + "_ms"] += 1e3 * (time.perf_counter() - self._t0)

    def stats(self) -> dict:
        """Per-step means since the last reset of the host-clock regions (CPU
        tensors; on a GPU the regions are library stages, read by the caller with
        _C.timing_read and divided by timed_calls), the calls, the steps whose regions
        were recorded (every timing_every-th), and the bytes this rank sends per step."""
        n = max(self._tstats["timed_calls"], 1)
        return {"exchange_wait_ms": self._tstats["exchange_wait_ms"] / n,
                "sh_rebuild_ms": self._tstats["sh_rebuild_ms"] / n, "calls": self._tstats["calls"],
                "timed_calls": self._tstats["timed_calls"],
                "bytes_per_rank": self.nbytes}

    def reset_stats(self) -> None:
        self._tstats = {"exchange_wait_ms": 0.0, "sh_rebuild_ms": 0.0, "calls": 0, "timed_calls": 0}

    def __call__(self):
        """Finish this step's exchange: the bucket's all-reduce (started at the end
        of the backward, or packed and reduced here when it was not: flat mode, a
        parameter swap, fewer backwards than announced), then the SH gradients from
        the gathered colour gradients (SH exchange on).  Returns the bucket."""
        self._check_flag()  # an earlier step's flags (the device is past them)
        if self._stale() and not self._early:
            # the model's tensors were replaced since the hooks were bound (densify /
            # prune): their gradients go through the bucket here, and the hooks move
            # to them for the next step
            self._work = None
            self._bind()
        if self._work is None:
            bucket = self._pack()
            if self._active():
                self._work = self._reduce(bucket)
        bucket = self._bucket
        # the SH rebuild needs only the gathered records: it runs while the bucket's
        # all-reduce is still in flight (queued at the end of the backward already,
        # unless nothing started there), and the compute stream waits for the bucket last
        self._sh_rebuild()
        self._begin("exchange_wait")
        sh_out, self._sh_out = self._sh_out, None
        if sh_out is not None:
            torch.cuda.current_stream(sh_out[0].device).wait_event(sh_out[2])
        if self._work is not None:
            self._work.wait()
        self._end("exchange_wait")
        self._copy_flag()
        if sh_out is not None:
            self._install_sh(sh_out[0], sh_out[1])
        if self._early:  # the views become the leaves' .grad again
            for p, v in zip(self._reduced, self._views):
                p.grad = v
        self._tstats["timed_calls"] += int(self._timed_now())
        self._tstats["calls"] += 1
        self._early = False
        self._gather_done = None
        self._work = None
        self._pushes = 0
        self._rast_seen = False
        if self._mode == "probe":
            self._late_local = False  # the probe's own flag was sent with its bucket
        # the grads keep the storage; the next step reuses it only if they were let go
        self._bucket_cache = (self._bucket, self._views) if self._views is not None else None
        self._bucket = self._views = None
        self._backwards = 0
        self.launched_in_backward = False
        return bucket


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
