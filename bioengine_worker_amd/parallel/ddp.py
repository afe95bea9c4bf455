"""Data-parallel training over RCCL: flat parameter/gradient buffers + bucketed, overlapped all-reduce.

The reference trains on one GPU only (``apps/cellpose-finetuning/main.py:3603`` num_gpus=1,
batch 1 at ``:1292``).  This module is the MI355X data-parallel path (BASELINE
config 3): one process per GPU, ``torch.distributed`` with the ``nccl`` backend (= RCCL on ROCm)
over xGMI.

Design
------
* **Flat buffers.**  Every trainable parameter becomes a view into ONE contiguous fp32 buffer, and
  every ``.grad`` a view into ONE contiguous fp32 gradient buffer.  The fused AdamW kernel then
  updates all parameters in a single launch, and gradient buckets are plain slices — no
  pack/unpack copies around the collectives.
* **Buckets in backward order.**  Parameters are laid out in *reverse* registration order (the
  order autograd produces their gradients), and the flat gradient buffer is cut into buckets of
  ``bucket_mb``.  A post-accumulate-grad hook counts arrivals; the moment a bucket is complete its
  ``all_reduce`` is issued asynchronously, so communication of late layers overlaps the backward of
  early layers.
* **Sized for xGMI.**  MI355X has 7 point-to-point xGMI links (~153 GB/s each); RCCL's ring/tree
  all-reduce is per-link bound, so per-collective latency (not NVSwitch bandwidth) decides the
  bucket size: a handful of multi-MB buckets (default 16 MB) amortise launch/latency while still
  overlapping.  CPnet (6.6 M params, 26 MB fp32 grads) becomes ~2 buckets.
* **Mean folded into the optimizer.**  Buckets are summed (``ReduceOp.SUM``); the 1/world factor is
  passed to the AdamW kernel as ``grad_scale`` instead of a separate scaling pass.
* Optional bf16 gradient communication (``comm_dtype=torch.bfloat16``) halves bytes on the wire.

Works on gloo (CPU tests, world_size 2) and RCCL (GPU) unchanged.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def bucket_bounds(sizes: list[int], cap: int, multiple: int = 4) -> tuple[list[int], list[tuple[int, int, list[int]]]]:
    """Parameter offsets and gradient buckets (start, end, member indices) for parameters of the
    given element counts in gradient-arrival order.  Every parameter segment is padded to 4 elements
    (16 B, so vector kernels never straddle parameters); a bucket closes at the first parameter
    boundary past ``cap`` elements and its end is padded up to ``multiple`` elements (the sharded
    optimizer needs every bucket to split into world equal, 4-aligned chunks)."""
    offsets, buckets = [], []
    off, start, members = 0, 0, []
    for i, n in enumerate(sizes):
        offsets.append(off)
        off += (n + 3) // 4 * 4
        members.append(i)
        if off - start >= cap:
            off = (off + multiple - 1) // multiple * multiple
            buckets.append((start, off, members))
            start, members = off, []
    if members:
        off = (off + multiple - 1) // multiple * multiple
        buckets.append((start, off, members))
    return offsets, buckets


class FlatParams:
    """Re-home a module's trainable parameters into flat fp32 param / grad buffers.

    ``bucket_mb`` / ``bucket_multiple``: lay the buffers out for gradient buckets of that size whose
    ends are padded to a multiple of ``bucket_multiple`` elements (:class:`ShardedAdamW` passes
    4 x world); the layout is then recorded in :attr:`buckets` and every reducer uses it."""

    def __init__(self, module: torch.nn.Module, device: torch.device | str | None = None,
                 bucket_mb: float | None = None, bucket_multiple: int = 4):
        params = [p for p in module.parameters() if p.requires_grad]
        params = list(reversed(params))  # gradient-arrival order
        self.params = params
        device = torch.device(device) if device is not None else params[0].device
        n = sum(p.numel() for p in params)
        # without a bucket layout the buffer keeps the plain 4-element padding: its size must not
        # depend on the world size (checkpoints move between worlds, e.g. after an elastic shrink)
        cap = max(1, int(bucket_mb * 1024 * 1024 / 4)) if bucket_mb is not None else 1 << 62
        self.offsets, bks = bucket_bounds([p.numel() for p in params], cap,
                                          bucket_multiple if bucket_mb is not None else 4)
        self.buckets = bks if bucket_mb is not None else None
        off = bks[-1][1] if bks else 0
        self.numel = off
        self.flat = torch.zeros(off, dtype=torch.float32, device=device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=device)
        for p, o in zip(params, self.offsets):
            k = p.numel()
            self.flat[o: o + k].copy_(p.detach().reshape(-1).float())
            p.data = self.flat[o: o + k].view_as(p)
            p.grad = self.grad[o: o + k].view_as(p)
        self.nparams = n

    def zero_grad(self):
        self.grad.zero_()


class BucketedAllReduce:
    """Overlapped gradient all-reduce over slices of a FlatParams gradient buffer."""

    def __init__(self, fp: FlatParams, group=None, bucket_mb: float = 16.0, comm_dtype: torch.dtype | None = None,
                 force: bool = False):
        self.fp = fp
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # force: run the collectives even on a 1-rank group (measures the data-parallel code path,
        # its launches and graph segmentation, on one GPU)
        self.active = self.world > 1 or (force and dist.is_initialized())
        self.comm_dtype = comm_dtype
        cap = max(1, int(bucket_mb * 1024 * 1024 / 4))
        # bucket boundaries on parameter boundaries, in gradient-arrival order (the layout the
        # FlatParams was built for, if it was built for one)
        if getattr(fp, "buckets", None) is not None:
            self.buckets = [(s, e, list(m)) for (s, e, m) in fp.buckets]
        else:
            _, self.buckets = bucket_bounds([p.numel() for p in fp.params], cap)
            if self.buckets:
                s, _, m = self.buckets[-1]
                self.buckets[-1] = (s, fp.numel, m)
        self.param_bucket = {}
        for bi, (_, _, mem) in enumerate(self.buckets):
            for i in mem:
                self.param_bucket[i] = bi
        self.pending = [0] * len(self.buckets)
        self.works: list = []
        self._hooks = []
        self._index = {id(p): i for i, p in enumerate(fp.params)}
        if self.active:
            for i, p in enumerate(fp.params):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
        self.reset()

    def bucket_of(self, p) -> int:
        return self.param_bucket[self._index[id(p)]]

    def launch_bucket(self, bi: int) -> None:
        """Issue bucket ``bi``'s all-reduce now (segmented-graph replay knows the completion order)."""
        if self.active and self.pending[bi] > 0:
            self.pending[bi] = 0
            self._launch(bi)

    def reset(self):
        self.pending = [len(m) for (_, _, m) in self.buckets]
        self.works = []
        self._bufs = []
        self._order = []

    def mark_ready(self, params) -> None:
        """Explicit readiness for engines that write gradients without autograd
        (:class:`~bioengine_worker_amd.train.cpnet_engine.CPnetTrainEngine`): the moment the last
        parameter of a bucket is reported, that bucket's all-reduce is issued."""
        if not self.active:
            return
        for p in params:
            bi = self.param_bucket[self._index[id(p)]]
            self.pending[bi] -= 1
            if self.pending[bi] == 0:
                self._launch(bi)

    def _make_hook(self, i: int):
        def hook(_p):
            bi = self.param_bucket[i]
            self.pending[bi] -= 1
            if self.pending[bi] == 0:
                self._launch(bi)
        return hook

    def _launch(self, bi: int):
        s, e, _ = self.buckets[bi]
        view = self.fp.grad[s:e]
        if self.comm_dtype is not None and self.comm_dtype != torch.float32:
            buf = view.to(self.comm_dtype)
            w = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            self._bufs.append((view, buf))
        else:
            buf = None
            w = dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self.works.append(w)
        self._order.append((bi, w, view, buf))

    def finish_each(self, fn) -> None:
        """Like :meth:`finish`, but hands each bucket to ``fn(start, end, grad_scale)`` as soon as ITS
        all-reduce is done, in launch order (the order the backward completed them): the optimizer
        update of the early buckets runs while the last buckets are still on the wire, instead of
        one whole-model AdamW after the final all-reduce."""
        if not self.active:
            fn(0, self.fp.numel, 1.0)
            return
        for bi, n in enumerate(self.pending):
            if n > 0:
                self.pending[bi] = 0
                self._launch(bi)
        scale = 1.0 / self.world
        for bi, w, view, buf in self._order:
            w.wait()  # the current stream waits for this bucket's collective only
            if buf is not None:
                view.copy_(buf.float())
            s, e, _ = self.buckets[bi]
            fn(s, e, scale)
        self.reset()

    def finish(self) -> float:
        """Wait for every bucket (launching any that never filled, e.g. unused params).
        Returns the gradient scale (1/world) the optimizer must apply."""
        if not self.active:
            return 1.0
        for bi, n in enumerate(self.pending):
            if n > 0:
                self.pending[bi] = 0
                self._launch(bi)
        for w in self.works:
            w.wait()
        for view, buf in self._bufs:
            view.copy_(buf.float())
        self.reset()
        return 1.0 / self.world

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []


def broadcast_params(fp: FlatParams, src: int = 0, group=None) -> None:
    """Weights broadcast at replica start."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(fp.flat, src=src, group=group)


def init_distributed(backend: str | None = None) -> tuple[int, int, int]:
    """Initialise torch.distributed from torchrun env vars. Returns (world, rank, local_rank)."""
    import os

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


class ShardedAdamW:
    """ZeRO-1 data-parallel AdamW over a :class:`FlatParams` laid out for padded buckets.

    Per gradient bucket (same buckets, hooks and readiness interface as :class:`BucketedAllReduce`,
    so the segmented-graph step drives either): a ``reduce_scatter`` leaves rank r the summed
    gradient of chunk r of the bucket only; AdamW updates that chunk (1/world of the parameters, so
    the optimizer's HBM stream is cut by the world size); an ``all_gather`` then re-assembles the
    updated fp32 parameters of the bucket on every rank (and the bf16 compute mirror, when given, is
    refreshed from them).  Bytes on the wire equal one all-reduce (reduce-scatter + all-gather are
    its two halves); with ``comm_dtype=bfloat16`` the gradient half moves bf16.

    The moments live in full-size buffers, but a rank only updates its own chunks: call
    :meth:`sync_moments` before reading them (checkpoints).  Works on gloo (CPU tests) and RCCL.
    """

    def __init__(self, fp: FlatParams, m: torch.Tensor, v: torch.Tensor, group=None, comm_dtype=None,
                 force: bool = False):
        self.fp, self.m, self.v = fp, m, v
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.active = self.world > 1 or (force and dist.is_initialized())
        self.comm_dtype = comm_dtype
        if fp.buckets is None:
            raise ValueError("ShardedAdamW needs FlatParams(..., bucket_mb=..., bucket_multiple=4 * world)")
        self.buckets = [(s, e, list(mem)) for (s, e, mem) in fp.buckets]
        for s, e, _ in self.buckets:
            if (e - s) % (4 * self.world):
                raise ValueError(f"bucket [{s}, {e}) does not split into {self.world} 4-aligned chunks")
        self.param_bucket = {i: bi for bi, (_, _, mem) in enumerate(self.buckets) for i in mem}
        self._index = {id(p): i for i, p in enumerate(fp.params)}
        self._inplace = dist.is_initialized() and dist.get_backend(group) == "nccl"
        self._hooks = []
        if self.active:
            for i, p in enumerate(fp.params):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
        self.reset()

    # -- the BucketedAllReduce readiness interface
    def chunk(self, bi: int) -> tuple[int, int]:
        s, e, _ = self.buckets[bi]
        L = (e - s) // self.world
        return s + self.rank * L, s + (self.rank + 1) * L

    def bucket_of(self, p) -> int:
        return self.param_bucket[self._index[id(p)]]

    def reset(self):
        self.pending = [len(m) for (_, _, m) in self.buckets]
        self._order = []

    def launch_bucket(self, bi: int) -> None:
        if self.active and self.pending[bi] > 0:
            self.pending[bi] = 0
            self._launch(bi)

    def mark_ready(self, params) -> None:
        if not self.active:
            return
        for p in params:
            bi = self.param_bucket[self._index[id(p)]]
            self.pending[bi] -= 1
            if self.pending[bi] == 0:
                self._launch(bi)

    def _make_hook(self, i: int):
        def hook(_p):
            bi = self.param_bucket[i]
            self.pending[bi] -= 1
            if self.pending[bi] == 0:
                self._launch(bi)
        return hook

    def _launch(self, bi: int):
        s, e, _ = self.buckets[bi]
        cs, ce = self.chunk(bi)
        full, own = self.fp.grad[s:e], self.fp.grad[cs:ce]
        if self.comm_dtype is not None and self.comm_dtype != torch.float32:
            src = full.to(self.comm_dtype)
            out = torch.empty(ce - cs, dtype=self.comm_dtype, device=full.device)
        else:
            src = full if self._inplace else full.clone()
            out = own
        w = dist.reduce_scatter_tensor(out, src, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self._order.append((bi, w, out, src))

    def step(self, lr: float, step: int, weight_decay: float = 0.0, mirror: torch.Tensor | None = None,
             betas=(0.9, 0.999), eps: float = 1e-8) -> None:
        """Finish the gradient reduce-scatters (launching buckets that never filled), update the own
        chunk of every bucket as soon as ITS collective is done, and gather the parameters back."""
        from ..ops import train_ops

        for bi, n in enumerate(self.pending):
            if n > 0:
                self.pending[bi] = 0
                self._launch(bi)
        scale = 1.0 / self.world
        gathers = []
        for bi, w, out, _src in self._order:
            w.wait()
            s, e, _ = self.buckets[bi]
            cs, ce = self.chunk(bi)
            if out.data_ptr() != self.fp.grad[cs:ce].data_ptr():
                self.fp.grad[cs:ce].copy_(out.float())
            train_ops.adamw_flat_(self.fp.flat[cs:ce], self.fp.grad[cs:ce], self.m[cs:ce], self.v[cs:ce], lr=lr,
                                  step=step, betas=betas, eps=eps, weight_decay=weight_decay, grad_scale=scale)
            own = self.fp.flat[cs:ce]
            g = dist.all_gather_into_tensor(self.fp.flat[s:e], own if self._inplace else own.clone(),
                                            group=self.group, async_op=True)
            gathers.append((g, s, e))
        for g, s, e in gathers:
            g.wait()
            if mirror is not None and mirror.data_ptr() != self.fp.flat.data_ptr():
                mirror[s:e].copy_(self.fp.flat[s:e])
        self.reset()

    def sync_moments(self) -> None:
        """All-gather every bucket's moment chunks, so m / v are whole on every rank (checkpoint)."""
        if not self.active:
            return
        for bi, (s, e, _) in enumerate(self.buckets):
            cs, ce = self.chunk(bi)
            for t in (self.m, self.v):
                own = t[cs:ce]
                dist.all_gather_into_tensor(t[s:e], own if self._inplace else own.clone(), group=self.group)

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
