"""Cellpose fine-tuning loop (single GPU or data-parallel over RCCL).

Mirrors the reference training core ``train_seg_with_callbacks``
(``apps/cellpose-finetuning/main.py:1278-1713``): AdamW (``:1451-1453``), the reference's LR
schedule (10-epoch linear warm-up, halving tail for n_epochs > 99 / > 300, ``:1430-1445``),
per-epoch LR (``:1479-1480``), random rotate/resize augmentation to ``bsize`` crops
(``:1501-1503``), ``_loss_fn_seg`` (``:1514-1517``), validation at epoch 0 and every
``validation_interval`` epochs with pixel TP/FP/FN/TN on the cell-probability channel
(``:1554-1675``, ``:1225-1270``), batch/epoch callbacks and a cooperative stop check.

MI355X specifics: augmentation is a batched HIP affine-warp kernel on device-resident training
images; the loss is a fused fwd+bwd HIP kernel; all parameters live in one flat fp32 buffer updated
by ONE fused AdamW launch; in DP mode gradient buckets are all-reduced over RCCL while backward is
still running (:mod:`bioengine_worker_amd.parallel.ddp`).  Optimizer moments, step, LR-schedule
position and RNG state are checkpointed, so resume is exact (the reference resumes weights only,
SURVEY.md §5 "Checkpoint / resume").
"""
from __future__ import annotations

import math
import time
from dataclasses import asdict, dataclass, field

import numpy as np
import torch
import torch.distributed as dist

from ..models.cpnet import CPnet
from ..ops import train_ops
from ..parallel.ddp import BucketedAllReduce, FlatParams, ShardedAdamW, broadcast_params


@dataclass
class TrainConfig:
    batch_size: int = 1
    bsize: int = 256
    lr: float = 5e-5
    weight_decay: float = 0.1
    n_epochs: int = 100
    scale_range: float = 0.5
    validation_interval: int = 10
    min_train_masks: int = 5
    # "auto": BatchNorm (cellpose cyto3) on one GPU, GroupNorm for data-parallel runs -- per-image
    # statistics make the DP step independent of how the global batch is split across ranks
    norm: str = "auto"
    autocast_bf16: bool = True
    bucket_mb: float = 16.0
    comm_bf16: bool = False
    seed: int = 0
    # "hip": hand-written fwd/bwd engine (train/cpnet_engine.py); "autograd": PyTorch autograd + MIOpen;
    # "auto": hip on GPU for BatchNorm nets, autograd otherwise
    engine: str = "auto"
    # capture the engine's forward+backward (~250 launches) in one HIP graph (single GPU; the
    # augment's host-side random affine and the AdamW step with its per-step scalars stay outside)
    graph: bool = True
    # data-parallel with the HIP engine: True = replay the captured fwd+bwd graph, then all-reduce
    # every bucket (launch-free backward, no comm overlap); False = eager backward with each bucket's
    # all-reduce issued the moment its gradients are written (overlap).  Measured on MI355X
    # (tools/train_ddp_mode_ab.py): eager 5.86 vs graph 5.98 ms at 8 crops, 13.39 vs 13.44 ms at
    # 32 — the engine's launches already hide behind its kernels, so overlap wins.
    ddp_graph: bool = False
    # CPSAM single-GPU graph: run each parameter group's AdamW inside the captured step on a side
    # stream the moment its gradients are final (per-step lr / bias corrections read from a device
    # buffer; same math as the flat update).  Measured slower on MI355X (profiles/r02/attn/README.md:
    # batch 8 39.7 -> 41.4-41.8 ms, batch 1 15.3 -> 16.9-17.6 ms: the optimizer's HBM stream slows
    # the backward kernels more than it hides), so the flat update after the replay stays the default.
    # Re-measured in round 4 with the streaming kernel (profiles/r04/cpsam/overlap_adamw_ab.jsonl):
    # batch 1 11.34 -> 12.02 ms, batch 8 33.11 -> 33.90 ms; capping its grid only makes it later.
    cpsam_overlap_adamw: bool = False
    # data-parallel CPSAM: AdamW per gradient bucket, each right after its own all-reduce
    cpsam_bucket_adamw: bool = True
    # run the data-parallel step path (segmented graph + bucket all-reduces) even at world 1 over a
    # 1-rank process group: the on-one-GPU measurement of the DP code path's own overhead
    force_dp_path: bool = False
    # data-parallel CPSAM step: capture fwd+bwd as a chain of HIP graphs cut where gradient buckets
    # complete; each bucket's all-reduce is issued right after its segment replays, so RCCL traffic
    # overlaps the remaining backward while the step stays launch-free
    cpsam_dp_graph: bool = True
    # data-parallel optimizer: False = bucketed all-reduce + AdamW over all parameters on every rank;
    # True = ZeRO-1 (parallel/ddp.py ShardedAdamW): bucketed reduce-scatter, AdamW on the rank's
    # 1/world chunk of every bucket, all-gather of the updated parameters
    zero_adamw: bool = False


def lr_schedule(learning_rate: float, n_epochs: int) -> np.ndarray:
    """Exact replica of the reference schedule (main.py:1430-1445)."""
    s = np.linspace(0, learning_rate, 10)
    s = np.append(s, learning_rate * np.ones(max(0, n_epochs - 10)))
    if n_epochs > 300:
        s = s[:-100]
        for _ in range(10):
            s = np.append(s, s[-1] / 2 * np.ones(10))
    elif n_epochs > 99:
        s = s[:-50]
        for _ in range(10):
            s = np.append(s, s[-1] / 2 * np.ones(5))
    return s


class CellposeTrainer:
    def __init__(self, net: CPnet, cfg: TrainConfig, device, world_size: int = 1, rank: int = 0, group=None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.world = world_size
        self.rank = rank
        from ..models.cpsam import CPSAM

        self.is_cpsam = isinstance(net, CPSAM)
        self.net = net.to(self.device).train()
        if self.device.type == "cuda" and not self.is_cpsam:
            self.net = self.net.to(memory_format=torch.channels_last)
        zero = cfg.zero_adamw and (world_size > 1 or cfg.force_dp_path)
        self.fp = FlatParams(self.net, self.device, bucket_mb=cfg.bucket_mb if zero else None,
                             bucket_multiple=4 * world_size)
        if world_size > 1:
            broadcast_params(self.fp, 0, group)
        self.m = torch.zeros_like(self.fp.flat)
        self.v = torch.zeros_like(self.fp.flat)
        comm = torch.bfloat16 if cfg.comm_bf16 else None
        if zero:
            self.ar = ShardedAdamW(self.fp, self.m, self.v, group=group, comm_dtype=comm, force=cfg.force_dp_path)
        else:
            self.ar = BucketedAllReduce(self.fp, group=group, bucket_mb=cfg.bucket_mb, comm_dtype=comm,
                                        force=cfg.force_dp_path)
        self.step_count = 0
        self.epoch = 0  # completed epochs (exact resume point)
        self.lr = cfg.lr
        self.gen = torch.Generator().manual_seed(cfg.seed * 1000 + rank)
        eng = cfg.engine
        if self.is_cpsam:
            eng = "cpsam"  # explicit fwd/bwd engine (train/cpsam_engine.py) on CPU and GPU
        elif eng == "auto":
            eng = "hip" if (self.device.type == "cuda" and cfg.norm in ("batch", "group")) else "autograd"
        self.engine_kind = eng
        self._eng = None
        self._cpsam_engs: dict = {}
        self._cpsam_graph = None
        self._cpsam_graph_failed = False
        self._graph = None
        self._graph_io = None

    # ------------------------------------------------------------------ core step
    def set_lr(self, lr: float):
        self.lr = float(lr)

    def augment(self, imgs, lbls, rescale=None):
        """Random rotate / flip / resize to ``bsize`` crops (cellpose ``random_rotate_and_resize``).
        ``imgs`` / ``lbls`` may be lists of differently sized images: each is warped on its own
        (no cropping to a common size) and the crops are batched."""
        if isinstance(imgs, (list, tuple)):
            outs = [self.augment(i[None], l[None], None if rescale is None else [rescale[k]])
                    for k, (i, l) in enumerate(zip(imgs, lbls))]
            return torch.cat([o[0] for o in outs]), torch.cat([o[1] for o in outs])
        B, C, H, W = imgs.shape
        aff, flip, _ = train_ops.random_affine_params(B, H, W, xy=(self.cfg.bsize, self.cfg.bsize),
                                                      scale_range=self.cfg.scale_range, rescale=rescale,
                                                      generator=self.gen)
        return train_ops.affine_warp(imgs, lbls, aff, flip, self.cfg.bsize, self.cfg.bsize)

    def forward_loss(self, x: torch.Tensor, lbl: torch.Tensor) -> torch.Tensor:
        if self.device.type == "cuda":
            x = x.contiguous(memory_format=torch.channels_last)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.cfg.autocast_bf16):
                y = self.net(x)[0]
        else:
            y = self.net(x)[0]
        return train_ops.seg_loss(y, lbl)

    def step(self, imgs: torch.Tensor, lbls: torch.Tensor, rescale=None) -> torch.Tensor:
        """One optimisation step on a batch of (full-size) training images + [cellprob, flowY, flowX] labels."""
        from ..profiling import trace

        with trace.span("train.augment", cuda=True):
            x, lbl = self.augment(imgs, lbls, rescale)
        if self.engine_kind == "cpsam":
            return self._step_cpsam(x, lbl)
        if self.engine_kind == "hip":
            return self._step_engine(x, lbl)
        self.fp.zero_grad()
        with trace.span("train.forward_loss", cuda=True):
            loss = self.forward_loss(x, lbl)
        with trace.span("train.backward", cuda=True):
            loss.backward()
        if self._sharded_update():
            return loss.detach()
        with trace.span("train.grad_allreduce_finish", cuda=True):
            gscale = self.ar.finish()
        self.step_count += 1
        with trace.span("train.adamw", cuda=True):
            train_ops.adamw_flat_(self.fp.flat, self.fp.grad, self.m, self.v, lr=self.lr, step=self.step_count,
                                  weight_decay=self.cfg.weight_decay, grad_scale=gscale)
        return loss.detach()

    def _engine(self, B: int, S: int):
        from .cpnet_engine import CPnetTrainEngine

        if self._eng is None or (self._eng.B, self._eng.S) != (B, S):
            self._eng = CPnetTrainEngine(self.net, self.fp, B, S, self.device)
        return self._eng

    def _step_engine(self, x: torch.Tensor, lbl: torch.Tensor) -> torch.Tensor:
        from ..profiling import trace

        eng = self._engine(x.shape[0], x.shape[-1])
        with trace.span("train.fwd_bwd_engine", cuda=True):
            if self.cfg.graph and self.device.type == "cuda" and (not self.ar.active or self.cfg.ddp_graph):
                loss = self._graph_step(eng, x, lbl)  # ar.finish() then all-reduces every bucket
            else:
                loss = eng.loss_and_backward(x, lbl, on_params_ready=self.ar.mark_ready if self.ar.active else None)
        if self._sharded_update():
            return loss
        with trace.span("train.grad_allreduce_finish", cuda=True):
            gscale = self.ar.finish()
        self.step_count += 1
        with trace.span("train.adamw", cuda=True):
            train_ops.adamw_flat_(self.fp.flat, self.fp.grad, self.m, self.v, lr=self.lr, step=self.step_count,
                                  weight_decay=self.cfg.weight_decay, grad_scale=gscale)
        return loss

    def _cpsam_engine(self, B: int):
        from .cpsam_engine import CPSAMTrainEngine

        eng = self._cpsam_engs.get(B)
        if eng is None:
            # all engines of this trainer share one bf16 weight mirror (refreshed by the AdamW kernel)
            first = next(iter(self._cpsam_engs.values()), None)
            eng = CPSAMTrainEngine(self.net, self.fp, B, self.device)
            if first is not None:
                eng.mirror = first.mirror
            self._cpsam_engs[B] = eng
        return eng

    def _step_cpsam(self, x: torch.Tensor, lbl: torch.Tensor) -> torch.Tensor:
        from ..profiling import trace
        from .cpsam_engine import stochastic_depth_keep

        eng = self._cpsam_engine(x.shape[0])
        keep = None
        if self.net.rdrop > 0:
            keep = stochastic_depth_keep(x.shape[0], len(eng.blocks), self.net.rdrop, self.device, self.gen)
        with trace.span("train.fwd_bwd_cpsam", cuda=True):
            fused_opt = False
            graphable = self.cfg.graph and self.device.type == "cuda" and not self._cpsam_graph_failed
            if graphable and not self.ar.active:
                loss = self._cpsam_graph_step(eng, x, lbl, keep)
                fused_opt = getattr(self, "_adamw_in_graph", False)
            elif graphable and self.cfg.cpsam_dp_graph:
                loss = self._cpsam_dp_graph_step(eng, x, lbl, keep)
            else:
                loss = eng.loss_and_backward(x, lbl, keep,
                                             on_params_ready=self.ar.mark_ready if self.ar.active else None)
        if self._sharded_update(eng.mirror if eng.mirror is not self.fp.flat else None):
            return loss
        if self.ar.active and not fused_opt and self.cfg.cpsam_bucket_adamw:
            # per-bucket AdamW, each on its own bucket's all-reduce completion: the update of the
            # buckets the backward finished first overlaps the last buckets' collectives
            self.step_count += 1
            mirror = eng.mirror if eng.mirror is not self.fp.flat else None
            with trace.span("train.grad_allreduce_adamw", cuda=True):
                self.ar.finish_each(lambda s, e, sc: self._adamw_range(s, e, sc, mirror))
            return loss
        with trace.span("train.grad_allreduce_finish", cuda=True):
            gscale = self.ar.finish()
        self.step_count += 1
        if fused_opt:
            return loss  # the update already ran inside the replayed graph
        with trace.span("train.adamw", cuda=True):
            mirror = eng.mirror if eng.mirror is not self.fp.flat else None
            train_ops.adamw_flat_(self.fp.flat, self.fp.grad, self.m, self.v, lr=self.lr, step=self.step_count,
                                  weight_decay=self.cfg.weight_decay, grad_scale=gscale, p_bf16=mirror)
        return loss

    def _sharded_update(self, mirror=None) -> bool:
        """ZeRO-1 optimizer step (ShardedAdamW): True when it ran (the caller's AdamW is skipped)."""
        if not (isinstance(self.ar, ShardedAdamW) and self.ar.active):
            return False
        from ..profiling import trace

        self.step_count += 1
        with trace.span("train.reduce_scatter_adamw_allgather", cuda=True):
            self.ar.step(lr=self.lr, step=self.step_count, weight_decay=self.cfg.weight_decay, mirror=mirror)
        return True

    def _adamw_range(self, s: int, e: int, grad_scale: float, mirror) -> None:
        """AdamW over flat elements [s, e) (bucket boundaries are 4-element aligned)."""
        # the streaming kernel reads flat/grad/m/v[s:] as float4 and the bf16 mirror as 4 x bf16:
        # a sub-range must start on a 4-element boundary (16 B fp32 / 8 B bf16)
        if s % 4:
            raise ValueError(f"AdamW sub-range start {s} is not 4-element aligned")
        sl = slice(s, e)
        train_ops.adamw_flat_(self.fp.flat[sl], self.fp.grad[sl], self.m[sl], self.v[sl], lr=self.lr,
                              step=self.step_count, weight_decay=self.cfg.weight_decay, grad_scale=grad_scale,
                              p_bf16=mirror[sl] if mirror is not None else None)

    def _adamw_group_cb(self, eng, side):
        """on_params_ready callback used during capture: AdamW over the group's flat range on ``side``."""
        from ..ops import _native

        fp = self.fp
        off = {id(p): o for p, o in zip(fp.params, fp.offsets)}
        mirror = eng.mirror if eng.mirror is not fp.flat else None
        cur = torch.cuda.current_stream(self.device)

        def cb(params):
            lo = min(off[id(p)] for p in params)
            hi = max(off[id(p)] + (p.numel() + 3) // 4 * 4 for p in params)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                _native.call("be_adamw_flat_dev", _native.ptr(fp.flat[lo:]), _native.ptr(fp.grad[lo:]),
                             _native.ptr(self.m[lo:]), _native.ptr(self.v[lo:]),
                             _native.ptr(mirror[lo:] if mirror is not None else None), hi - lo,
                             _native.ptr(self._hp), 0.9, 0.999, 1e-8, _native.stream(self.device))
        return cb

    def _set_hp(self, step: int) -> None:
        b1, b2 = 0.9, 0.999
        vals = [self.lr, float(self.cfg.weight_decay), 1.0 - b1 ** step, 1.0 - b2 ** step, 1.0]
        self._hp.copy_(torch.tensor(vals, dtype=torch.float32))  # pageable source: staged before return

    def _cpsam_graph_step(self, eng, x, lbl, keep):
        """Replay the captured CPSAM fwd+bwd (~1.3k launches at ViT-L) on static buffers; the
        stochastic-depth mask is drawn on the host and copied in, AdamW runs outside the graph."""
        key = (tuple(x.shape), tuple(lbl.shape))
        if self._cpsam_graph is None or self._cpsam_graph[0] != key:
            xs, ls = x.clone(), lbl.clone()
            ks = (keep.clone() if keep is not None else
                  torch.ones(x.shape[0], len(eng.blocks), device=self.device))
            try:
                side = torch.cuda.Stream(self.device)
                side.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(side):
                    for _ in range(2):
                        eng.loss_and_backward(xs, ls, ks)
                torch.cuda.current_stream(self.device).wait_stream(side)
                fuse = bool(self.cfg.cpsam_overlap_adamw)
                if fuse and not hasattr(self, "_hp"):
                    self._hp = torch.zeros(5, device=self.device, dtype=torch.float32)
                g = torch.cuda.CUDAGraph()
                opt_side = torch.cuda.Stream(self.device)
                with torch.cuda.graph(g):
                    cur = torch.cuda.current_stream(self.device)
                    cb = self._adamw_group_cb(eng, opt_side) if fuse else None
                    out = eng.loss_and_backward(xs, ls, ks, on_params_ready=cb)
                    if fuse:
                        cur.wait_stream(opt_side)  # join the optimizer branch before the graph ends
                self._adamw_in_graph = fuse
            except Exception as e:  # noqa: BLE001  (e.g. a library call that cannot be captured)
                import logging

                logging.getLogger("bioengine.train").warning("CPSAM graph capture failed (%s); running eagerly", e)
                self._cpsam_graph_failed = True
                self._adamw_in_graph = False
                torch.cuda.synchronize(self.device)
                return eng.loss_and_backward(x, lbl, keep)
            self._cpsam_graph = (key, g, xs, ls, ks, out)
        _, g, xs, ls, ks, out = self._cpsam_graph
        if getattr(self, "_adamw_in_graph", False):
            self._set_hp(self.step_count + 1)
        xs.copy_(x)
        ls.copy_(lbl)
        if keep is not None:
            ks.copy_(keep)
        else:
            ks.fill_(1.0)
        g.replay()
        return out.clone()

    def _cpsam_dp_graph_step(self, eng, x, lbl, keep):
        """Data-parallel CPSAM step: fwd+bwd captured as a CHAIN of graphs cut at every point where
        a gradient bucket becomes complete (simulated with the bucket arrival counts during
        capture).  Replay: segment k, then the all-reduces of the buckets it completed (async, RCCL
        stream), then segment k+1 -- communication overlaps the rest of the backward exactly as in
        the eager hook path, but with no per-kernel launch cost.  Segments share one memory pool and
        are replayed in capture order."""
        key = (tuple(x.shape), tuple(lbl.shape))
        if getattr(self, "_cpsam_dp", None) is None or self._cpsam_dp[0] != key:
            xs, ls = x.clone(), lbl.clone()
            ks = (keep.clone() if keep is not None else
                  torch.ones(x.shape[0], len(eng.blocks), device=self.device))
            try:
                side = torch.cuda.Stream(self.device)
                side.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(side):
                    for _ in range(2):
                        eng.loss_and_backward(xs, ls, ks)
                torch.cuda.current_stream(self.device).wait_stream(side)
                torch.cuda.synchronize(self.device)
                pending = [len(m) for (_, _, m) in self.ar.buckets]
                segs: list = []
                state = {"g": torch.cuda.CUDAGraph(), "pool": None}
                cap = torch.cuda.Stream(self.device)
                cap.wait_stream(torch.cuda.current_stream(self.device))

                def cut(params):
                    done = []
                    for p in params:
                        bi = self.ar.bucket_of(p)
                        pending[bi] -= 1
                        if pending[bi] == 0:
                            done.append(bi)
                    if done and not any(pending):
                        # the last bucket: its all-reduce follows the FINAL segment (which ends with
                        # whatever the backward still does after this point) -- no empty segment
                        state["last"] = done
                        return
                    if done:
                        state["g"].capture_end()
                        segs.append((state["g"], done))
                        if state["pool"] is None:
                            state["pool"] = state["g"].pool()
                        state["g"] = torch.cuda.CUDAGraph()
                        state["g"].capture_begin(pool=state["pool"])

                with torch.cuda.stream(cap):
                    state["g"].capture_begin()
                    out = eng.loss_and_backward(xs, ls, ks, on_params_ready=cut)
                    state["g"].capture_end()
                segs.append((state["g"], state.get("last", []) + [bi for bi, n in enumerate(pending) if n > 0]))
                torch.cuda.current_stream(self.device).wait_stream(cap)
            except Exception as e:  # noqa: BLE001
                import logging

                logging.getLogger("bioengine.train").warning("CPSAM DP graph capture failed (%s); running eagerly", e)
                self._cpsam_graph_failed = True
                torch.cuda.synchronize(self.device)
                self.ar.reset()
                return eng.loss_and_backward(x, lbl, keep, on_params_ready=self.ar.mark_ready)
            self._cpsam_dp = (key, segs, xs, ls, ks, out)
        _, segs, xs, ls, ks, out = self._cpsam_dp
        xs.copy_(x)
        ls.copy_(lbl)
        if keep is not None:
            ks.copy_(keep)
        else:
            ks.fill_(1.0)
        for g, done in segs:
            g.replay()
            for bi in done:
                self.ar.launch_bucket(bi)
        return out.clone()

    def _refresh_mirrors(self) -> None:
        for eng in self._cpsam_engs.values():
            eng.refresh_mirror()
            break  # shared

    def _graph_step(self, eng, x: torch.Tensor, lbl: torch.Tensor) -> torch.Tensor:
        """Replay the captured fwd+bwd on static input buffers (captured on first use per shape)."""
        key = (tuple(x.shape), tuple(lbl.shape), x.dtype)
        if self._graph is None or self._graph_io[0] != key:
            xs, ls = x.clone(), lbl.clone()
            side = torch.cuda.Stream(self.device)
            side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(side):  # warm-up on a side stream (allocator + lazy state), as torch requires
                for _ in range(2):
                    eng.loss_and_backward(xs, ls)
            torch.cuda.current_stream(self.device).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                out = eng.loss_and_backward(xs, ls)
            self._graph, self._graph_io = g, (key, xs, ls, out)
        _, xs, ls, out = self._graph_io
        xs.copy_(x)
        ls.copy_(lbl)
        self._graph.replay()
        return out.clone()

    @torch.no_grad()
    def validate(self, imgs: torch.Tensor, lbls: torch.Tensor) -> dict:
        self.net.eval()
        x, lbl = self.augment(imgs, lbls)
        if self.is_cpsam:
            y = self._cpsam_engine(x.shape[0]).forward(x, None, save=False)
        elif self.device.type == "cuda":
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.cfg.autocast_bf16):
                y = self.net(x.contiguous(memory_format=torch.channels_last))[0]
        else:
            y = self.net(x)[0]
        loss = train_ops.seg_loss_ref(y.float(), lbl)
        pred = y[:, 2].float() > 0
        tgt = lbl[:, 0] > 0.5
        tp = (pred & tgt).sum().item()
        fp = (pred & ~tgt).sum().item()
        fn = (~pred & tgt).sum().item()
        tn = (~pred & ~tgt).sum().item()
        self.net.train()
        prec = tp / max(1, tp + fp)
        rec = tp / max(1, tp + fn)
        return {"loss": float(loss), "tp": tp, "fp": fp, "fn": fn, "tn": tn, "precision": prec, "recall": rec,
                "f1": 2 * prec * rec / max(1e-12, prec + rec), "iou": tp / max(1, tp + fp + fn)}

    def agree(self, loss, n_local: int, stop_local: bool = False) -> tuple[float, bool]:
        """One tiny all-reduce per step: the GLOBAL mean loss (sample-weighted over ranks) and a
        collective stop decision, so every rank leaves the loop after the same step (a rank that
        left alone would strand the others in the next gradient all-reduce until the PG timeout).
        Single process: (float(loss), stop_local)."""
        if self.world == 1:
            return float(loss), bool(stop_local)
        dev = self.fp.flat.device
        t = torch.stack([loss.detach().float().reshape(()) * float(n_local),
                         torch.tensor(float(n_local), device=loss.device),
                         torch.tensor(1.0 if stop_local else 0.0, device=loss.device)]).to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.ar.group)
        vals = t.tolist()
        return vals[0] / max(vals[1], 1e-12), vals[2] > 0

    def rebind(self, world_size: int, rank: int, group=None) -> None:
        """Adopt a new data-parallel world (elastic shrink, ``parallel/elastic.py``): rebuild the
        bucketed all-reduce for the new group and make every rank's weights, AdamW moments and BN
        buffers identical to the new rank 0's."""
        self.ar.remove()
        self.world, self.rank = int(world_size), int(rank)
        self.fp.zero_grad()
        # a shrunk world keeps the plain all-reduce path: the padded ZeRO bucket layout was cut for
        # the old world size (moment chunks a lost rank owned since the last checkpoint are stale)
        self.ar = BucketedAllReduce(self.fp, group=group, bucket_mb=self.cfg.bucket_mb,
                                    comm_dtype=torch.bfloat16 if self.cfg.comm_bf16 else None)
        self._graph = self._graph_io = None
        self._cpsam_graph = None
        self._cpsam_dp = None
        self._adamw_in_graph = False
        if self.world > 1:
            broadcast_params(self.fp, 0, group)
            for t in [self.m, self.v] + [b for b in self.net.buffers() if b.is_floating_point()]:
                dist.broadcast(t, src=0, group=group)
            st = torch.tensor([self.step_count], dtype=torch.int64, device=self.fp.flat.device)
            dist.broadcast(st, src=0, group=group)
            self.step_count = int(st.item())
        self._refresh_mirrors()

    # ------------------------------------------------------------------ checkpoint
    def state_dict(self) -> dict:
        if isinstance(self.ar, ShardedAdamW):
            self.ar.sync_moments()  # each rank updated only its own chunks
        return {"flat": self.fp.flat.detach().cpu(), "m": self.m.cpu(), "v": self.v.cpu(), "step": self.step_count,
                "epoch": self.epoch, "lr": self.lr, "rng": self.gen.get_state(), "cfg": asdict(self.cfg),
                "buffers": {k: v.cpu() for k, v in self.net.named_buffers()}}

    def load_state_dict(self, sd: dict) -> None:
        self.fp.flat.copy_(sd["flat"].to(self.device))
        self.m.copy_(sd["m"].to(self.device))
        self.v.copy_(sd["v"].to(self.device))
        self.step_count = int(sd["step"])
        self.epoch = int(sd.get("epoch", 0))
        self.lr = float(sd["lr"])
        self.gen.set_state(sd["rng"])
        bufs = dict(self.net.named_buffers())
        for k, v in sd.get("buffers", {}).items():
            if k in bufs:
                bufs[k].copy_(v.to(bufs[k].device))
        self._refresh_mirrors()


def resolve_norm(norm: str, world_size: int) -> str:
    return ("group" if world_size > 1 else "batch") if norm == "auto" else norm


def build_trainer(cfg: TrainConfig, device, world_size: int = 1, rank: int = 0, net: CPnet | None = None,
                  group=None) -> CellposeTrainer:
    cfg.norm = getattr(net, "norm_kind", None) or resolve_norm(cfg.norm, world_size)
    net = net or CPnet(norm=cfg.norm).randomize_(cfg.seed)
    return CellposeTrainer(net, cfg, device, world_size, rank, group)


# ------------------------------------------------------------------ data

def synthetic_instances(B: int, H: int, W: int, ncells: int | None = None, seed: int = 0):
    """Synthetic instance data: images [B, 2, H, W] float32 and label maps [B, H, W] int32 (disks)."""
    rng = np.random.default_rng(seed)
    ncells = ncells or max(4, H * W // 2500)
    imgs = np.zeros((B, 2, H, W), np.float32)
    labels = np.zeros((B, H, W), np.int32)
    yy, xx = np.mgrid[0:H, 0:W]
    for b in range(B):
        k = 0
        for _ in range(ncells * 4):
            if k >= ncells:
                break
            r = rng.uniform(5, 12)
            cy, cx = rng.uniform(r, H - r), rng.uniform(r, W - r)
            d2 = (yy - cy) ** 2 + (xx - cx) ** 2
            m = d2 <= r * r
            if labels[b][m].any():
                continue
            k += 1
            labels[b][m] = k
            imgs[b, 0] += np.exp(-d2 / (2 * r * r)) * m
            imgs[b, 1] += np.exp(-d2 / (2 * (0.4 * r) ** 2))
    imgs += 0.05 * rng.standard_normal(imgs.shape).astype(np.float32)
    return imgs, labels


def labels_to_flows(labels: torch.Tensor) -> torch.Tensor:
    """Label maps [B, H, W] -> training targets [B, 3, H, W] = (labels, flowY, flowX)."""
    if labels.is_cuda:
        from ..cellpose.gpu import masks_to_flows_gpu

        mu, _, _ = masks_to_flows_gpu(labels.int().contiguous())
    else:
        from ..cellpose import reference as ref

        mu = torch.stack([torch.from_numpy(ref.masks_to_flows(l.numpy())) for l in labels])
    return torch.cat([labels.float()[:, None], mu], 1)


def synthetic_train_batch(B: int, bsize: int = 256, device="cuda", seed: int = 0):
    """Device-resident (imgs [B, 2, S, S], lbl [B, 3, S, S]) with S = bsize + 64 source images."""
    S = bsize + 64
    imgs, labels = synthetic_instances(B, S, S, seed=seed)
    dev = torch.device(device)
    imgs_t = torch.from_numpy(imgs).to(dev)
    lbl = labels_to_flows(torch.from_numpy(labels).to(dev))
    return imgs_t, lbl


def _take(x, idx):
    if torch.is_tensor(x):
        return x[torch.as_tensor(idx, device=x.device)]
    return [x[int(i)] for i in idx]


def run_training(trainer: CellposeTrainer, train_imgs, train_lbls, n_epochs: int, test_imgs=None, test_lbls=None,
                 batch_callback=None, epoch_callback=None, stop_check=None, start_epoch: int = 0,
                 diams=None, rescale: bool = False) -> dict:
    """Epoch loop with the reference's schedule, callbacks and validation cadence.

    ``train_imgs`` / ``train_lbls``: stacked tensors or lists of per-image tensors (any sizes).
    ``rescale``: scale each crop by its image's cell diameter / the net's ``diam_mean`` (``diams``
    per image; reference ``rsc = diams / net.diam_mean`` at main.py:1494-1499).
    In DP mode each rank takes a disjoint shard of every epoch's permutation (global batch =
    batch_size * world)."""
    cfg = trainer.cfg
    sched = lr_schedule(cfg.lr, n_epochs)
    nimg = len(train_imgs)
    dmean = float(trainer.net.diam_mean.item()) if hasattr(trainer.net, "diam_mean") else 30.0
    losses = np.zeros(n_epochs)
    test_losses: list = [None] * n_epochs
    t0 = time.time()
    gb = cfg.batch_size * trainer.world
    for ep in range(start_epoch, n_epochs):
        rng = np.random.default_rng(ep)
        perm = rng.permutation(nimg)
        trainer.set_lr(float(sched[min(ep, len(sched) - 1)]))
        nb = math.ceil(nimg / gb)
        for k in range(nb):
            sl = perm[k * gb: (k + 1) * gb]
            mine = sl[trainer.rank::trainer.world] if trainer.world > 1 else sl
            rsc = None
            if rescale and diams is not None:
                rsc = [max(float(diams[int(i)]), 1e-3) / dmean for i in mine]
            n_mine = len(mine)
            if len(mine) == 0:  # fewer samples than ranks in the last batch: weight-0 filler
                mine = sl[:1]
            loss = trainer.step(_take(train_imgs, mine), _take(train_lbls, mine), rsc)
            # stop marker read by rank 0 only, decided collectively with the global loss
            stop_local = bool(stop_check()) if (stop_check is not None and trainer.rank == 0) else False
            lv, stop = trainer.agree(loss, n_mine, stop_local)
            losses[ep] += lv * len(sl)
            if batch_callback is not None:
                batch_callback(ep + 1, k, nb, lv, time.time() - t0, None)
            if stop:
                return {"train_losses": losses[: ep + 1].tolist(), "test_losses": test_losses[: ep + 1], "stopped": True,
                        "epoch": ep}
        losses[ep] /= nimg
        trainer.epoch = ep + 1
        metrics = None
        if test_imgs is not None and (ep == 0 or (ep + 1) % cfg.validation_interval == 0):
            metrics = trainer.validate(test_imgs, test_lbls)
            test_losses[ep] = metrics["loss"]
        if epoch_callback is not None:
            epoch_callback(ep + 1, losses[ep], test_losses[ep], time.time() - t0, metrics)
    return {"train_losses": losses.tolist(), "test_losses": test_losses, "stopped": False}
