"""End-to-end Cellpose inference: normalise -> (rescale) -> tile -> CPnet -> blend -> masks.

``CellposeRunner.eval`` mirrors the call the reference apps make on ``cellpose.models.CellposeModel``
(``model.eval(images, diameter, flow_threshold, cellprob_threshold, niter, min_size, ...)``;
``apps/cellpose-finetuning/main.py:4965-5052`` and ``:3559-3567``) but runs a whole *batch* of images
through one set of kernel launches: the tiles of every image in the batch are one CPnet batch,
blending and mask recovery are batched kernels.  This is what the continuous-batching router feeds.

GPU path: HIP kernels (:mod:`.gpu`, :class:`~bioengine_worker_amd.models.cpnet.CPnetEngine`).
CPU path: the numpy/torch oracle (:mod:`.reference`) — used by CPU tests and CPU-only workers.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

from ..models.cpnet import CPnet, CPnetEngine
from ..ops.resize import resize_bilinear
from ..profiling import trace
from . import reference as ref


@dataclass
class EvalParams:
    diameter: float | None = None
    niter: int = 200
    flow_threshold: float = 0.4
    cellprob_threshold: float = 0.0
    min_size: int = 15
    max_size_fraction: float = 0.4
    normalize: bool = True
    tile: bool = True
    bsize: int | None = None  # None: the network's native tile (224 CPnet, 256 Cellpose-SAM)
    tile_overlap: float = 0.1
    compute_masks: bool = True
    #: GPU: split a batch into this many micro-batches and run mask recovery of micro-batch i on a
    #: second HIP stream while the network runs micro-batch i+1 (the mask stage is a chain of
    #: latency-bound kernels and host syncs that leaves most CUs idle on its own).
    pipeline_chunks: int = 1  # measured: 2 -> -9 %, 4 -> -18 % (latency-bound mask stages run once per chunk)
    pipeline_min_chunk: int = 4
    max_tiles: int = 0  # network tiles per launch (0 = sized to free HBM, CellposeRunner.tile_budget)


def as_batch(images, nchan: int, device=None) -> torch.Tensor:
    """Accept [H,W], [H,W,C], [C,H,W], [B,C,H,W] numpy/torch -> float tensor [B, nchan, H, W] on
    ``device`` (copied in the input's own dtype, e.g. uint16, and converted there)."""
    x = torch.as_tensor(np.asarray(images) if not torch.is_tensor(images) else images)
    if device is not None:
        x = x.to(device)
    if x.dim() == 2:
        x = x[None, None]
    elif x.dim() == 3:
        # channel-last if the last dim is small and the first is not
        if x.shape[-1] <= 4 and x.shape[0] > 4:
            x = x.permute(2, 0, 1)
        x = x[None]
    x = x.float()
    B, C, H, W = x.shape
    if C < nchan:
        x = torch.cat([x, torch.zeros(B, nchan - C, H, W, dtype=x.dtype, device=x.device)], 1)
    elif C > nchan:
        x = x[:, :nchan]
    return x


class CellposeRunner:
    """Batched Cellpose inference on one device: cyto3-style CPnet (224 tiles, fused MFMA conv engine)
    or Cellpose-SAM (cellpose 4 ``cpsam``: 256 tiles, 3 channels, ViT-L/8 HIP engine)."""

    def __init__(self, net=None, device: str | torch.device = "cuda", seed: int = 0):
        from ..models.cpsam import CPSAM, CPSAMEngine

        self.device = torch.device(device)
        self.net = (net if net is not None else CPnet().randomize_(seed)).eval()
        self.is_sam = isinstance(self.net, CPSAM)
        if self.is_sam:
            self.nchan = 3
            self.bsize = int(self.net.bsize)
            self.engine = CPSAMEngine(self.net, self.device) if self.device.type == "cuda" else None
        else:
            self.nchan = self.net.nchan
            self.bsize = 224
            if getattr(self.net, "norm_kind", "batch") == "group":
                self.engine = _GroupNormEngine(self.net, self.device)
            else:
                self.engine = CPnetEngine(self.net, self.device)
        self.diam_mean = float(self.net.diam_mean.item())
        self.cin_pad = (self.nchan + 7) // 8 * 8
        self._pinned: torch.Tensor | None = None  # host staging for numpy batches (pinned -> async DMA)
        self._plans: dict = {}
        self._net_graphs: dict = {}

    # ---------------------------------------------------------------- network
    def _plan(self, H, W, p: EvalParams):
        from .gpu import TilePlan

        bs = p.bsize or self.bsize
        key = (H, W, bs, p.tile_overlap)
        if key not in self._plans:
            self._plans[key] = TilePlan(H, W, bs, p.tile_overlap, device=self.device)
        return self._plans[key]

    #: HBM bytes one 224^2 CPnet tile keeps live at the forward's peak (measured on MI355X: 23.0-23.4
    #: MB per tile at 16 / 64 tiles, max_memory_allocated over one engine call; rounded up)
    TILE_ACT_BYTES = 32 << 20

    def tile_budget(self, p: EvalParams | None = None) -> int:
        """Tiles per network launch: what the free HBM holds (288 GB MI355X: ~8k tiles of 224^2, a
        ~20k x 20k image) with a quarter kept back; ``EvalParams.max_tiles`` caps it explicitly."""
        cap = getattr(p, "max_tiles", 0) if p is not None else 0
        if self.device.type != "cuda":
            return cap or (1 << 30)
        free, _ = torch.cuda.mem_get_info(self.device)
        n = max(1, int(free * 0.75) // self.TILE_ACT_BYTES)
        return min(n, cap) if cap else n

    def _tile_queue(self, tiles: torch.Tensor, p: EvalParams):
        """Spatial tile queue: the tiles of one batch (or one huge image) go through the network in
        launches of at most :meth:`tile_budget` tiles, written into one output buffer that the blend
        then reads -- an image larger than the HBM-resident activation budget is tiled, not an OOM
        (SURVEY.md §5 "tile queues sized to HBM"; the per-tile outputs are 0.6 MB each)."""
        T = tiles.shape[0]
        budget = self.tile_budget(p)
        if T <= budget:
            return self.engine(tiles)
        yt = st = None
        for i in range(0, T, budget):
            y_i, s_i = self.engine(tiles[i: i + budget])
            if yt is None:
                yt = torch.empty((T,) + tuple(y_i.shape[1:]), dtype=y_i.dtype, device=y_i.device)
                st = torch.empty((T,) + tuple(s_i.shape[1:]), dtype=s_i.dtype, device=s_i.device)
            yt[i: i + y_i.shape[0]] = y_i
            st[i: i + s_i.shape[0]] = s_i
            del y_i, s_i
        return yt, st

    def _sam_tiles(self, tiles: torch.Tensor) -> torch.Tensor:
        """NHWC bf16 tiles [T, by, bx, cpad] -> CPSAM flows [T, 3, by, bx] fp32 (tiles smaller than
        the network's fixed 256 grid are zero-padded, as cellpose 4 pads small images)."""
        T, by, bx, _ = tiles.shape
        bs = self.bsize
        x = torch.zeros(T, 3, bs, bs, dtype=torch.bfloat16, device=tiles.device)
        x[:, :, :by, :bx] = tiles[..., :3].permute(0, 3, 1, 2)
        out = []
        for i in range(0, T, 64):  # bounded activation memory for very large batches
            out.append(self.engine.graphed(x[i: i + 64]))
        y = torch.cat(out) if len(out) > 1 else out[0]
        return y[:, :, :by, :bx].contiguous()

    @torch.no_grad()
    def run_net(self, x: torch.Tensor, p: EvalParams) -> tuple[torch.Tensor, torch.Tensor]:
        """x: normalised [B, nchan, H, W] on device -> (y [B, 3, H, W] fp32, style [B, S])."""
        B, C, H, W = x.shape
        if self.device.type == "cuda":
            if p.tile:
                plan = self._plan(H, W, p)
                with trace.span("cellpose.tiles_gather", cuda=True, tiles=B * plan.nt):
                    tiles = plan.gather(x, self.cin_pad)
                with trace.span("cellpose.net", cuda=True, tiles=B * plan.nt):
                    if self.is_sam:
                        yt = self._sam_tiles(tiles)
                        st = torch.zeros(B * plan.nt, 256, device=x.device)
                    else:
                        yt, st = self._tile_queue(tiles, p)
                with trace.span("cellpose.blend", cuda=True):
                    y = plan.blend(yt, B)
                style = st.view(B, plan.nt, -1).sum(1)
            elif self.is_sam:
                raise ValueError("Cellpose-SAM inference needs tile=True (fixed 256x256 network grid)")
            else:
                Hp, Wp = math.ceil(H / 8) * 8, math.ceil(W / 8) * 8
                xin = torch.zeros(B, Hp, Wp, self.cin_pad, dtype=torch.bfloat16, device=x.device)
                xin[:, :H, :W, :C] = x.permute(0, 2, 3, 1)
                y, style = self.engine(xin)
                y = y[:, :, :H, :W].contiguous()
            style = style / torch.sqrt((style * style).sum(1, keepdim=True)).clamp_min(1e-12)
            return y, style
        # CPU oracle path
        ys, styles = [], []
        bs = p.bsize or self.bsize
        for b in range(B):
            img = x[b].numpy()
            if p.tile:
                ya, yb = ref.pad_amounts(H)
                xa, xb = ref.pad_amounts(W)
                imgp = np.pad(img, ((0, 0), (ya, yb), (xa, xb)))
                tiles, tys, txs = ref.make_tiles(imgp, bs, p.tile_overlap)
                tt = torch.from_numpy(tiles).float()
                if self.is_sam:
                    T, _, by, bx = tt.shape
                    tp = torch.zeros(T, 3, self.bsize, self.bsize)
                    tp[:, :, :by, :bx] = tt[:, :3]
                    yt = self.net(tp)[0][:, :, :by, :bx].detach()
                    st = torch.zeros(T, 256)
                else:
                    yt, st, _ = self.net(tt)
                yf = ref.average_tiles(yt.numpy(), tys, txs, imgp.shape[1], imgp.shape[2])
                ys.append(torch.from_numpy(yf[:, ya: ya + H, xa: xa + W].copy()))
                styles.append(st.sum(0))
            else:
                yt, st, _ = self.net(x[b: b + 1])
                ys.append(yt[0])
                styles.append(st[0])
        style = torch.stack(styles)
        return torch.stack(ys), style / torch.sqrt((style * style).sum(1, keepdim=True)).clamp_min(1e-12)

    # ---------------------------------------------------------------- full eval
    @torch.no_grad()
    def eval(self, images, p: EvalParams | None = None, **kw):
        """Returns (masks [B, H, W] int32 tensor, flows [B, 3, H, W] fp32 tensor, styles [B, S])."""
        p = p or EvalParams()
        for k, v in kw.items():
            setattr(p, k, v)
        x = as_batch(self._stage(images), self.nchan, self.device)
        B, C, H, W = x.shape
        nch = min(p.pipeline_chunks, B // max(1, p.pipeline_min_chunk))
        if self.device.type == "cuda" and p.compute_masks and nch >= 2:
            return self._eval_pipelined(x, p, nch)
        return self._eval_one(x, p)

    def _stage(self, images):
        """numpy batch -> view of a reusable pinned host buffer, so the H2D copy is one DMA at full
        PCIe rate instead of a pageable staged copy.  The previous eval has finished with the buffer
        (its results were synchronised back) by the time it is reused."""
        if self.device.type != "cuda" or torch.is_tensor(images) or not isinstance(images, np.ndarray):
            return images
        a = np.ascontiguousarray(images)
        if self._pinned is None or self._pinned.numel() < a.nbytes:
            self._pinned = torch.empty(max(a.nbytes, 1 << 20), dtype=torch.uint8, pin_memory=True)
        tdt = torch.from_numpy(np.empty(0, a.dtype)).dtype
        t = self._pinned[: a.nbytes].view(tdt).view(a.shape)  # still a pinned tensor
        np.copyto(t.numpy(), a)
        return t

    #: batches up to this many images run normalize99 + tiling + network + blend from a HIP graph
    #: (captured once per shape / params).  Off by default: measured on MI355X it did not help --
    #: headline 1,813 / 1,813 img/s graphed vs 1,819 / 1,815 eager, batch-1 p50 2.05 / 2.08 vs
    #: 1.99 / 2.03 ms (profiles/r05/headline/graph_ab_s5.jsonl): the eager launches already hide
    #: behind the kernels and the replay adds the static-buffer copies.
    GRAPH_NET_MAX_B = int(os.environ.get("BE_CELLPOSE_GRAPH_MAX_B", "0"))

    def _net_graphed(self, x, p: EvalParams):
        """(y, style) of the network stage (rescale 1) replayed from its HIP graph, or None when this
        call should run eagerly (large batch, CPU, capture failed for this shape)."""
        B = x.shape[0]
        if self.device.type != "cuda" or B > self.GRAPH_NET_MAX_B or not x.is_cuda:
            return None
        key = (tuple(x.shape), x.dtype, bool(p.normalize), bool(p.tile), p.bsize, p.tile_overlap, p.max_tiles)
        ent = self._net_graphs.get(key)
        if ent is False:
            return None
        if ent is None:
            xs = x.clone()
            side = torch.cuda.Stream(self.device)
            side.wait_stream(torch.cuda.current_stream(self.device))

            def body():
                xx = self._normalize(xs) if p.normalize else xs
                return self.run_net(xx, p)

            try:
                with torch.cuda.stream(side):
                    body()  # lazy state (plans, kernel attributes, workspaces) outside the capture
                torch.cuda.current_stream(self.device).wait_stream(side)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    y, style = body()
            except Exception:  # noqa: BLE001 -- this shape runs eagerly
                self._net_graphs[key] = False
                return None
            ent = self._net_graphs[key] = (g, xs, y, style)
        g, xs, y, style = ent
        xs.copy_(x)
        g.replay()
        return y.clone(), style.clone()

    def _eval_one(self, x, p: EvalParams):
        B, C, H, W = x.shape
        if not (p.diameter is not None and p.diameter > 0 and abs(self.diam_mean / float(p.diameter) - 1.0) > 1e-3):
            r = self._net_graphed(x, p)
            if r is not None:
                y, style = r
                if not p.compute_masks:
                    return None, y, style
                with trace.span("cellpose.masks", cuda=True, images=B):
                    masks = self.compute_masks(y, p, 1.0)
                return masks, y, style
        if p.normalize:
            with trace.span("cellpose.normalize99", cuda=True, images=B):
                x = self._normalize(x)
        rescale = 1.0
        if p.diameter is not None and p.diameter > 0:
            rescale = self.diam_mean / float(p.diameter)
        if abs(rescale - 1.0) > 1e-3:
            Hs, Ws = max(8, int(round(H * rescale))), max(8, int(round(W * rescale)))
            xs = resize_bilinear(x, (Hs, Ws))
            y, style = self.run_net(xs, p)
            y = resize_bilinear(y, (H, W))
        else:
            y, style = self.run_net(x, p)
        if not p.compute_masks:
            return None, y, style
        with trace.span("cellpose.masks", cuda=True, images=B):
            masks = self.compute_masks(y, p, rescale)
        return masks, y, style

    def _net_stage(self, x, p: EvalParams):
        B, C, H, W = x.shape
        if not (p.diameter is not None and p.diameter > 0 and abs(self.diam_mean / float(p.diameter) - 1.0) > 1e-3):
            r = self._net_graphed(x, p)
            if r is not None:
                return r[0], r[1], 1.0
        if p.normalize:
            with trace.span("cellpose.normalize99", cuda=True, images=B):
                x = self._normalize(x)
        rescale = 1.0
        if p.diameter is not None and p.diameter > 0:
            rescale = self.diam_mean / float(p.diameter)
        if abs(rescale - 1.0) > 1e-3:
            Hs, Ws = max(8, int(round(H * rescale))), max(8, int(round(W * rescale)))
            xs = resize_bilinear(x, (Hs, Ws))
            y, style = self.run_net(xs, p)
            y = resize_bilinear(y, (H, W))
        else:
            y, style = self.run_net(x, p)
        return y, style, rescale

    def _eval_pipelined(self, x, p: EvalParams, nch: int):
        """Two-stream software pipeline over micro-batches: net(i+1) on the current stream is queued
        before mask recovery of micro-batch i (which syncs the host on its own stream) starts."""
        main = torch.cuda.current_stream(self.device)
        if getattr(self, "_mask_stream", None) is None:
            self._mask_stream = mask_stream(self.device)
        side = self._mask_stream
        parts = x.tensor_split(nch)
        ys, styles, masks = [], [], []
        pending = None

        def finish(item):
            y, rescale, ev = item
            with torch.cuda.stream(side):
                side.wait_event(ev)
                y.record_stream(side)
                with trace.span("cellpose.masks", cuda=True, images=y.shape[0]):
                    m = self.compute_masks(y, p, rescale)
            masks.append(m)

        for part in parts:
            y, style, rescale = self._net_stage(part, p)
            ys.append(y)
            styles.append(style)
            ev = torch.cuda.Event()
            ev.record(main)
            if pending is not None:
                finish(pending)
            pending = (y, rescale, ev)
        finish(pending)
        main.wait_stream(side)
        for m in masks:
            m.record_stream(main)
        return torch.cat(masks), torch.cat(ys), torch.cat(styles)

    @torch.no_grad()
    def eval_locked(self, images, net_lock, mask_lock, p: EvalParams | None = None, **kw):
        """:meth:`eval` for concurrent callers (serving threads): the network stage runs under
        ``net_lock`` on the caller's stream, mask recovery under ``mask_lock`` on the runner's second
        stream -- so one batch's mask recovery overlaps the next batch's network (the cross-batch
        overlap of :meth:`stream`, for batches that arrive on different threads).  Returns
        ``(masks, flows, styles, ready)``: ``ready`` is a HIP event recorded after the masks (None
        off the GPU path) -- wait on it on a copy stream rather than on the caller's stream, which may
        already hold the next batch's network."""
        p = p or EvalParams()
        for k, v in kw.items():
            setattr(p, k, v)
        if self.device.type != "cuda" or not p.compute_masks:
            with net_lock:
                m, y, st = self.eval(images, p)
                ev = None
                if self.device.type == "cuda":
                    ev = torch.cuda.Event()
                    ev.record()
                return m, y, st, ev
        with net_lock:
            # no shared pinned staging buffer here: the previous batch's H2D may still be reading it
            x = as_batch(images, self.nchan, self.device)
            y, style, rescale = self._net_stage(x, p)
            main = torch.cuda.current_stream(self.device)
            ev = torch.cuda.Event()
            ev.record(main)
        with mask_lock:
            if getattr(self, "_mask_stream", None) is None:
                self._mask_stream = mask_stream(self.device)
            side = self._mask_stream
            with torch.cuda.stream(side):
                side.wait_event(ev)
                y.record_stream(side)
                with trace.span("cellpose.masks", cuda=True, images=y.shape[0]):
                    m = self.compute_masks(y, p, rescale)
            done = torch.cuda.Event()
            done.record(side)
        return m, y, style, done

    def stream(self, p: EvalParams | None = None) -> "_EvalStream":
        """Cross-batch pipeline for a stream of batches (continuous serving / offline throughput):
        ``submit(images)`` queues batch i's network on the current stream, then runs mask recovery of
        batch i-1 on a second HIP stream (so its latency-bound kernels and host syncs overlap batch
        i's convs) and returns batch i-1's ``(masks, flows, styles)`` (None for the first batch);
        ``flush()`` returns the last batch's.  Same per-batch results as :meth:`eval`."""
        return _EvalStream(self, p or EvalParams())

    def _normalize(self, x):
        if self.device.type == "cuda":
            from .gpu import normalize99

            return normalize99(x)
        return torch.stack([torch.from_numpy(ref.normalize99(x[b].numpy())) for b in range(x.shape[0])])

    def compute_masks(self, y: torch.Tensor, p: EvalParams, rescale: float = 1.0) -> torch.Tensor:
        niter = p.niter if p.niter else int(200 / max(rescale, 1e-3))
        if self.device.type == "cuda":
            from .gpu import compute_masks_gpu

            return compute_masks_gpu(y, niter=niter, cellprob_threshold=p.cellprob_threshold,
                                     flow_threshold=p.flow_threshold, min_size=p.min_size,
                                     max_size_fraction=p.max_size_fraction)
        out = []
        for b in range(y.shape[0]):
            yb = y[b].numpy()
            m = ref.compute_masks(yb[:2], yb[2], niter=niter, cellprob_threshold=p.cellprob_threshold,
                                  flow_threshold=p.flow_threshold, min_size=p.min_size,
                                  max_size_fraction=p.max_size_fraction)
            out.append(torch.from_numpy(m.astype(np.int32)))
        return torch.stack(out)


def mask_stream(device) -> "torch.cuda.Stream":
    """The second stream mask recovery runs on, beside the next batch's network.
    ``BE_MASK_STREAM_PRIO`` (A/B): HIP stream priority, -1 = high (its kernels dispatch ahead of the
    queued conv workgroups), 0 = normal."""
    prio = int(os.environ.get("BE_MASK_STREAM_PRIO", "0"))
    return torch.cuda.Stream(device, priority=prio)


class _GroupNormEngine:
    """Inference for GroupNorm CPnets (e.g. sessions trained data-parallel): GroupNorm statistics are
    per image, so nothing folds into the weights; the HIP training engine's forward -- GN statistics
    kernel + fused conv per layer, no activations saved for a backward -- runs the tiles instead
    (one engine per tile-batch size).  Non-square tile grids fall back to bf16 autocast PyTorch."""

    def __init__(self, net: CPnet, device):
        import copy

        from ..parallel.ddp import FlatParams

        self.device = torch.device(device)
        self.net = copy.deepcopy(net).to(self.device).eval()
        self.fp = FlatParams(self.net, self.device) if self.device.type == "cuda" else None
        self._engs: dict = {}

    @torch.no_grad()
    def __call__(self, tiles: torch.Tensor):
        from ..train.cpnet_engine import CPnetTrainEngine

        T, by, bx, _ = tiles.shape
        x = tiles[..., : self.net.nchan].permute(0, 3, 1, 2).float()
        if by != bx or by % 16 or self.fp is None:
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.device.type == "cuda"):
                y, style = self.net(x.contiguous())[:2]
            return y.float().contiguous(), style.float()
        eng = self._engs.get((T, by))
        if eng is None:
            eng = self._engs[(T, by)] = CPnetTrainEngine(self.net, self.fp, T, by, self.device)
        y = eng.forward(x)
        style = eng._act["style"].float()
        eng._act = None
        return y, style


def synthetic_cells(B: int, H: int = 512, W: int = 512, nchan: int = 2, ncells: int = 150, seed: int = 0) -> np.ndarray:
    """Synthetic fluorescence-like images [B, nchan, H, W] uint16: Gaussian blobs (cells) + nuclei + noise."""
    rng = np.random.default_rng(seed)
    out = np.zeros((B, nchan, H, W), np.float32)
    yy, xx = np.mgrid[0:H, 0:W]
    for b in range(B):
        cy = rng.uniform(0, H, ncells)
        cx = rng.uniform(0, W, ncells)
        r = rng.uniform(6, 14, ncells)
        img = np.zeros((H, W), np.float32)
        nuc = np.zeros((H, W), np.float32)
        for i in range(ncells):
            y0, y1 = int(max(0, cy[i] - 3 * r[i])), int(min(H, cy[i] + 3 * r[i]))
            x0, x1 = int(max(0, cx[i] - 3 * r[i])), int(min(W, cx[i] + 3 * r[i]))
            d2 = (yy[y0:y1, x0:x1] - cy[i]) ** 2 + (xx[y0:y1, x0:x1] - cx[i]) ** 2
            img[y0:y1, x0:x1] += np.exp(-d2 / (2 * r[i] ** 2))
            nuc[y0:y1, x0:x1] += np.exp(-d2 / (2 * (0.4 * r[i]) ** 2))
        out[b, 0] = img
        if nchan > 1:
            out[b, 1] = nuc
    out += 0.05 * rng.standard_normal(out.shape).astype(np.float32)
    out = np.clip(out, 0, None)
    return (out / out.max() * 4000).astype(np.uint16)


class _EvalStream:
    """See :meth:`CellposeRunner.stream` (GPU only; a CPU runner evaluates each batch directly)."""

    def __init__(self, runner: CellposeRunner, p: EvalParams):
        self.r, self.p = runner, p
        self.pending = None
        self.cuda = runner.device.type == "cuda" and p.compute_masks
        if self.cuda:
            if getattr(runner, "_mask_stream", None) is None:
                runner._mask_stream = mask_stream(runner.device)
            self.side = runner._mask_stream

    @torch.no_grad()
    def submit(self, images):
        if not self.cuda:
            return self.r.eval(images, self.p)
        x = as_batch(images, self.r.nchan, self.r.device)  # device tensors only: no shared pinned staging
        y, style, rescale = self.r._net_stage(x, self.p)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.r.device))
        prev, self.pending = self.pending, (y, style, rescale, ev)
        return self._finish(prev) if prev is not None else None

    def _finish(self, item):
        y, style, rescale, ev = item
        main = torch.cuda.current_stream(self.r.device)
        with torch.cuda.stream(self.side):
            self.side.wait_event(ev)
            y.record_stream(self.side)
            with trace.span("cellpose.masks", cuda=True, images=y.shape[0]):
                m = self.r.compute_masks(y, self.p, rescale)
        done = torch.cuda.Event()
        done.record(self.side)
        main.wait_event(done)  # consumers on the main stream see finished masks
        m.record_stream(main)
        return m, y, style

    def flush(self):
        if self.pending is None:
            return None
        prev, self.pending = self.pending, None
        return self._finish(prev)
