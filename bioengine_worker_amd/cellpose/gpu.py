"""GPU (HIP) implementation of Cellpose pre/post-processing on batches of images.

Every heavy step is a kernel in ``csrc/kernels/{tiles,cellpose_dynamics,cellpose_masks}.hip``;
torch is only used for tiny bookkeeping (sorting the seed keys, prefix sums over labels, building
per-mask job lists).  The semantics are those of :mod:`bioengine_worker_amd.cellpose.reference`
(the CPU oracle), which the GPU tests compare against.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from ..ops import _native
from . import reference as ref

RPAD = 20
_JOB_BYTES = 32
LDS_DIFFUSE_BYTES = 156 * 1024  # one mask per CU up to ~95 x 95 boxes; larger ones run tiled
LDS_FILL_BYTES = 32 * 1024


def _launch_cfg(n: int):
    return n


# ------------------------------------------------------------------ percentiles / tiles


_pct_ws: dict = {}


def normalize99(x: torch.Tensor, lower: float = 1.0, upper: float = 99.0) -> torch.Tensor:
    """x [B, C, H, W] -> float32 normalised per (image, channel) with np.percentile 'linear' semantics.

    On the GPU: radix-select HIP kernel (``csrc/kernels/percentile.hip``; six order statistics per
    row in four digit passes, no sort).  :func:`normalize99_sort` is the torch formulation it is
    tested against."""
    if x.device.type != "cuda":
        return normalize99_sort(x, lower, upper)
    B, C, H, W = x.shape
    xf = x.float().contiguous()
    rows = B * C
    sptr = _native.stream(x.device)
    key = (x.device, getattr(sptr, "value", sptr))  # one workspace per stream: concurrent streams never share histograms
    ws = _pct_ws.get(key)
    need = rows * 6 * 258 * 4
    if ws is None or ws.numel() < need:  # hist part must start zeroed; every call leaves it zeroed
        ws = _pct_ws[key] = torch.zeros(max(need, 64 * 6 * 258 * 4), dtype=torch.uint8, device=x.device)
    out = torch.empty_like(xf)
    _native.call("be_pct_normalize", _native.ptr(xf), rows, H * W, float(lower), float(upper), _native.ptr(out),
                 _native.ptr(ws), ws.numel() // 4 * 4, sptr)
    return out


def normalize99_sort(x: torch.Tensor, lower: float = 1.0, upper: float = 99.0) -> torch.Tensor:
    """Sort-based torch formulation of :func:`normalize99` (CPU path and test oracle)."""
    B, C, H, W = x.shape
    xf = x.float().reshape(B * C, H * W)
    srt, _ = torch.sort(xf, dim=1)
    n = H * W

    def pct(q):
        pos = q / 100.0 * (n - 1)
        lo = int(np.floor(pos))
        hi = min(lo + 1, n - 1)
        frac = pos - lo
        return srt[:, lo] * (1 - frac) + srt[:, hi] * frac

    p1, p99 = pct(lower), pct(upper)
    rng = (p99 - p1)
    ok = rng > 1e-3
    scale = torch.where(ok, 1.0 / torch.where(ok, rng, torch.ones_like(rng)), torch.ones_like(rng))
    const = (srt[:, -1] - srt[:, 0]) == 0
    out = (xf - p1[:, None]) * scale[:, None]
    out = torch.where(const[:, None], torch.zeros_like(out), out)
    return out.reshape(B, C, H, W)


class TilePlan:
    """Cellpose tiling of an (H, W) image: pad to a multiple of 16 (+8 margin), 224 tiles, 10 % overlap."""

    def __init__(self, H: int, W: int, bsize: int = 224, overlap: float = 0.1, device="cpu"):
        self.H, self.W = H, W
        ya, yb = ref.pad_amounts(H)
        xa, xb = ref.pad_amounts(W)
        self.pad_y, self.pad_x = ya, xa
        self.Hp, self.Wp = H + ya + yb, W + xa + xb
        self.ys = ref.tile_starts(self.Hp, bsize, overlap)
        self.xs = ref.tile_starts(self.Wp, bsize, overlap)
        self.by, self.bx = min(bsize, self.Hp), min(bsize, self.Wp)
        self.nt = len(self.ys) * len(self.xs)
        m = ref.taper_mask(self.by, self.bx)
        # the 2-D taper is separable: recover the 1-D factors from its centre row/col
        cy, cx = self.by // 2, self.bx // 2
        wy = m[:, cx] / np.sqrt(m[cy, cx])
        wx = m[cy, :] / np.sqrt(m[cy, cx])
        dev = torch.device(device)
        self.ys_t = torch.tensor(self.ys, dtype=torch.int32, device=dev)
        self.xs_t = torch.tensor(self.xs, dtype=torch.int32, device=dev)
        self.wy = torch.tensor(wy, dtype=torch.float32, device=dev)
        self.wx = torch.tensor(wx, dtype=torch.float32, device=dev)

    def gather(self, img: torch.Tensor, cpad: int) -> torch.Tensor:
        B, C, H, W = img.shape
        out = torch.empty(B * self.nt, self.by, self.bx, cpad, dtype=torch.bfloat16, device=img.device)
        img = img.float().contiguous()
        _native.call("be_tiles_gather", _native.ptr(img), B, C, H, W, self.pad_y, self.pad_x, _native.ptr(self.ys_t),
                     _native.ptr(self.xs_t), len(self.ys), len(self.xs), self.by, self.bx, cpad, _native.ptr(out),
                     _native.stream(img.device))
        return out

    def blend(self, yt: torch.Tensor, B: int) -> torch.Tensor:
        nout = yt.shape[1]
        out = torch.empty(B, nout, self.H, self.W, dtype=torch.float32, device=yt.device)
        _native.call("be_tiles_blend", _native.ptr(yt), B, nout, self.H, self.W, self.pad_y, self.pad_x,
                     _native.ptr(self.ys_t), _native.ptr(self.xs_t), len(self.ys), len(self.xs), self.by, self.bx,
                     _native.ptr(self.wy), _native.ptr(self.wx), _native.ptr(out), _native.stream(yt.device))
        return out


# ------------------------------------------------------------------ mask recovery


def _jobs_tensor(b, lab, y0, x0, ly, lx, scratch) -> torch.Tensor:
    """Pack MaskJob structs {int b, lab, y0, x0, ly, lx; int64 scratch} as int64 words."""
    w0 = (b.long() & 0xFFFFFFFF) | (lab.long() << 32)
    w1 = (y0.long() & 0xFFFFFFFF) | (x0.long() << 32)
    w2 = (ly.long() & 0xFFFFFFFF) | (lx.long() << 32)
    return torch.stack([w0, w1, w2, scratch.long()], 1).contiguous()


def _plan_jobs(bbox_valid, labs_b, labs_l, lds_fn, caps, scratch_fn, valid=None):
    """Bucket masks by their LDS need with ONE host sync.

    Bucket k < len(caps) holds masks with caps[k-1] < need <= caps[k]; bucket len(caps) holds the
    masks too big for LDS, which get scratch offsets.  Jobs are sorted by bucket on the device and
    only the per-bucket counts (+ the scratch total) come back to the host, so the slices below
    are views -- replacing one boolean-index gather (a nonzero + sync, ~75 us) per field and bucket.
    ``valid`` (optional bool per row) drops rows without a separate nonzero (and its sync).
    Returns ``(jobs_by_bucket: list of [n_k, 4] int64 views, scratch_total)``."""
    y0, y1, x0, x1 = bbox_valid.unbind(1)
    ly, lx = y1 - y0 + 1, x1 - x0 + 1
    need = lds_fn(ly, lx)
    dev = bbox_valid.device
    edges = torch.tensor(caps, dtype=need.dtype, device=dev)
    bucket = torch.bucketize(need, edges)  # need <= caps[k]  ->  k
    nb = len(caps) + 1
    if valid is not None:
        bucket = torch.where(valid, bucket, torch.full_like(bucket, nb))  # dropped rows sort last
    order = torch.argsort(bucket, stable=True)
    counts = torch.bincount(bucket, minlength=nb + 1)[:nb]
    big = bucket[order] == len(caps)
    ly_s, lx_s = ly[order], lx[order]
    sz = torch.where(big, scratch_fn(ly_s, lx_s), torch.zeros_like(ly_s)).long()
    off = torch.cumsum(sz, 0) - sz
    scr = torch.where(big, off, torch.full_like(off, -1))
    jobs = _jobs_tensor(labs_b[order], labs_l[order], y0[order], x0[order], ly_s, lx_s, scr)
    host = torch.cat([counts.long(), sz.sum().view(1)]).cpu().tolist()  # the one sync
    out, start = [], 0
    for k in range(nb):
        out.append(jobs[start:start + host[k]])
        start += host[k]
    return out, int(host[nb])


def _plan_masks(bbox: torch.Tensor, valid: torch.Tensor | None, kind: int, caps):
    """Device-side :func:`_plan_jobs` (one ``be_cp_plan_masks`` launch + one host sync): returns
    ``(jobs_by_bucket, scratch_total, niter_img)``; ``kind`` 0 = diffusion (LDS need / scratch of
    :func:`_diffuse_lds_bytes` / :func:`_diffuse_scratch_doubles`, and cellpose's per-image
    ``niter_img``), 1 = hole filling (``R`` bytes).  Job order inside a bucket is arbitrary."""
    return _plan_finish([_plan_launch(bbox, valid, kind, caps)])[0]


def _plan_finish(launched: list) -> list:
    """Read back the bucket sizes of several :func:`_plan_launch` plans with ONE host sync."""
    host = torch.cat([torch.cat([counts.long(), tot]) for _, counts, tot, _ in launched]).cpu().tolist()
    out, o = [], 0
    for jobs, counts, _, niter_img in launched:
        nb = counts.shape[0]
        out.append(([jobs[k, :host[o + k]] for k in range(nb)], int(host[o + nb]), niter_img))
        o += nb + 1
    return out


def _plan_launch(bbox: torch.Tensor, valid: torch.Tensor | None, kind: int, caps, counts: torch.Tensor | None = None):
    """``counts`` (kind 0): per-label pixel counts; the too-big-for-LDS masks then split into a
    big-sparse bucket (``len(caps)``) and the tiled one (last)."""
    B, nlab = bbox.shape[:2]
    dev = bbox.device
    n = B * nlab
    split = kind in (0, 2) and counts is not None
    if split:
        assert counts.shape == (B, nlab) and counts.dtype == torch.int32
        px_counts = counts.contiguous()
    # kind 2 (needs counts): the compact work-queue buckets (wave jobs, workgroup jobs) in front of
    # kind 0's buckets, which keep the masks the queue kernel cannot take
    nb = len(caps) + 1 + int(split) + (2 if kind == 2 and split else 0) + (2 if kind == 3 else 0)
    jobs = torch.empty(nb, max(n, 1), 4, dtype=torch.int64, device=dev)
    bucket_n = torch.zeros(nb, dtype=torch.int32, device=dev)
    tot = torch.zeros(1, dtype=torch.int64, device=dev)
    niter_img = torch.zeros(B, dtype=torch.int32, device=dev)
    carr = (ctypes.c_int * max(1, len(caps)))(*[int(c) for c in caps])
    vptr = _native.ptr(valid.contiguous().view(torch.uint8)) if valid is not None else None
    cptr = _native.ptr(px_counts) if split else None
    _native.call("be_cp_plan_masks", _native.ptr(bbox.contiguous()), vptr, cptr, B, nlab, kind, ctypes.addressof(carr),
                 len(caps), _native.ptr(jobs), _native.ptr(bucket_n), _native.ptr(tot), _native.ptr(niter_img),
                 _native.stream(dev))
    return jobs, bucket_n, tot, niter_img


#: compact work-queue diffusion (be_cp_diffuse_q) for the masks it can take; 0 = the LDS-box buckets
DIFFUSE_QUEUE = os.environ.get("BE_DIFFUSE_QUEUE", "1") != "0"


def _diffuse_plan_kind() -> int:
    return 2 if DIFFUSE_QUEUE else 0


#: one-wave hole filling (be_cp_fill_holes_wave) for boxes up to 64 x 64 with the ring; 0 = LDS kernel only
FILL_WAVE = os.environ.get("BE_FILL_WAVE", "1") != "0"


def _fill_plan_kind() -> int:
    return 3 if FILL_WAVE else 1


def _diffuse_lds_bytes(ly, lx):
    R = (ly + 2) * (lx + 2)
    return 16 * R + 4 * (ly + 2 + lx + 2) + R + 16


def _diffuse_scratch_doubles(ly, lx):
    R = (ly + 2) * (lx + 2)
    return 2 * R + (ly + 2 + lx + 2 + 1) // 2 + (R + 7) // 8 + 2


#: (LDS bytes, threads) buckets of the one-workgroup-per-mask diffusion: a block reserves only its
#: bucket's LDS, so small masks run many blocks per CU (one 48 KiB reservation per mask allowed 3).
DIFFUSE_BUCKETS = ((6 * 1024, 64), (12 * 1024, 128), (24 * 1024, 256), (48 * 1024, 256), (80 * 1024, 512),
                   (LDS_DIFFUSE_BYTES, 512))
DIFFUSE_CAPS = [c for c, _ in DIFFUSE_BUCKETS]
#: rows per work item of the diffusion sweep (``BE_DIFFUSE_DV``): a smaller DV gives every mask
#: proportionally more threads (buckets scale up to 1024) and a shorter serial LDS chain per sweep
DIFFUSE_DV = 4


def _diffuse_dv() -> int:
    return int(os.environ.get("BE_DIFFUSE_DV", DIFFUSE_DV))


def _diffuse_buckets(dv: int):
    return tuple((cap, min(1024, t * (8 // dv))) for cap, t in DIFFUSE_BUCKETS)


_DEBUG_STATS = os.environ.get("BIOENGINE_MASK_STATS", "0") == "1"


#: flow-following launch: LDS-staged flow window per 32 x 32 tile (default), XCD-ordered +
#: block-compacted L2 gathers, or the plain pixel-per-lane one (all bit-identical)
FOLLOW_FLOWS_ENTRY = os.environ.get("BIOENGINE_FOLLOW_ENTRY", "be_cp_follow_flows_lds")

_SIDE_STREAMS: dict = {}
#: LDS buckets run on their own HIP streams so their launch tails (a few CUs finishing the
#: largest masks of a bucket) overlap the next bucket instead of idling the rest of the chip.
N_SIDE_STREAMS = 3


def _side_streams(dev):
    key = (dev.type, dev.index)
    if key not in _SIDE_STREAMS:
        _SIDE_STREAMS[key] = [torch.cuda.Stream(dev) for _ in range(N_SIDE_STREAMS)]
    return _SIDE_STREAMS[key]


def _bucket_small(slices):
    """(bucket index, LDS cap, threads, jobs) of the non-empty one-workgroup buckets, largest first
    (they set the critical path)."""
    out = []
    for i, (cap, threads) in enumerate(_diffuse_buckets(_diffuse_dv())):
        if slices[i].shape[0]:
            out.append((i, cap, threads, slices[i]))
    if _DEBUG_STATS:
        print(f"[diffuse_small] buckets={[int(x.shape[0]) for x in slices[:-1]]} big={int(slices[-1].shape[0])}", flush=True)
    return out[::-1]


def _diffuse_small(Mc, buckets, niter_img, L, st, ready=None, scratch=None) -> None:
    """``ready``: event recorded on the current stream once the inputs exist; the buckets start
    from it instead of from the stream's tail, so they run alongside the big-mask kernel.

    Every bucket kernel runs ``niter`` dependent sweeps, so its time grows with its mask size and a
    stream's tail is the sum of its buckets: the buckets (largest first) go to the queues in snake
    order (0, 1, .., n-1, n-1, .., 0), and without a big-mask kernel the main stream is one of the
    queues (4 hardware queues per process: main + 3 side streams)."""
    B, H, W = Mc.shape
    concurrent = Mc.is_cuda and N_SIDE_STREAMS > 0
    if concurrent:
        main = torch.cuda.current_stream(Mc.device)
        sides = _side_streams(Mc.device)
        for sd in sides:
            if ready is not None:
                sd.wait_event(ready)
            else:
                sd.wait_stream(main)
        queues = sides if ready is not None else [None] + sides  # None = the main stream itself
        nq = len(queues)
    for k, (i, cap, threads, jobs) in enumerate(buckets):
        if concurrent:
            r = k % (2 * nq)
            sd = queues[r if r < nq else 2 * nq - 1 - r]
            if sd is None:
                sptr = st
            else:
                for t in (jobs, Mc, niter_img, L) + ((scratch,) if scratch is not None else ()):
                    t.record_stream(sd)
                sptr = ctypes.c_void_p(sd.cuda_stream)
        else:
            sptr = st
        if i < 0:  # big-sparse bucket: global-scratch heat field, one workgroup per mask
            _native.call("be_cp_diffuse_sparse_big", _native.ptr(Mc), _native.ptr(jobs), jobs.shape[0], H, W,
                         _native.ptr(niter_img), _native.ptr(scratch), _native.ptr(L), sptr)
            continue
        _native.call("be_cp_diffuse_nt", _native.ptr(Mc), _native.ptr(jobs), jobs.shape[0], H, W,
                     _native.ptr(niter_img), _native.ptr(L), cap, threads, _diffuse_dv(), sptr)
    if concurrent:
        for sd in sides:
            main.wait_stream(sd)


_TILE_PARAMS: tuple | None = None
#: "tiled" = multi-workgroup time-blocked diffusion for masks larger than LDS (default);
#: "block" = one workgroup per mask on a global scratch slab (kept as a cross-check).
BIG_MASK_MODE = "tiled"


def _diffuse_big(Mc, bj, niter_img, scratch, L, st, between=None) -> None:
    """Diffusion of masks too large for one workgroup's LDS (see diffuse_tiled_kernel).
    ``between()`` runs after the short per-mask centre kernel is queued and before the long
    cooperative sweep (the caller releases its other streams there)."""
    global _TILE_PARAMS
    B, H, W = Mc.shape
    if BIG_MASK_MODE == "block":
        if between is not None:
            between()
        _native.call("be_cp_diffuse", _native.ptr(Mc), _native.ptr(bj), bj.shape[0], H, W, _native.ptr(niter_img),
                     _native.ptr(scratch), _native.ptr(L), 0, st)
        return None
    if _TILE_PARAMS is None:
        import ctypes

        buf = (ctypes.c_int * 3)()
        _native.call("be_cp_diffuse_tile_params", ctypes.addressof(buf))
        _TILE_PARAMS = (buf[0], buf[1], buf[2])
    core = _TILE_PARAMS[0]
    w2 = bj[:, 2].cpu()
    ly, lx = (w2 & 0xFFFFFFFF), (w2 >> 32)
    nty = (ly + 2 + core - 1) // core
    ntx = (lx + 2 + core - 1) // core
    per = (nty * ntx)
    job = torch.repeat_interleave(torch.arange(bj.shape[0]), per)
    start = torch.cumsum(per, 0) - per
    k = torch.arange(int(per.sum())) - start[job]
    ty = (k // ntx[job]) * core
    tx = (k % ntx[job]) * core
    tiles = torch.stack([job, ty, tx, torch.zeros_like(job)], 1).to(torch.int32).to(Mc.device)
    if _DEBUG_STATS:
        print(f"[diffuse_big] masks={bj.shape[0]} tiles={tiles.shape[0]} box_ly={ly.tolist()} box_lx={lx.tolist()} "
              f"niter={niter_img.tolist()}", flush=True)
    centers = torch.empty(bj.shape[0], dtype=torch.int32, device=Mc.device)
    ws = torch.zeros(4, dtype=torch.int32, device=Mc.device)
    args = (_native.ptr(Mc), _native.ptr(bj), bj.shape[0], _native.ptr(tiles), tiles.shape[0], H, W,
            _native.ptr(niter_img), _native.ptr(scratch), _native.ptr(L), _native.ptr(centers), _native.ptr(ws))
    _native.call("be_cp_diffuse_tiled", *args, 1, st)
    if between is not None:
        between()
    _native.call("be_cp_diffuse_tiled", *args, 2, st)
    return ws  # ws[1] != 0 <=> the grid barrier timed out; checked by the caller after queuing the rest


def _check_tiled(ws) -> None:
    if ws is not None and int(ws[1].item()) != 0:
        raise RuntimeError("diffuse_tiled_kernel: grid barrier timed out (workgroups not co-resident)")


def label_counts(M: torch.Tensor, nlab: int) -> torch.Tensor:
    """Pixels per label [B, nlab] (label 0 not counted)."""
    B = M.shape[0]
    counts = torch.zeros(B, nlab, dtype=torch.int32, device=M.device)
    Mc = M.contiguous()
    _native.call("be_label_counts", _native.ptr(Mc), B, Mc[0].numel(), nlab, _native.ptr(counts), _native.stream(M.device))
    return counts


def mask_bboxes(M: torch.Tensor, nlab: int) -> torch.Tensor:
    B, H, W = M.shape
    bbox = torch.empty(B, nlab, 4, dtype=torch.int32, device=M.device)
    bbox[..., 0] = 2 ** 31 - 1
    bbox[..., 1] = -1
    bbox[..., 2] = 2 ** 31 - 1
    bbox[..., 3] = -1
    _native.call("be_cp_bbox", _native.ptr(M), B, H, W, nlab, _native.ptr(bbox), _native.stream(M.device))
    return bbox


def masks_to_flows_gpu(M: torch.Tensor, dp: torch.Tensor | None = None, niter: int | None = None,
                       nlab: int | None = None, counts: torch.Tensor | None = None, plan=None, want_mu: bool = True):
    """Heat-diffusion flows of label images M [B, H, W] int32 (labels 1..n, contiguous per image).

    Returns (mu [B, 2, H, W] fp32, err_sum [B, nlab] fp32 or None, counts [B, nlab]).  When ``dp``
    ([B, >=2, H, W] network output) is given, err_sum[b, l] = sum over mask l of |mu - dp/5|^2.
    ``counts`` / ``plan`` (label_counts and a kind-0 plan of the same labels) skip recomputing them;
    ``want_mu=False`` (flow QC: only the errors are used) returns ``mu=None`` and skips its writes.
    """
    B, H, W = M.shape
    dev = M.device
    if nlab is None:  # an upper bound on the labels + 1 is enough (absent labels have no pixels)
        nlab = int(M.max().item()) + 1 if M.numel() else 1
    mu = torch.zeros(B, 2, H, W, dtype=torch.float32, device=dev) if (want_mu or dp is None) else None
    if counts is None:
        counts = label_counts(M, nlab)
    if nlab <= 1:
        return mu, (torch.zeros(B, nlab, device=dev) if dp is not None else None), counts
    if plan is None:
        plan = _plan_finish([_plan_launch(mask_bboxes(M, nlab), None, _diffuse_plan_kind(), DIFFUSE_CAPS, counts)])[0]
    slices, ssize, niter_img = plan
    qjobs = None
    if len(slices) == len(DIFFUSE_BUCKETS) + 4:  # kind 2: queue buckets first
        qjobs, slices = slices[:2], slices[2:]
    if niter is not None:
        niter_img = torch.full((B,), niter, dtype=torch.int32, device=dev)
    bj = slices[-1]
    L = torch.zeros(B, H, W, dtype=torch.float64, device=dev)
    scratch = torch.empty(max(ssize, 1), dtype=torch.float64, device=dev)
    st = _native.stream(dev)
    Mc = M.contiguous()
    buckets = _bucket_small(slices)
    if len(slices) == len(DIFFUSE_BUCKETS) + 2 and slices[len(DIFFUSE_BUCKETS)].shape[0]:
        # big sparse masks: the longest-running launches (niter sweeps of the largest boxes), so
        # they head the queue order
        buckets.insert(0, (-1, 0, 1024, slices[len(DIFFUSE_BUCKETS)]))
    ws = None
    ready = None
    if bj.shape[0] and Mc.is_cuda and buckets:
        ready = torch.cuda.Event()

        def release():  # the buckets start once the big masks' centre kernel is done
            ready.record(torch.cuda.current_stream(dev))
    else:
        release = None
    if qjobs is not None and (qjobs[0].shape[0] or qjobs[1].shape[0]):
        # one persistent launch over every mask the compact kernel takes (nearly all of them),
        # queued first: the box-bucket kernels below then only see the rare leftovers
        qws = torch.empty(2, dtype=torch.int32, device=dev)
        _native.call("be_cp_diffuse_q", _native.ptr(Mc), _native.ptr(qjobs[0]), qjobs[0].shape[0], _native.ptr(qjobs[1]),
                     qjobs[1].shape[0], H, W, _native.ptr(niter_img), _native.ptr(L), _native.ptr(qws), st)
    if bj.shape[0]:
        # first, on an idle device: the centre kernel runs alone (~0.07 ms instead of ~0.36 ms
        # among the bucket kernels), then the cooperative tiled sweep -- the critical path -- is
        # queued right behind it; its few workgroups are resident before the bucket kernels
        # (which never wait on it) fill the remaining CUs, so its grid barrier cannot starve
        ws = _diffuse_big(Mc, bj, niter_img, scratch, L, st, between=release)
    if buckets:
        _diffuse_small(Mc, buckets, niter_img, L, st, ready=ready, scratch=scratch)
    err = None
    dpp = None
    bstride = 0
    if dp is not None:
        dpp = dp.float().contiguous()
        bstride = dpp.shape[1] * H * W
        err = torch.zeros(B, nlab, dtype=torch.float32, device=dev)
    _native.call("be_cp_flow_grad", _native.ptr(Mc), _native.ptr(L), B, H, W, _native.ptr(mu), _native.ptr(dpp),
                 bstride, _native.ptr(err), nlab, st)
    _check_tiled(ws)
    return mu, err, counts


def _renumber(M: torch.Tensor, keep: torch.Tensor) -> torch.Tensor:
    """keep [B, nlab] bool (index 0 ignored) -> M relabelled 1..k per image, dropped labels -> 0."""
    keep = keep.clone()
    keep[:, 0] = False
    lut = torch.cumsum(keep.int(), dim=1) * keep.int()
    B = M.shape[0]
    return torch.gather(lut, 1, M.reshape(B, -1).long()).reshape(M.shape).to(torch.int32)


def fill_holes_gpu(M: torch.Tensor, min_size: int = 15, nlab: int | None = None) -> torch.Tensor:
    """``nlab``: optional upper bound on the labels + 1 (saves the host sync on ``M.max()``)."""
    B, H, W = M.shape
    dev = M.device
    if nlab is None:
        nlab = int(M.max().item()) + 1 if M.numel() else 1
    if nlab <= 1:
        return M.clone()
    counts = label_counts(M, nlab)
    keep = counts > 0
    if min_size > 0:
        keep &= counts >= min_size
    keep[:, 0] = False
    plan = _plan_masks(mask_bboxes(M, nlab), keep, _fill_plan_kind(), [LDS_FILL_BYTES])
    return _fill_run(M, _rank_lut(keep), nlab, plan)


def _rank_lut(keep: torch.Tensor) -> torch.Tensor:
    """keep [B, nlab] bool -> int32 lut: kept label -> its rank 1..k (id order), dropped -> 0."""
    keep = keep.clone()
    keep[:, 0] = False
    return (torch.cumsum(keep.int(), dim=1) * keep.int()).to(torch.int32).contiguous()


def _fill_run(M: torch.Tensor, lut: torch.Tensor, nlab: int, plan) -> torch.Tensor:
    """Hole filling of the planned jobs (a kind-1 plan); jobs whose lut entry is 0 write nothing."""
    B, H, W = M.shape
    dev = M.device
    out = torch.zeros_like(M)
    slices, ssize, _ = plan
    wjs = []
    if len(slices) == 4:  # kind 3: the one-wave buckets (<= 64 x 64, <= 256 x 128 boxes) first
        wjs, slices = slices[:2], slices[2:]
    sj, bj = slices
    if sj.shape[0] + bj.shape[0] + sum(w.shape[0] for w in wjs) == 0:
        return out
    scratch = torch.empty(max(ssize, 1), dtype=torch.uint8, device=dev)
    st = _native.stream(dev)
    Mc = M.contiguous()
    for big, wj in enumerate(wjs):
        if wj.shape[0]:
            _native.call("be_cp_fill_holes_wave", _native.ptr(Mc), _native.ptr(wj), wj.shape[0], H, W, _native.ptr(lut), nlab,
                         _native.ptr(out), big, st)
    if sj.shape[0]:
        _native.call("be_cp_fill_holes", _native.ptr(Mc), _native.ptr(sj), sj.shape[0], H, W, _native.ptr(lut), nlab,
                     _native.ptr(scratch), _native.ptr(out), LDS_FILL_BYTES, st)
    if bj.shape[0]:
        _native.call("be_cp_fill_holes", _native.ptr(Mc), _native.ptr(bj), bj.shape[0], H, W, _native.ptr(lut), nlab,
                     _native.ptr(scratch), _native.ptr(out), 0, st)
    return out


def follow_and_label(y: torch.Tensor, niter: int = 200, cellprob_threshold: float = 0.0,
                     max_size_fraction: float = 0.4, with_bound: bool = False):
    """Network output y [B, 3, H, W] -> raw masks M0 [B, H, W] int32 (before QC / fill); with
    ``with_bound`` also an upper bound on its labels + 1 (known from the seed count, no extra sync)."""
    B, _, H, W = y.shape
    dev = y.device
    st = _native.stream(dev)
    y = y.float().contiguous()
    flow2 = torch.empty(B, H, W, 2, dtype=torch.float32, device=dev)
    fg = torch.empty(B, H, W, dtype=torch.uint8, device=dev)
    _native.call("be_cp_prep_flow", _native.ptr(y), B, H, W, float(cellprob_threshold), _native.ptr(flow2),
                 _native.ptr(fg), st)
    Hp, Wp = H + 2 * RPAD, W + 2 * RPAD
    hist = torch.zeros(B, Hp, Wp, dtype=torch.int32, device=dev)
    pos = torch.empty(B, H, W, dtype=torch.int32, device=dev)
    _native.call(FOLLOW_FLOWS_ENTRY, _native.ptr(flow2), _native.ptr(fg), _native.ptr(hist), _native.ptr(pos), B, H,
                 W, int(niter), st)
    cap = H * W // 11 + 1
    keys = torch.full((B, cap), torch.iinfo(torch.int64).max, dtype=torch.int64, device=dev)
    nseeds = torch.zeros(B, dtype=torch.int32, device=dev)
    _native.call("be_cp_seeds", _native.ptr(hist), B, Hp, Wp, _native.ptr(keys), _native.ptr(nseeds), cap, st)
    kmax = int(nseeds.max().item()) if B else 0  # host sync: sizes the sort and the expansion grid
    kmax = min(kmax, cap)
    M1 = torch.zeros(B, Hp, Wp, dtype=torch.int32, device=dev)
    M0 = torch.zeros(B, H, W, dtype=torch.int32, device=dev)
    if kmax == 0:
        return (M0, 1) if with_bound else M0
    # seeds are compacted at the front of each row: sort only the first kmax slots (a few hundred)
    # instead of the whole cap-wide buffer of sentinels
    keys_sorted, _ = torch.sort(keys[:, :kmax].contiguous(), dim=1)
    _native.call("be_cp_expand", _native.ptr(hist), _native.ptr(keys_sorted), _native.ptr(nseeds), B, Hp, Wp, kmax, kmax,
                 _native.ptr(M1), st)
    nlab = kmax + 1
    counts = torch.zeros(B, nlab, dtype=torch.int32, device=dev)
    _native.call("be_cp_label_lookup", _native.ptr(pos), _native.ptr(M1), B, H * W, Hp * Wp, _native.ptr(M0),
                 _native.ptr(counts), nlab, st)
    big = H * W * max_size_fraction
    keep = (counts > 0) & (counts <= big)
    M = _renumber(M0, keep)
    return (M, nlab) if with_bound else M


def compute_masks_gpu(y: torch.Tensor, niter: int = 200, cellprob_threshold: float = 0.0, flow_threshold: float = 0.4,
                      min_size: int = 15, max_size_fraction: float = 0.4) -> torch.Tensor:
    """Full Cellpose mask recovery for a batch: y [B, 3, H, W] -> masks [B, H, W] int32."""
    M, nlab = follow_and_label(y, niter, cellprob_threshold, max_size_fraction, with_bound=True)
    if nlab <= 1:
        return M
    # Label counts, boxes and BOTH job plans (QC diffusion, hole filling) come from the raw labels,
    # read back with one host sync.  QC only drops labels: the fill then runs on the raw ids with
    # QC-dropped masks zeroed (identical geometry to renumbering first) and a lut that ranks the
    # labels kept by QC and min_size in id order (= QC renumber followed by the fill's renumber).
    counts = label_counts(M, nlab)
    bbox = mask_bboxes(M, nlab)
    fill_keep = counts > 0
    if min_size > 0:
        fill_keep &= counts >= min_size
    fill_keep[:, 0] = False
    qc = flow_threshold is not None and flow_threshold > 0
    # masks below min_size are dropped whatever their flow error: the QC diffusion skips them (the
    # plan still takes cellpose's per-image niter over ALL masks, so the kept masks' flows are
    # unchanged)
    plans = _plan_finish(([_plan_launch(bbox, fill_keep, _diffuse_plan_kind(), DIFFUSE_CAPS, counts)] if qc else [])
                         + [_plan_launch(bbox, fill_keep, _fill_plan_kind(), [LDS_FILL_BYTES])])
    if qc:
        _, err, _ = masks_to_flows_gpu(M, dp=y, nlab=nlab, counts=counts, plan=plans[0], want_mu=False)
        qc_keep = (counts > 0) & ~(err / counts.clamp(min=1).float() > flow_threshold)
        qc_keep[:, 0] = False
        M = torch.gather(qc_keep.to(torch.int32), 1, M.reshape(M.shape[0], -1).long()).reshape(M.shape) * M
        fill_keep &= qc_keep
    return _fill_run(M.contiguous(), _rank_lut(fill_keep), nlab, plans[-1])
