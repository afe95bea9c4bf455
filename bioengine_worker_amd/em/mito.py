"""EM mitochondria instance segmentation pipeline on MI355X.

Reference semantics (apps/fibsem-mito-analysis/analysis_deployment.py): percentile (1, 99)
normalisation; 512 tiles with 64 overlap, reflect-padded edge tiles, Gaussian window
``exp(-2y^2) exp(-2x^2)`` blending (:108-156); ``_prob_to_instances`` (:160-176): threshold 0.5,
``remove_small_objects(min_size=300)`` (4-connectivity), ``binary_closing(disk(4))``, EDT,
``peak_local_max(min_distance=8, labels=closed)``, ``watershed(-dist, label(peaks), mask=closed)``;
regionprops area / axis lengths / eccentricity / centroid (:256-271).

Dense stages are HIP kernels (``imageproc.hip``: CCL; ``morphology.hip``: blend, disk morphology,
EDT, max filter, moments; ``em_watershed.hip``: marker watershed 2-D/3-D and the 3-D EDT); the
greedy peak spacing and the CPU priority-flood watershed (oracle and CPU path) run in the C++ host
runtime (``csrc/runtime/watershed.cpp``).  skimage is not available in this image, so
exact parity with it is "unpinned": every stage is tested against scipy/numpy oracles of the same
definition (tests/test_em_*.py).
"""
from __future__ import annotations

import math
import os
from typing import Callable

import numpy as np
import torch

from ..ops import _native


def gaussian_window(n: int) -> torch.Tensor:
    t = torch.linspace(-1, 1, n, dtype=torch.float64)
    return torch.exp(-2 * t ** 2).float()


def normalize_percentile(img: torch.Tensor, p1: float = 1.0, p99: float = 99.0) -> torch.Tensor:
    from ..search.preprocess import percentiles

    lo, hi = percentiles(img.reshape(1, -1).float(), (p1, p99))
    return ((img.float() - lo) / (hi - lo + 1e-6)).clamp(0, 1)


def tile_stack(img: torch.Tensor, tile: int = 512, overlap: int = 64) -> torch.Tensor:
    """The [T, 1, tile, tile] tiles :func:`infer_tiled` feeds its model for ``img`` [H, W], in order."""
    H, W = img.shape
    stride = tile - overlap
    ys, xs = list(range(0, H, stride)), list(range(0, W, stride))
    padded = torch.nn.functional.pad(img[None, None].float(), (0, max(0, xs[-1] + tile - W), 0, max(0, ys[-1] + tile - H)),
                                     mode="reflect" if (xs[-1] + tile - W < W and ys[-1] + tile - H < H) else "replicate")[0, 0]
    return torch.stack([padded[y:y + tile, x:x + tile] for y in ys for x in xs])[:, None]


def infer_tiled(img: torch.Tensor, predict: Callable[[torch.Tensor], torch.Tensor], tile: int = 512,
                overlap: int = 64, batch: int = 8) -> torch.Tensor:
    """img [H, W] (GPU) -> blended prediction [C, H, W].  ``predict`` maps [T, 1, tile, tile] ->
    [T, C, tile, tile].  Tiles are batched; stitching is the HIP gather-blend kernel."""
    H, W = img.shape
    stride = tile - overlap
    ys, xs = list(range(0, H, stride)), list(range(0, W, stride))
    padded = torch.nn.functional.pad(img[None, None].float(), (0, max(0, xs[-1] + tile - W), 0, max(0, ys[-1] + tile - H)),
                                     mode="reflect" if (xs[-1] + tile - W < W and ys[-1] + tile - H < H) else "replicate")[0, 0]
    coords = [(y, x) for y in ys for x in xs]
    outs = []
    for i in range(0, len(coords), batch):
        t = torch.stack([padded[y:y + tile, x:x + tile] for y, x in coords[i:i + batch]])[:, None]
        outs.append(predict(t).float())
    probs = torch.cat(outs).contiguous()
    C = probs.shape[1]
    w = gaussian_window(tile).to(img.device)
    out = torch.empty(C, H, W, dtype=torch.float32, device=img.device)
    if img.is_cuda:
        _native.call("be_blend_gather", _native.ptr(probs), C, 1, H, W, 1, len(ys), len(xs), stride, 1, 1, tile,
                     _native.ptr(w), _native.ptr(w), _native.ptr(w), _native.ptr(out), _native.stream(img.device))
    else:
        out = blend_reference(probs, H, W, ys, xs, tile)
    return out


def blend_reference(probs: torch.Tensor, H: int, W: int, ys, xs, tile: int) -> torch.Tensor:
    """float64 scatter-add blend exactly as the reference does (CPU oracle)."""
    C = probs.shape[1]
    w = gaussian_window(tile).double()
    win = w[:, None] * w[None, :]
    acc = torch.zeros(C, H, W, dtype=torch.float64)
    wacc = torch.zeros(H, W, dtype=torch.float64)
    k = 0
    for y in ys:
        for x in xs:
            th, tw = min(tile, H - y), min(tile, W - x)
            acc[:, y:y + th, x:x + tw] += probs[k, :, :th, :tw].double().cpu() * win[:th, :tw]
            wacc[y:y + th, x:x + tw] += win[:th, :tw]
            k += 1
    return (acc / wacc.clamp(min=1e-300)).float()


# ------------------------------------------------------------------ post-processing (GPU)

def ccl(mask: torch.Tensor, conn: int = 8) -> torch.Tensor:
    B = 1 if mask.dim() == 2 else mask.shape[0]
    m = mask.reshape(B, mask.shape[-2], mask.shape[-1]).to(torch.uint8).contiguous()
    lab = torch.empty(m.shape, dtype=torch.int32, device=m.device)
    _native.call("be_ccl_conn", _native.ptr(m), B, m.shape[1], m.shape[2], conn, _native.ptr(lab), _native.stream(m.device))
    return lab.reshape(mask.shape)


def compact_labels(roots: torch.Tensor) -> tuple[torch.Tensor, int]:
    """Root-index labels (-1 bg) -> 1..n in raster order of each component's first pixel."""
    fg = roots >= 0
    u, inv = torch.unique(roots[fg], return_inverse=True)  # sorted roots = raster order of first pixel
    out = torch.zeros_like(roots)
    out[fg] = inv.to(roots.dtype) + 1
    return out, int(u.numel())


def _keep_large(roots: torch.Tensor, min_size: int) -> torch.Tensor:
    """Foreground voxels whose component (CCL root index, -1 = background) has >= ``min_size``
    voxels.  GPU: per-chunk LDS hash maps, one global atomic per root and chunk
    (``be_component_keep``) -- plain per-voxel atomics serialised on large components (millions of
    adds to one address took 5 s on a 128 x 2048^2 volume), and the sort-based ``unique`` took
    0.25 s per 256 x 2048^2 slab.  CPU: ``unique`` with counts."""
    flat = roots.reshape(-1)
    if COMP_KEEP_GPU and flat.is_cuda and flat.dtype == torch.int32 and flat.numel() < 2 ** 31:
        # run-length atomics into a per-root counter (be_component_keep), no sort
        rc = flat.contiguous()
        counts = torch.empty(rc.numel(), dtype=torch.int32, device=rc.device)
        out = torch.empty(rc.numel(), dtype=torch.uint8, device=rc.device)
        _native.call("be_component_keep", _native.ptr(rc), rc.numel(), _native.ptr(counts), int(min_size), _native.ptr(out),
                     _native.stream(rc.device))
        return out.view(torch.bool).reshape(roots.shape)
    fg = flat >= 0
    _, inv, cnt = torch.unique(flat[fg], return_inverse=True, return_counts=True)
    keep = torch.zeros(flat.shape, dtype=torch.bool, device=roots.device)
    keep[fg] = cnt[inv] >= min_size
    return keep.reshape(roots.shape)


def remove_small_objects(mask: torch.Tensor, min_size: int = 300, conn: int = 4) -> torch.Tensor:
    return _keep_large(ccl(mask, conn), min_size)


def binary_closing_disk(mask: torch.Tensor, r: int = 4) -> torch.Tensor:
    H, W = mask.shape
    m = mask.to(torch.uint8).contiguous()
    tmp, out = torch.empty_like(m), torch.empty_like(m)
    st = _native.stream(m.device)
    _native.call("be_morph_disk", _native.ptr(m), _native.ptr(tmp), 1, H, W, r, 0, 0, st)
    _native.call("be_morph_disk", _native.ptr(tmp), _native.ptr(out), 1, H, W, r, 1, 0, st)
    return out.bool()


def edt(mask: torch.Tensor) -> torch.Tensor:
    H, W = mask.shape
    m = mask.to(torch.uint8).contiguous()
    dev = m.device
    dist = torch.empty(H, W, dtype=torch.float32, device=dev)
    g = torch.empty(H, W, dtype=torch.int32, device=dev)
    v = torch.empty(H * W + H, dtype=torch.int32, device=dev)  # tail: fallback row flags
    z = torch.empty(H, W + 1, dtype=torch.float64, device=dev)
    _native.call("be_edt", _native.ptr(m), _native.ptr(dist), _native.ptr(g), _native.ptr(v), _native.ptr(z), 1, H, W,
                 _native.stream(dev))
    return dist


def max_filter(x: torch.Tensor, r: int) -> torch.Tensor:
    H, W = x.shape
    a = x.float().contiguous()
    t, o = torch.empty_like(a), torch.empty_like(a)
    st = _native.stream(a.device)
    _native.call("be_max_filter_1d", _native.ptr(a), _native.ptr(t), 1, H, W, r, 0, st)
    _native.call("be_max_filter_1d", _native.ptr(t), _native.ptr(o), 1, H, W, r, 1, st)
    return o


def ensure_spacing(coords: np.ndarray, spacing: int) -> np.ndarray:
    import ctypes

    c = np.ascontiguousarray(coords, dtype=np.int32)
    keep = np.zeros(len(c), np.uint8)
    if len(c):
        _native.rt_call("be_rt_ensure_spacing", c.ctypes.data_as(ctypes.c_void_p), len(c), c.shape[1], int(spacing),
                        keep.ctypes.data_as(ctypes.c_void_p))
    return c[keep.astype(bool)]


def peak_local_max(dist: torch.Tensor, closed: torch.Tensor, min_distance: int = 8) -> np.ndarray:
    """skimage.feature.peak_local_max(dist, min_distance, labels=closed) (exclude_border=True)."""
    H, W = dist.shape
    b = min_distance
    inner = torch.zeros_like(closed)
    if H > 2 * b and W > 2 * b:
        inner[b:H - b, b:W - b] = True
    lm = closed & inner
    img = torch.where(lm, dist, torch.full_like(dist, -3.0e38))
    mx = max_filter(img, min_distance)
    thr = float(dist.min())
    cand = (img == mx) & (img > thr) & lm
    yx = cand.nonzero()
    if yx.shape[0] == 0:
        return np.zeros((0, 2), np.int64)
    inten = img[yx[:, 0], yx[:, 1]]
    order = torch.sort(-inten, stable=True).indices
    coords = yx[order].cpu().numpy()
    return ensure_spacing(coords, min_distance).astype(np.int64)


def watershed(neg_dist: np.ndarray, markers: np.ndarray, mask: np.ndarray, conn: int = 1) -> np.ndarray:
    import ctypes

    img = np.ascontiguousarray(neg_dist, np.float32)
    mk = np.ascontiguousarray(markers, np.int32)
    ms = np.ascontiguousarray(mask, np.uint8)
    out = np.zeros(img.shape, np.int32)
    D, H, W = (1,) + img.shape if img.ndim == 2 else img.shape
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    _native.rt_call("be_rt_watershed", vp(img), vp(mk), vp(ms), D, H, W, conn, vp(out))
    return out


#: component sizes in per-chunk LDS hash maps (be_component_keep; BE_COMP_KEEP=0: the torch.unique
#: sort): remove_small 0.19 vs 0.25 s per 256 x 2048^2 slab (s41; the first, run-length version
#: took 0.50 s, s39)
COMP_KEEP_GPU = os.environ.get("BE_COMP_KEEP", "1") != "0"

#: closing on bit-packed rows (BE_MORPH_BITS=0: the per-pixel window kernel)
MORPH_BITS = os.environ.get("BE_MORPH_BITS", "1") != "0"

#: relax only the tiles whose neighbourhood changed in the previous sweep (BE_WS_ACTIVE=0: every tile)
WS_ACTIVE_TILES = os.environ.get("BE_WS_ACTIVE", "1") != "0"


#: relaxation iterations inside a tile per sweep / launches between convergence checks (A/B knobs)
WS_MAX_LOCAL = int(os.environ.get("BE_WS_MAX_LOCAL", "64"))  # 32: 0.063 s, 64: 0.060 s per 64-slice slab (profiles/r06/em3d/ws_knobs_s20.txt)
WS_CHECK_EVERY = int(os.environ.get("BE_WS_CHECK_EVERY", "4"))
#: sweeps of the last watershed_gpu call (reported in the split-stage timings)
LAST_WS_SWEEPS = 0
#: wide watershed tiles when the volume has more than this many voxels per marker (a basin ~64^3)
WS_WIDE_VOXELS_PER_BASIN = 64 ** 3


def watershed_gpu(elev: torch.Tensor, markers: torch.Tensor, mask: torch.Tensor | None = None,
                  max_local: int | None = None, check_every: int | None = None,
                  max_sweeps: int = 100000) -> torch.Tensor:
    """Marker watershed of ``elev`` ([H, W] or [D, H, W] fp32, device) with 4/6-connectivity as the
    parallel minimax-path fixpoint of ``em_watershed.hip`` (skimage ``watershed(elev, markers,
    mask=mask)``; ties between basins may resolve differently from the CPU priority flood).
    Sweeps repeat until no tile changes (checked every ``check_every`` launches)."""
    global LAST_WS_SWEEPS
    max_local = WS_MAX_LOCAL if max_local is None else max_local
    check_every = WS_CHECK_EVERY if check_every is None else check_every
    dev = elev.device
    shape = tuple(elev.shape)
    D, H, W = (1,) + shape if elev.dim() == 2 else shape
    n = D * H * W
    mk = markers.to(torch.int32).contiguous()
    nmk = int(mk.max()) if mk.numel() else 0
    if nmk > _ws_max_label():
        raise ValueError(f"watershed_gpu supports up to {_ws_max_label()} markers")
    e = elev.float().contiguous()
    m = mask.to(torch.uint8).contiguous() if mask is not None else None
    key = torch.empty(n, dtype=torch.int64, device=dev)
    flags = torch.empty(n, dtype=torch.uint8, device=dev)
    changed = torch.zeros(1, dtype=torch.int32, device=dev)
    st = _native.stream(dev)
    # tile width from the marker density: wide (32) tiles when the basins are large (fewer sweeps for
    # a front spanning the volume), 16 when many small basins keep the active front sparse
    # (profiles/r06/README.md §10)
    _native.call("be_ws_set_tile", 32 if nmk * WS_WIDE_VOXELS_PER_BASIN < n else 16)
    _native.call("be_ws_init", _native.ptr(e), _native.ptr(mk), _native.ptr(m), n, _native.ptr(key), _native.ptr(flags), st)
    sweeps = 0
    if WS_ACTIVE_TILES:
        # active-tile sweeps: only tiles whose neighbourhood changed in the previous sweep run
        import ctypes

        lib = _native.hip()
        lib.be_ws_tiles.restype = ctypes.c_longlong
        nt = int(lib.be_ws_tiles(D, H, W))
        dirty = [torch.ones(nt, dtype=torch.uint8, device=dev), torch.empty(nt, dtype=torch.uint8, device=dev)]
    while sweeps < max_sweeps:
        changed.zero_()
        for _ in range(check_every):
            if WS_ACTIVE_TILES:
                _native.call("be_ws_relax_active", _native.ptr(e), _native.ptr(flags), _native.ptr(key), D, H, W, max_local,
                             _native.ptr(changed), _native.ptr(dirty[0]), _native.ptr(dirty[1]), st)
                dirty.reverse()
            else:
                _native.call("be_ws_relax", _native.ptr(e), _native.ptr(flags), _native.ptr(key), D, H, W, max_local,
                             _native.ptr(changed), st)
        sweeps += check_every
        if int(changed.item()) == 0:
            break
    LAST_WS_SWEEPS = sweeps
    out = torch.empty(shape, dtype=torch.int32, device=dev)
    _native.call("be_ws_labels", _native.ptr(key), _native.ptr(flags), n, _native.ptr(out), st)
    return out


_WS_MAX = None


def _ws_max_label() -> int:
    global _WS_MAX
    if _WS_MAX is None:
        _WS_MAX = int(_native.hip().be_ws_max_label())
    return _WS_MAX


def edt3d(mask: torch.Tensor) -> torch.Tensor:
    """Exact 3-D Euclidean distance to the nearest background voxel (scipy
    ``distance_transform_edt`` on a [D, H, W] volume, unit spacing)."""
    D, H, W = mask.shape
    dev = mask.device
    if not mask.is_cuda:
        from scipy import ndimage

        return torch.from_numpy(ndimage.distance_transform_edt(mask.cpu().numpy()).astype(np.float32))
    m = mask.to(torch.uint8).contiguous()
    dist = torch.empty(D, H, W, dtype=torch.float32, device=dev)
    tmp = torch.empty_like(dist)
    v = torch.empty(D * H * W + D * max(H, W), dtype=torch.int32, device=dev)  # tail: fallback line flags
    z = torch.empty(D * H * W + D * max(H, W), dtype=torch.float64, device=dev)
    _native.call("be_edt3d", _native.ptr(m), _native.ptr(dist), _native.ptr(tmp), _native.ptr(v), _native.ptr(z), D, H, W,
                 _native.stream(dev))
    return dist


def max_filter3d(x: torch.Tensor, r: int) -> torch.Tensor:
    """Cubic (2r+1)^3 maximum filter, nearest-edge mode (scipy ``maximum_filter(size=2r+1)``)."""
    D, H, W = x.shape
    if not x.is_cuda:
        from scipy import ndimage

        return torch.from_numpy(ndimage.maximum_filter(x.float().numpy(), size=2 * r + 1, mode="nearest"))
    a = x.float().contiguous()
    t, o = torch.empty_like(a), torch.empty_like(a)
    st = _native.stream(a.device)
    _native.call("be_max_filter_1d", _native.ptr(a), _native.ptr(t), D, H, W, r, 0, st)   # along x
    _native.call("be_max_filter_1d", _native.ptr(t), _native.ptr(o), D, H, W, r, 1, st)   # along y
    _native.call("be_max_filter_1d", _native.ptr(o), _native.ptr(t), 1, D, H * W, r, 1, st)  # along z
    return t


def peak_local_max3d(dist: torch.Tensor, closed: torch.Tensor, min_distance: int = 8) -> np.ndarray:
    """skimage ``peak_local_max(dist, min_distance, labels=closed)`` on a volume (exclude_border)."""
    D, H, W = dist.shape
    b = min_distance
    inner = torch.zeros_like(closed)
    if D > 2 * b and H > 2 * b and W > 2 * b:
        inner[b:D - b, b:H - b, b:W - b] = True
    lm = closed & inner
    img = torch.where(lm, dist, torch.full_like(dist, -3.0e38))
    mx = max_filter3d(img, min_distance)
    cand = (img == mx) & (img > float(dist.min())) & lm
    zyx = cand.nonzero()
    if zyx.shape[0] == 0:
        return np.zeros((0, 3), np.int64)
    order = torch.sort(-img[zyx[:, 0], zyx[:, 1], zyx[:, 2]], stable=True).indices
    return ensure_spacing(zyx[order].cpu().numpy(), min_distance).astype(np.int64)


def _markers_from_peaks(peaks: np.ndarray, shape, device) -> torch.Tensor:
    """One marker label per peak (peaks are >= min_distance apart, so ``measure.label`` of the
    peak image gives each its own component), numbered in raster order like ``measure.label``."""
    mk = torch.zeros(shape, dtype=torch.int32, device=device)
    if len(peaks):
        pk = np.asarray(peaks)[np.lexsort(np.asarray(peaks).T[::-1])]
        mk[tuple(torch.from_numpy(pk).to(device).T)] = torch.arange(1, len(pk) + 1, dtype=torch.int32, device=device)
    return mk


def prob_to_instances(prob: torch.Tensor, threshold: float = 0.5, min_size: int = 300, closing_radius: int = 4,
                      min_distance: int = 8, gpu_watershed: bool = True) -> np.ndarray:
    """[H, W] probability (GPU) -> int32 instance labels (numpy).  The watershed runs on the GPU
    (``gpu_watershed``) or in the C++ priority flood of the host runtime."""
    binary = remove_small_objects(prob > threshold, min_size, conn=4)
    if not bool(binary.any()):
        return np.zeros(tuple(prob.shape), np.int32)
    closed = binary_closing_disk(binary, closing_radius)
    dist = edt(closed)
    peaks = peak_local_max(dist, closed, min_distance)
    if gpu_watershed and prob.is_cuda:
        markers = _markers_from_peaks(peaks, tuple(closed.shape), prob.device)
        return watershed_gpu(-dist, markers, closed).cpu().numpy()
    m = torch.zeros_like(closed)
    if len(peaks):
        pk = torch.from_numpy(peaks).to(prob.device)
        m[pk[:, 0], pk[:, 1]] = True
    markers, _ = compact_labels(ccl(m, 8))
    return watershed((-dist).cpu().numpy(), markers.cpu().numpy(), closed.cpu().numpy(), conn=1)


def closing_per_slice(binary: torch.Tensor, r: int) -> torch.Tensor:
    """Binary closing of every z-slice with a radius-``r`` disk (the reference's 2-D ``disk(4)``
    structuring element applied slice by slice), [D, H, W] bool; GPU: ``be_morph_disk`` dilate + erode."""
    if r <= 0:
        return binary
    D, H, W = binary.shape
    if not binary.is_cuda:
        from scipy import ndimage

        yy, xx = np.mgrid[-r:r + 1, -r:r + 1]
        disk = (yy ** 2 + xx ** 2) <= r ** 2
        b = binary.cpu().numpy()
        return torch.from_numpy(np.stack([ndimage.binary_closing(b[z], structure=disk) for z in range(D)]))
    m8 = binary.to(torch.uint8).contiguous()
    st = _native.stream(binary.device)
    if MORPH_BITS and r < 64:  # bit-packed rows (be_closing_disk_bits), same result
        out = torch.empty_like(m8)
        bits = torch.empty(2 * D * H * ((W + 63) // 64), dtype=torch.int64, device=binary.device)
        _native.call("be_closing_disk_bits", _native.ptr(m8), _native.ptr(out), _native.ptr(bits), D, H, W, r, 0, st)
        return out.bool()
    tmp, out = torch.empty_like(m8), torch.empty_like(m8)
    _native.call("be_morph_disk", _native.ptr(m8), _native.ptr(tmp), D, H, W, r, 0, 0, st)
    _native.call("be_morph_disk", _native.ptr(tmp), _native.ptr(out), D, H, W, r, 1, 0, st)
    return out.bool()


def peak_candidates3d(dist: torch.Tensor, closed: torch.Tensor, min_distance: int, z_lo: int, z_hi: int,
                      z_global0: int, Z_global: int, floor: float) -> tuple[np.ndarray, np.ndarray]:
    """Local-maximum candidates of :func:`peak_local_max3d` BEFORE the min-distance thinning, for a
    z-window of a larger volume: ``dist``/``closed`` cover global slices [z_global0, z_global0 + D);
    only candidates with local z in [z_lo, z_hi) are returned, as (global zyx [n, 3], values [n]) in
    raster order.  The border exclusion uses the GLOBAL volume extent."""
    D, H, W = dist.shape
    b = min_distance
    inner = torch.zeros_like(closed)
    if Z_global > 2 * b and H > 2 * b and W > 2 * b:
        za = max(0, b - z_global0)
        zb = min(D, Z_global - b - z_global0)
        if zb > za:
            inner[za:zb, b:H - b, b:W - b] = True
    lm = closed & inner
    img = torch.where(lm, dist, torch.full_like(dist, -3.0e38))
    mx = max_filter3d(img, min_distance)
    cand = (img == mx) & (img > floor) & lm
    cand[:z_lo] = False
    cand[z_hi:] = False
    zyx = cand.nonzero()
    if zyx.shape[0] == 0:
        return np.zeros((0, 3), np.int64), np.zeros(0, np.float32)
    vals = img[zyx[:, 0], zyx[:, 1], zyx[:, 2]].float().cpu().numpy()
    zyx = zyx.cpu().numpy().astype(np.int64)
    zyx[:, 0] += z_global0
    return zyx, vals


def _stage(timings, name, t0, dev):
    if timings is None:
        return t0
    import time

    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t = time.perf_counter()
    timings[name] = round(timings.get(name, 0.0) + (t - t0), 4)
    return t


def prob_to_instances_3d(mask: torch.Tensor, min_size: int = 300, closing_radius: int = 4, min_distance: int = 8,
                         gpu_watershed: bool = True, timings: dict | None = None) -> tuple[torch.Tensor, int]:
    """Foreground volume [D, H, W] (bool, GPU) -> (int32 instance labels, count): the 3-D form of
    the reference post-processing -- remove components under ``min_size`` voxels (6-connected),
    binary closing with a disk per z-slice, 3-D EDT, 3-D peak_local_max, marker watershed on
    -EDT (6-connected) -- so touching objects are split instead of merged by plain CCL."""
    import time

    from .volume import ccl3d

    dev = mask.device
    t = time.perf_counter()
    roots = ccl3d(mask)
    binary = _keep_large(roots, min_size)
    t = _stage(timings, "remove_small", t, dev)
    if not bool(binary.any()):
        return torch.zeros(mask.shape, dtype=torch.int32, device=dev), 0
    D, H, W = binary.shape
    closed = closing_per_slice(binary, closing_radius)
    t = _stage(timings, "closing", t, dev)
    dist = edt3d(closed)
    t = _stage(timings, "edt3d", t, dev)
    peaks = peak_local_max3d(dist, closed, min_distance)
    t = _stage(timings, "peaks", t, dev)
    markers = _markers_from_peaks(peaks, (D, H, W), dev)
    t = _stage(timings, "markers", t, dev)
    if gpu_watershed and mask.is_cuda:
        labels = watershed_gpu(-dist, markers, closed)
    else:
        labels = torch.from_numpy(watershed((-dist).cpu().numpy(), markers.cpu().numpy(), closed.cpu().numpy(), conn=1)).to(dev)
    _stage(timings, "watershed", t, dev)
    if timings is not None and gpu_watershed:
        timings["ws_sweeps"] = LAST_WS_SWEEPS
    return labels, int(len(peaks))


def prob_to_instances_cpu(prob: np.ndarray) -> np.ndarray:
    """CPU path (scipy + the C++ runtime) of the same post-processing definition."""
    from scipy import ndimage


    binary = prob > 0.5
    lab, n = ndimage.label(binary)
    sizes = np.bincount(lab.ravel())
    binary = binary & (sizes[lab] >= 300) & (lab > 0)
    if not binary.any():
        return np.zeros(prob.shape, np.int32)
    r = 4
    yy, xx = np.mgrid[-r:r + 1, -r:r + 1]
    closed = ndimage.binary_closing(binary, structure=(yy ** 2 + xx ** 2) <= r * r)
    dist = ndimage.distance_transform_edt(closed).astype(np.float32)
    img = np.where(closed, dist, -3.0e38).astype(np.float32)
    img[:8, :] = img[-8:, :] = -3.0e38
    img[:, :8] = img[:, -8:] = -3.0e38
    mx = ndimage.maximum_filter(img, size=17, mode="nearest")
    cand = np.argwhere((img == mx) & (img > dist.min()))
    cand = cand[np.argsort(-img[tuple(cand.T)], kind="stable")]
    peaks = ensure_spacing(cand, 8)
    m = np.zeros(prob.shape, bool)
    if len(peaks):
        m[tuple(peaks.T)] = True
    markers, _ = ndimage.label(m, structure=np.ones((3, 3)))
    return watershed(-dist, markers, closed)


def region_properties(labels: np.ndarray, pixel_size_nm: float, device=None) -> dict:
    """regionprops subset: label, area_um2, aspect_ratio (major/minor), eccentricity, centroid."""
    n = int(labels.max()) if labels.size else 0
    props = {"label": [], "area_um2": [], "aspect_ratio": [], "eccentricity": [], "centroid_y": [], "centroid_x": []}
    if n == 0:
        return props
    dev = torch.device(device) if device is not None else (torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
    lab = torch.from_numpy(labels.astype(np.int32)).to(dev)
    H, W = labels.shape
    if dev.type == "cuda":
        mom = torch.zeros(n + 1, 6, dtype=torch.float64, device=dev)
        _native.call("be_label_moments", _native.ptr(lab), 1, H, W, n + 1, _native.ptr(mom), _native.stream(dev))
        mom = mom.cpu().numpy()
    else:
        yy, xx = np.mgrid[0:H, 0:W]
        l = labels.ravel()
        mom = np.zeros((n + 1, 6))
        for j, v in enumerate((np.ones(l.size), yy.ravel(), xx.ravel(), yy.ravel() ** 2.0, xx.ravel() ** 2.0,
                               (xx * yy).ravel())):
            mom[:, j] = np.bincount(l, weights=v, minlength=n + 1)[: n + 1]
    um = pixel_size_nm / 1000.0
    for lb in range(1, n + 1):
        c, sy, sx, syy, sxx, sxy = mom[lb]
        if c == 0:
            continue
        cy, cx = sy / c, sx / c
        vy, vx, cov = syy / c - cy * cy, sxx / c - cx * cx, sxy / c - cx * cy
        tr, det = vx + vy, vx * vy - cov * cov
        disc = math.sqrt(max(tr * tr / 4 - det, 0.0))
        l1, l2 = tr / 2 + disc, max(tr / 2 - disc, 0.0)
        major, minor = 4 * math.sqrt(max(l1, 0.0)), 4 * math.sqrt(l2)
        props["label"].append(lb)
        props["area_um2"].append(float(c) * um ** 2)
        props["aspect_ratio"].append(float(major / (minor + 1e-6)))
        props["eccentricity"].append(float(math.sqrt(1 - l2 / l1)) if l1 > 0 else 0.0)
        props["centroid_y"].append(float(cy))
        props["centroid_x"].append(float(cx))
    return props
