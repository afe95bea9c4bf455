"""EM mitochondria instance segmentation pipeline on MI355X.

Reference semantics (apps/fibsem-mito-analysis/analysis_deployment.py): percentile (1, 99)
normalisation; 512 tiles with 64 overlap, reflect-padded edge tiles, Gaussian window
``exp(-2y^2) exp(-2x^2)`` blending (:108-156); ``_prob_to_instances`` (:160-176): threshold 0.5,
``remove_small_objects(min_size=300)`` (4-connectivity), ``binary_closing(disk(4))``, EDT,
``peak_local_max(min_distance=8, labels=closed)``, ``watershed(-dist, label(peaks), mask=closed)``;
regionprops area / axis lengths / eccentricity / centroid (:256-271).

Dense stages are HIP kernels (``imageproc.hip``: CCL; ``morphology.hip``: blend, disk morphology,
EDT, max filter, moments); the priority-flood watershed and the greedy peak spacing run in the C++
host runtime (``csrc/runtime/watershed.cpp``).  skimage is not available in this image, so
exact parity with it is "unpinned": every stage is tested against scipy/numpy oracles of the same
definition (tests/test_em_*.py).
"""
from __future__ import annotations

import math
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
        _native.call("be_blend_gather", _native.ptr(probs), C, 1, H, W, 1, len(ys), len(xs), stride, 1, tile,
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


def remove_small_objects(mask: torch.Tensor, min_size: int = 300, conn: int = 4) -> torch.Tensor:
    roots = ccl(mask, conn)
    flat = roots.reshape(-1).long()
    fg = flat >= 0
    cnt = torch.zeros(flat.numel(), dtype=torch.int32, device=mask.device)
    cnt.index_add_(0, flat[fg], torch.ones(int(fg.sum()), dtype=torch.int32, device=mask.device))
    keep = torch.zeros_like(flat, dtype=torch.bool)
    keep[fg] = cnt[flat[fg]] >= min_size
    return keep.reshape(mask.shape)


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
    v = torch.empty(H, W, dtype=torch.int32, device=dev)
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


def prob_to_instances(prob: torch.Tensor, threshold: float = 0.5, min_size: int = 300, closing_radius: int = 4,
                      min_distance: int = 8) -> np.ndarray:
    """[H, W] probability (GPU) -> int32 instance labels (numpy)."""
    binary = remove_small_objects(prob > threshold, min_size, conn=4)
    if not bool(binary.any()):
        return np.zeros(tuple(prob.shape), np.int32)
    closed = binary_closing_disk(binary, closing_radius)
    dist = edt(closed)
    peaks = peak_local_max(dist, closed, min_distance)
    m = torch.zeros_like(closed)
    if len(peaks):
        pk = torch.from_numpy(peaks).to(prob.device)
        m[pk[:, 0], pk[:, 1]] = True
    markers, _ = compact_labels(ccl(m, 8))
    return watershed((-dist).cpu().numpy(), markers.cpu().numpy(), closed.cpu().numpy(), conn=1)


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
