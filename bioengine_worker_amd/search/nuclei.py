"""Nucleus detection + crop extraction on the GPU (reference ingestion.py:317-387):
DNA channel percentile-stretched to uint8, Otsu threshold (skimage semantics), 8-connected
components (HIP union-find, ``be_ccl``), area/centroid reductions (``be_region_stats``), the
largest ``n_crops`` nuclei with area > 200, grid fallback when fewer than 10 are found."""
from __future__ import annotations

import numpy as np
import torch

from ..ops import _native
from . import reference as ref
from .preprocess import percentiles


def otsu_from_hist(hist: np.ndarray, mn: int) -> int:
    hist = hist.astype(np.float64)
    centers = np.arange(mn, mn + hist.size, dtype=np.float64)
    if hist.size == 1:
        return mn
    w1 = np.cumsum(hist)
    w2 = np.cumsum(hist[::-1])[::-1]
    m1 = np.cumsum(hist * centers) / np.maximum(w1, 1e-300)
    m2 = (np.cumsum((hist * centers)[::-1]) / np.maximum(w2[::-1], 1e-300))[::-1]
    var = w1[:-1] * w2[1:] * (m1[:-1] - m2[1:]) ** 2
    return int(centers[int(np.argmax(var))])


def label_components(mask: torch.Tensor) -> torch.Tensor:
    """mask bool/uint8 [B, H, W] (GPU) -> int32 root labels (-1 background)."""
    B, H, W = mask.shape
    m = mask.to(torch.uint8).contiguous()
    lab = torch.empty(B, H, W, dtype=torch.int32, device=mask.device)
    _native.call("be_ccl", _native.ptr(m), B, H, W, _native.ptr(lab), _native.stream(mask.device))
    return lab


def region_stats(lab: torch.Tensor):
    """-> (roots [K] linear index, area [K], cy [K], cx [K]) for image 0 of lab [1, H, W]."""
    B, H, W = lab.shape
    stats = torch.zeros(B * H * W, 3, dtype=torch.int64, device=lab.device)
    _native.call("be_region_stats", _native.ptr(lab), B, H, W, _native.ptr(stats), _native.stream(lab.device))
    roots = (stats[:, 0] > 0).nonzero().squeeze(1)
    s = stats[roots]
    area = s[:, 0]
    return roots, area, s[:, 1].double() / area, s[:, 2].double() / area


def nucleus_centroids(image: torch.Tensor, n_crops: int = 100, dna_channel: int = 0, min_area: int = 200):
    """image [H, W, C] (GPU) -> [(cy, cx)] of the largest nuclei (area > min_area), sorted by area."""
    dna = image[..., dna_channel].float()
    H, W = dna.shape
    lo, hi = percentiles(dna.reshape(1, -1), (1.0, 99.0))
    lo, hi = float(lo), float(hi)
    if hi <= lo:
        hi = lo + 1.0
    dn = (((dna - lo) / (hi - lo)).clamp(0, 1) * 255.0).to(torch.uint8)
    mn = int(dn.min())
    hist = torch.bincount((dn.reshape(-1).long() - mn), minlength=1).cpu().numpy()
    thr = otsu_from_hist(hist, mn)
    lab = label_components((dn > thr)[None])
    roots, area, cy, cx = region_stats(lab)
    keep = area > min_area
    roots, area, cy, cx = roots[keep], area[keep], cy[keep], cx[keep]
    # area descending, ties in raster order of the component's first pixel (= root index)
    order = np.lexsort((roots.cpu().numpy(), -area.cpu().numpy()))[:n_crops]
    cy, cx = cy.cpu().numpy()[order], cx.cpu().numpy()[order]
    return [(int(a), int(b)) for a, b in zip(cy, cx)]


def extract_cell_crops(image: torch.Tensor, crop_size: int = 224, n_crops: int = 100, dna_channel: int = 0):
    """image [H, W, C] tensor (GPU: HIP path, CPU: numpy oracle) -> crops [k, crop, crop, C] tensor."""
    if image.dim() == 2:
        image = image[..., None]
    H, W = image.shape[:2]
    if not image.is_cuda:
        crops = ref.extract_cell_crops(image.numpy(), crop_size, n_crops, dna_channel)
        return torch.from_numpy(np.stack(crops)) if crops else image.new_zeros((0, crop_size, crop_size, image.shape[2]))
    try:
        cents = nucleus_centroids(image, n_crops, dna_channel)
    except Exception:  # noqa: BLE001
        cents = []
    if len(cents) < 10:
        cents = ref.grid_centroids(H, W, crop_size, n_crops)
    half = crop_size // 2
    cents = [(y, x) for y, x in cents[:n_crops] if y - half >= 0 and x - half >= 0 and y - half + crop_size <= H
             and x - half + crop_size <= W]
    if not cents:
        return image.new_zeros((0, crop_size, crop_size, image.shape[2]))
    ys = torch.tensor([c[0] - half for c in cents], device=image.device)
    xs = torch.tensor([c[1] - half for c in cents], device=image.device)
    ar = torch.arange(crop_size, device=image.device)
    yy = (ys[:, None] + ar[None, :])[:, :, None]
    xx = (xs[:, None] + ar[None, :])[:, None, :]
    if image.dtype == torch.uint16:  # no uint16 gather kernel in torch: move the bits as int16
        return image.view(torch.int16)[yy, xx].view(torch.uint16)
    return image[yy, xx]
