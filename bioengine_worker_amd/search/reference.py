"""CPU oracle of the cell-image-search pre-processing (numpy + PIL), mirroring the reference's
normalizer.py:32-153 and ingestion.py:317-387 semantics.  Used by tests and as the CPU path."""
from __future__ import annotations

import numpy as np

IMAGENET_MEAN = np.array([0.485, 0.456, 0.406], np.float32)
IMAGENET_STD = np.array([0.229, 0.224, 0.225], np.float32)
JUMP_CH_DNA, JUMP_CH_ER, JUMP_CH_RNA, JUMP_CH_AGP, JUMP_CH_MITO = 0, 1, 2, 3, 4


def percentile_stretch(img: np.ndarray, plow: float = 1.0, phigh: float = 99.0) -> np.ndarray:
    lo, hi = np.percentile(img, plow), np.percentile(img, phigh)
    if hi <= lo:
        hi = lo + 1.0
    t = (img.astype(np.float32) - lo) / (hi - lo)
    return (np.clip(t, 0.0, 1.0) * 255.0).astype(np.uint8)


def channel_map(n_ch: int, rgb_channels=None) -> list[int]:
    """Source channel per RGB output; -1 means (ch0 + ch1) / 2 (two-channel images)."""
    if rgb_channels is not None:
        return list(rgb_channels)
    if n_ch == 1:
        return [0, 0, 0]
    if n_ch == 2:
        return [0, 1, -1]
    if n_ch == 3 or n_ch == 4:
        return [0, 1, 2]
    return [JUMP_CH_AGP, JUMP_CH_ER, JUMP_CH_DNA]


def to_hwc(img: np.ndarray) -> np.ndarray:
    if img.ndim == 3 and img.shape[0] <= 7 and img.shape[0] < img.shape[2]:
        img = np.moveaxis(img, 0, -1)
    if img.ndim == 2:
        img = img[..., None]
    return img


def to_rgb_uint8(img: np.ndarray, rgb_channels=None, plow: float = 1.0, phigh: float = 99.0) -> np.ndarray:
    img = to_hwc(img)
    cm = channel_map(img.shape[-1], rgb_channels)
    out = np.zeros(img.shape[:2] + (3,), np.uint8)
    for c, sc in enumerate(cm):
        src = img[..., sc] if sc >= 0 else (img[..., 0].astype(np.float32) + img[..., 1]) / 2
        out[..., c] = percentile_stretch(src, plow, phigh)
    return out


def to_dinov2_array(img_rgb_uint8: np.ndarray, size: int = 224) -> np.ndarray:
    from PIL import Image

    pil = Image.fromarray(img_rgb_uint8, mode="RGB").resize((size, size), Image.BICUBIC)
    arr = np.asarray(pil, dtype=np.float32) / 255.0
    return ((arr - IMAGENET_MEAN) / IMAGENET_STD).transpose(2, 0, 1)


def otsu_threshold_u8(img: np.ndarray) -> int:
    """skimage.filters.threshold_otsu on an integer image (histogram over [min, max])."""
    v = img.ravel().astype(np.int64)
    mn = int(v.min())
    hist = np.bincount(v - mn).astype(np.float64)
    centers = np.arange(mn, mn + hist.size, dtype=np.float64)
    if hist.size == 1:
        return mn
    w1 = np.cumsum(hist)
    w2 = np.cumsum(hist[::-1])[::-1]
    m1 = np.cumsum(hist * centers) / np.maximum(w1, 1e-300)
    m2 = (np.cumsum((hist * centers)[::-1]) / np.maximum(w2[::-1], 1e-300))[::-1]
    var = w1[:-1] * w2[1:] * (m1[:-1] - m2[1:]) ** 2
    return int(centers[int(np.argmax(var))])


def label8(mask: np.ndarray) -> np.ndarray:
    """8-connected components, labels 1..n in raster order of each component's first pixel."""
    from scipy import ndimage

    lab, n = ndimage.label(mask, structure=np.ones((3, 3), int))
    # ndimage numbers components in raster order of first pixel as well
    return lab


def nucleus_centroids(image: np.ndarray, n_crops: int = 100, dna_channel: int = 0, min_area: int = 200):
    img = to_hwc(image)
    dna = img[..., dna_channel].astype(np.float32)
    dn = percentile_stretch(dna)
    mask = dn > otsu_threshold_u8(dn)
    lab = label8(mask)
    n = int(lab.max())
    if n == 0:
        return []
    idx = np.arange(1, n + 1)
    from scipy import ndimage

    area = ndimage.sum(np.ones_like(lab), lab, idx)
    cy, cx = np.array(ndimage.center_of_mass(np.ones_like(lab), lab, idx)).T
    keep = [i for i in range(n) if area[i] > min_area]
    keep.sort(key=lambda i: -area[i])
    return [(int(cy[i]), int(cx[i])) for i in keep[:n_crops]]


def grid_centroids(H: int, W: int, crop_size: int, n_crops: int):
    half = crop_size // 2
    stride = max(crop_size, min(H, W) // max(1, int(np.sqrt(n_crops))))
    return [(y + half, x + half) for y in range(half, H - half, stride) for x in range(half, W - half, stride)][:n_crops]


def crops_at(image: np.ndarray, centroids, crop_size: int = 224):
    img = to_hwc(image)
    H, W = img.shape[:2]
    half = crop_size // 2
    out = []
    for cy, cx in centroids:
        y0, x0 = cy - half, cx - half
        if y0 < 0 or x0 < 0 or y0 + crop_size > H or x0 + crop_size > W:
            continue
        out.append(img[y0:y0 + crop_size, x0:x0 + crop_size])
    return out


def extract_cell_crops(image: np.ndarray, crop_size: int = 224, n_crops: int = 100, dna_channel: int = 0):
    img = to_hwc(image)
    H, W = img.shape[:2]
    try:
        cents = nucleus_centroids(img, n_crops, dna_channel)
    except Exception:  # noqa: BLE001
        cents = []
    if len(cents) < 10:
        cents = grid_centroids(H, W, crop_size, n_crops)
    return crops_at(img, cents[:n_crops], crop_size)
