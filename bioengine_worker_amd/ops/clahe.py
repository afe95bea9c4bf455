"""CLAHE for the Cellpose fine-tuning pre-processing.

The reference converts every training image to grayscale uint8 and applies
``cv2.createCLAHE(clipLimit=3.0, tileGridSize=(16, 16))`` (apps/cellpose-finetuning/main.py:273-308).
:func:`clahe_u8` runs the HIP kernel (``csrc/kernels/clahe.hip``) on a GPU batch; :func:`clahe_u8_ref`
is the numpy oracle of the same algorithm (OpenCV's 8-bit CLAHE: reflect-101 extension to a
multiple of the grid, clip limit ``max(1, int(clip * area / 256))``, even + strided-residual
redistribution, ``round(cumsum * 255 / area)`` LUTs, fp32 bilinear blend rounded half-even).
OpenCV is not installed in this environment, so parity with cv2 itself is unpinned; the GPU kernel
is checked bit-exactly against the oracle.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _native


def to_gray_u8(img) -> np.ndarray:
    """The reference's grayscale/uint8 conversion (main.py:281-304): CHW -> HWC when the first dim
    looks like channels, ITU-R 601 luminance for >= 3 channels, channel 0 of 1/2-channel images,
    min-max scaling with truncation for non-uint8 input."""
    a = np.asarray(img)
    if a.ndim == 3 and a.shape[0] in (1, 2, 3, 4) and a.shape[0] < a.shape[1]:
        a = a.transpose(1, 2, 0)
    if a.ndim == 3:
        if a.shape[2] >= 3:
            a = (0.299 * a[:, :, 0].astype(np.float32) + 0.587 * a[:, :, 1].astype(np.float32)
                 + 0.114 * a[:, :, 2].astype(np.float32)).astype(np.uint8)
        else:
            a = a[:, :, 0]
    if a.dtype != np.uint8:
        lo, hi = float(a.min()), float(a.max())
        if hi > lo:
            a = ((a.astype(np.float32) - lo) / (hi - lo) * 255).astype(np.uint8)
        else:
            a = np.zeros(a.shape, np.uint8)
    return np.ascontiguousarray(a)


def _reflect101(i: np.ndarray, n: int) -> np.ndarray:
    if n == 1:
        return np.zeros_like(i)
    period = 2 * n - 2
    i = np.abs(i) % period
    return np.where(i >= n, period - i, i)


def clahe_u8_ref(img: np.ndarray, clip: float = 3.0, grid: tuple[int, int] = (16, 16)) -> np.ndarray:
    """numpy oracle. img: uint8 [H, W]; grid = (tiles_x, tiles_y) as in cv2."""
    src = np.asarray(img, np.uint8)
    H, W = src.shape
    tx_n, ty_n = grid
    He = H + (ty_n - H % ty_n if H % ty_n else 0)
    We = W + (tx_n - W % tx_n if W % tx_n else 0)
    th, tw = He // ty_n, We // tx_n
    ext = src[_reflect101(np.arange(He), H)[:, None], _reflect101(np.arange(We), W)[None, :]]
    area = th * tw
    limit = max(1, int(np.float32(clip) * np.float32(area) / np.float32(256))) if clip > 0 else None
    scale = np.float32(255) / np.float32(area)
    lut = np.zeros((ty_n, tx_n, 256), np.uint8)
    for ty in range(ty_n):
        for tx in range(tx_n):
            h = np.bincount(ext[ty * th:(ty + 1) * th, tx * tw:(tx + 1) * tw].ravel(), minlength=256).astype(np.int64)
            if limit is not None:
                clipped = int(np.maximum(h - limit, 0).sum())
                h = np.minimum(h, limit)
                batch, residual = divmod(clipped, 256)
                h += batch
                if residual:
                    step = max(256 // residual, 1)
                    idx = np.arange(0, 256, step)[:residual]
                    h[idx] += 1
            c = np.cumsum(h).astype(np.float32)
            lut[ty, tx] = np.clip(np.rint(c * scale), 0, 255).astype(np.uint8)
    f32 = np.float32
    tyf = np.arange(H, dtype=f32) * (f32(1) / f32(th)) - f32(0.5)
    txf = np.arange(W, dtype=f32) * (f32(1) / f32(tw)) - f32(0.5)
    ty1 = np.floor(tyf).astype(np.int64)
    tx1 = np.floor(txf).astype(np.int64)
    ya = (tyf - ty1.astype(f32)).astype(f32)[:, None]
    xa = (txf - tx1.astype(f32)).astype(f32)[None, :]
    ty2, tx2 = np.minimum(ty1 + 1, ty_n - 1), np.minimum(tx1 + 1, tx_n - 1)
    ty1, tx1 = np.maximum(ty1, 0), np.maximum(tx1, 0)
    v = src
    l11 = lut[ty1[:, None], tx1[None, :], v].astype(f32)
    l12 = lut[ty1[:, None], tx2[None, :], v].astype(f32)
    l21 = lut[ty2[:, None], tx1[None, :], v].astype(f32)
    l22 = lut[ty2[:, None], tx2[None, :], v].astype(f32)
    xa1 = (f32(1) - xa).astype(f32)
    top = (l11 * xa1 + l12 * xa).astype(f32)
    bot = (l21 * xa1 + l22 * xa).astype(f32)
    r = (top * (f32(1) - ya) + bot * ya).astype(f32)
    return np.clip(np.rint(r), 0, 255).astype(np.uint8)


def clahe_u8(x: torch.Tensor, clip: float = 3.0, grid: tuple[int, int] = (16, 16)) -> torch.Tensor:
    """x: uint8 [H, W] or [B, H, W] (GPU: HIP kernel, one launch per batch; CPU: the oracle)."""
    squeeze = x.dim() == 2
    xb = x.unsqueeze(0) if squeeze else x
    if xb.dtype != torch.uint8:
        raise TypeError("clahe_u8 expects uint8 input (use to_gray_u8 first)")
    if not xb.is_cuda:
        out = torch.from_numpy(np.stack([clahe_u8_ref(im, clip, grid) for im in xb.numpy()]))
        return out[0] if squeeze else out
    B, H, W = xb.shape
    xb = xb.contiguous()
    out = torch.empty_like(xb)
    lut = torch.empty(B, grid[1], grid[0], 256, dtype=torch.uint8, device=xb.device)
    _native.call("be_clahe_u8", _native.ptr(xb), _native.ptr(out), _native.ptr(lut), B, H, W, int(grid[0]),
                 int(grid[1]), float(clip), _native.stream(xb.device))
    return out[0] if squeeze else out
