"""CPU oracle of the Cellpose mask-recovery algorithm (numpy / torch-CPU).

Re-derived from the Cellpose algorithm (cellpose 3.x ``dynamics.compute_masks``, EXT — the
reference reaches it through ``model.eval(..., niter, flow_threshold, cellprob_threshold)`` in
``apps/cellpose-finetuning/main.py:3559-3567,4998-5027`` and the model-runner cellpose pin,
SURVEY.md §2.5 K2-K7).  The HIP kernels in ``csrc/kernels/cellpose_*.hip`` implement the same
semantics; this module is what their tests compare against.

Stages
------
normalize99      per-channel 1st/99th percentile scaling (linear-interpolated percentiles)
make_tiles       224x224 tiles with 10 % overlap over an image padded to a multiple of 16 (+8 margin)
average_tiles    tapered-mask weighted blend of tile outputs
follow_flows     niter Euler steps along dP (bilinear, grid_sample align_corners=False semantics)
get_masks        histogram of end points -> 5x5 max seeds (count > 10) -> 5x 3x3 dilation in 11x11
                 windows over histogram support (> 2) -> per-pixel label, drop masks > 40 % of image
masks_to_flows   per-mask heat diffusion from the median-nearest pixel, gradient of log(1 + T)
flow QC          mean squared error between mask flows and dP/5 per mask; drop masks above threshold
fill_holes       drop masks smaller than min_size, fill holes, renumber
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F
from scipy import ndimage

# ------------------------------------------------------------------ normalization / tiling


def normalize99(img: np.ndarray, lower: float = 1.0, upper: float = 99.0) -> np.ndarray:
    """img [C, H, W] -> float32, each channel mapped so its p1 -> 0 and p99 -> 1."""
    out = np.zeros(img.shape, np.float32)
    for c in range(img.shape[0]):
        x = img[c].astype(np.float32)
        lo, hi = np.percentile(x, lower), np.percentile(x, upper)
        if hi - lo > 1e-3:
            out[c] = (x - lo) / (hi - lo)
        else:
            out[c] = 0.0 if np.ptp(x) == 0 else x - lo
    return out


def pad_amounts(L: int, div: int = 16, extra: int = 1) -> tuple[int, int]:
    lpad = int(div * math.ceil(L / div) - L)
    a = extra * div // 2 + lpad // 2
    b = extra * div // 2 + lpad - lpad // 2
    return a, b


def tile_starts(L: int, bsize: int = 224, overlap: float = 0.1) -> list[int]:
    overlap = min(0.5, max(0.05, overlap))
    b = min(bsize, L)
    n = 1 if L <= bsize else int(math.ceil((1.0 + 2 * overlap) * L / bsize))
    return [int(v) for v in np.linspace(0, L - b, n).astype(int)]


def taper_mask(ly: int = 224, lx: int = 224, sig: float = 7.5) -> np.ndarray:
    bsize = max(224, max(ly, lx))
    xm = np.arange(bsize)
    xm = np.abs(xm - xm.mean())
    mask = 1 / (1 + np.exp((xm - (bsize / 2 - 20)) / sig))
    mask = mask * mask[:, np.newaxis]
    return mask[bsize // 2 - ly // 2: bsize // 2 - ly // 2 + ly, bsize // 2 - lx // 2: bsize // 2 - lx // 2 + lx].astype(np.float32)


def make_tiles(img: np.ndarray, bsize: int = 224, overlap: float = 0.1):
    """img [C, Ly, Lx] (already padded) -> tiles [nt, C, by, bx], ystart, xstart."""
    C, Ly, Lx = img.shape
    ys, xs = tile_starts(Ly, bsize, overlap), tile_starts(Lx, bsize, overlap)
    by, bx = min(bsize, Ly), min(bsize, Lx)
    tiles = np.stack([img[:, y: y + by, x: x + bx] for y in ys for x in xs])
    return tiles, ys, xs


def average_tiles(y: np.ndarray, ys, xs, Ly: int, Lx: int) -> np.ndarray:
    """y [nt, nout, by, bx] -> [nout, Ly, Lx] tapered weighted average."""
    nt, nout, by, bx = y.shape
    acc = np.zeros((nout, Ly, Lx), np.float32)
    nrm = np.zeros((Ly, Lx), np.float32)
    mask = taper_mask(by, bx)
    k = 0
    for yy in ys:
        for xx in xs:
            acc[:, yy: yy + by, xx: xx + bx] += y[k] * mask
            nrm[yy: yy + by, xx: xx + bx] += mask
            k += 1
    return acc / nrm


# ------------------------------------------------------------------ dynamics


def follow_flows(dP: np.ndarray, cellprob: np.ndarray, cellprob_threshold: float = 0.0, niter: int = 200):
    """Returns (p_final [2, npts] float32 (y, x), inds (y, x) arrays)."""
    fg = cellprob > cellprob_threshold
    inds = np.nonzero(fg)
    Ly, Lx = cellprob.shape
    flow = torch.from_numpy((dP * fg / 5.0).astype(np.float32))
    p = torch.from_numpy(np.stack(inds).astype(np.float32))  # [2, n] (y, x)
    if p.shape[1] == 0:
        return p.numpy(), inds
    # grid_sample with align_corners=False at normalised coords 2p/(L-1)-1 samples pixel
    # position p*L/(L-1) - 0.5; each step adds the sampled flow in pixel units, clamped to [0, L-1].
    im = flow[[1, 0]].unsqueeze(0)  # (x, y) channel order as grid_sample expects
    pt = torch.zeros(1, 1, p.shape[1], 2)
    for t in range(niter):
        pt[0, 0, :, 0] = 2 * p[1] / (Lx - 1) - 1
        pt[0, 0, :, 1] = 2 * p[0] / (Ly - 1) - 1
        d = F.grid_sample(im, pt, align_corners=False)[0, :, 0, :]  # [2 (x,y), n]
        p[1] = torch.clamp(p[1] + d[0], 0, Lx - 1)
        p[0] = torch.clamp(p[0] + d[1], 0, Ly - 1)
    return p.numpy(), inds


def get_masks(p: np.ndarray, inds, shape, rpad: int = 20, max_size_fraction: float = 0.4) -> np.ndarray:
    Ly, Lx = shape
    M0 = np.zeros(shape, np.int32)
    if p.shape[1] == 0:
        return M0
    pt = p.astype(np.int64) + rpad  # truncation (p >= 0)
    pt[0] = np.clip(pt[0], 0, Ly + rpad - 1)
    pt[1] = np.clip(pt[1], 0, Lx + rpad - 1)
    hs = (Ly + 2 * rpad, Lx + 2 * rpad)
    h1 = np.zeros(hs, np.int32)
    np.add.at(h1, (pt[0], pt[1]), 1)
    hmax = ndimage.maximum_filter(h1, size=5, mode="constant", cval=0)
    seeds = np.argwhere((h1 >= hmax) & (h1 > 10))
    if len(seeds) == 0:
        return M0
    npts = h1[seeds[:, 0], seeds[:, 1]]
    lin = seeds[:, 0] * hs[1] + seeds[:, 1]
    order = np.lexsort((lin, npts))  # ascending count, ties by raster index
    seeds = seeds[order]
    M1 = np.zeros(hs, np.int32)
    for k, (sy, sx) in enumerate(seeds):
        win = h1[sy - 5: sy + 6, sx - 5: sx + 6] > 2
        sm = np.zeros((11, 11), bool)
        sm[5, 5] = True
        for _ in range(5):
            sm = ndimage.binary_dilation(sm, structure=np.ones((3, 3), bool)) & win
        yy, xx = np.nonzero(sm)
        M1[yy + sy - 5, xx + sx - 5] = k + 1
    M0[inds] = M1[pt[0], pt[1]]
    # remove big masks, renumber
    big = Ly * Lx * max_size_fraction
    labels, counts = np.unique(M0, return_counts=True)
    for lab, c in zip(labels, counts):
        if lab != 0 and c > big:
            M0[M0 == lab] = 0
    return renumber(M0)


def renumber(M: np.ndarray) -> np.ndarray:
    labs = np.unique(M)
    labs = labs[labs != 0]
    lut = np.zeros(int(M.max()) + 1 if M.size else 1, np.int32)
    lut[labs] = np.arange(1, len(labs) + 1)
    return lut[M]


def mask_centers(masks: np.ndarray) -> np.ndarray:
    """Per-mask pixel nearest the (y, x) median, padded coordinates (+1).  [nmask, 2]"""
    n = int(masks.max())
    centers = np.zeros((n, 2), np.int64)
    for i, sl in enumerate(ndimage.find_objects(masks)):
        if sl is None:
            continue
        yi, xi = np.nonzero(masks[sl] == i + 1)
        ymed, xmed = np.median(yi), np.median(xi)
        imin = np.argmin((xi - xmed) ** 2 + (yi - ymed) ** 2)
        centers[i] = (yi[imin] + sl[0].start + 1, xi[imin] + sl[1].start + 1)
    return centers


def masks_to_flows(masks: np.ndarray, niter: int | None = None) -> np.ndarray:
    """Unit flow field [2, Ly, Lx] (dy, dx) from heat diffusion inside each mask."""
    Ly, Lx = masks.shape
    mu0 = np.zeros((2, Ly, Lx), np.float32)
    if masks.max() == 0:
        return mu0
    mp = np.pad(masks, 1)
    slices = ndimage.find_objects(masks)
    ext = [(sl[0].stop - sl[0].start + 1) + (sl[1].stop - sl[1].start + 1) for sl in slices if sl is not None]
    n_iter = 2 * max(ext) if niter is None else niter
    centers = mask_centers(masks)
    y, x = np.nonzero(mp)
    dy9 = np.array([0, -1, 1, 0, 0, -1, -1, 1, 1])
    dx9 = np.array([0, 0, 0, -1, 1, -1, 1, -1, 1])
    ny = y[None, :] + dy9[:, None]
    nx = x[None, :] + dx9[:, None]
    isn = mp[ny, nx] == mp[y, x][None, :]
    T = np.zeros(mp.shape, np.float64)
    valid = centers[:, 0] > 0
    cy, cx = centers[valid, 0], centers[valid, 1]
    for _ in range(n_iter):
        T[cy, cx] += 1
        Tn = T[ny, nx] * isn
        T[y, x] = Tn.mean(axis=0)
    T = np.log(1.0 + T)
    dy = T[y + 1, x] - T[y - 1, x]
    dx = T[y, x + 1] - T[y, x - 1]
    mu = np.stack([dy, dx])
    mu /= 1e-60 + np.sqrt((mu ** 2).sum(0))
    mu0[:, y - 1, x - 1] = mu
    return mu0


def flow_errors(masks: np.ndarray, dP: np.ndarray) -> np.ndarray:
    mu = masks_to_flows(masks)
    n = int(masks.max())
    err = np.zeros(n, np.float64)
    for c in range(2):
        err += ndimage.mean((mu[c] - dP[c] / 5.0) ** 2, masks, index=np.arange(1, n + 1))
    return err


def remove_bad_flow_masks(masks: np.ndarray, dP: np.ndarray, threshold: float = 0.4) -> np.ndarray:
    err = flow_errors(masks, dP)
    bad = 1 + np.nonzero(err > threshold)[0]
    out = masks.copy()
    out[np.isin(out, bad)] = 0
    return out


def fill_holes_and_remove_small_masks(masks: np.ndarray, min_size: int = 15) -> np.ndarray:
    out = np.zeros_like(masks)
    j = 0
    for i, sl in enumerate(ndimage.find_objects(masks)):
        if sl is None:
            continue
        msk = masks[sl] == i + 1
        npix = msk.sum()
        if min_size > 0 and npix < min_size:
            continue
        if npix > 0:
            filled = ndimage.binary_fill_holes(msk)
            # hole pixels are claimed only where no other mask lives (order-independent form)
            claim = filled & ((masks[sl] == 0) | msk)
            out[sl][claim] = j + 1
            j += 1
    return out


def compute_masks(dP, cellprob, niter=200, cellprob_threshold=0.0, flow_threshold=0.4, min_size=15,
                  max_size_fraction=0.4) -> np.ndarray:
    p, inds = follow_flows(dP, cellprob, cellprob_threshold, niter)
    mask = get_masks(p, inds, cellprob.shape, max_size_fraction=max_size_fraction)
    if mask.max() > 0 and flow_threshold is not None and flow_threshold > 0:
        mask = remove_bad_flow_masks(mask, dP, flow_threshold)
    return fill_holes_and_remove_small_masks(mask, min_size)
