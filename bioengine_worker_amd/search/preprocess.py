"""GPU pre-processing for DINOv2 embedding (kernels in ``csrc/kernels/imageproc.hip``).

``batch_to_dinov2`` reproduces, for a whole batch of crops at once, the reference per-image chain
``to_rgb_uint8`` (per-channel 1-99 percentile stretch to uint8, Cell-Painting AGP/ER/DNA -> RGB
mapping) followed by ``to_dinov2_tensor`` (PIL bicubic resize to 224, /255, ImageNet mean/std)
(reference apps/cell-image-search/normalizer.py:32-153).  The oracle is
:mod:`bioengine_worker_amd.search.reference` (numpy + PIL).
"""
from __future__ import annotations

import math
from functools import lru_cache

import numpy as np
import torch

from ..ops import _native
from . import reference as ref


def _bicubic(x: float, a: float = -0.5) -> float:
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1.0
    if x < 2.0:
        return (((x - 5.0) * x + 8.0) * x - 4.0) * a
    return 0.0


@lru_cache(maxsize=64)
def pil_bicubic_coeffs(in_len: int, out_len: int):
    """PIL ``precompute_coeffs`` for the bicubic filter: (weights [out, K] f32, start [out] i32)."""
    scale = in_len / out_len
    fs = max(scale, 1.0)
    support = 2.0 * fs
    K = int(math.ceil(support)) * 2 + 1
    W = np.zeros((out_len, K), np.float64)
    S = np.zeros(out_len, np.int32)
    for xx in range(out_len):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_len) - xmin
        ws = [_bicubic((x + xmin - center + 0.5) / fs) for x in range(xmax)]
        tot = sum(ws)
        if tot != 0:
            ws = [w / tot for w in ws]
        W[xx, :xmax] = ws
        S[xx] = xmin
    return W.astype(np.float32), S


def percentiles(planes: torch.Tensor, qs=(1.0, 99.0)) -> list[torch.Tensor]:
    """np.percentile('linear') of each row of planes [R, n] (float32), via one sort."""
    srt, _ = torch.sort(planes.float(), dim=1)
    n = srt.shape[1]
    out = []
    for q in qs:
        pos = q / 100.0 * (n - 1)
        lo = int(math.floor(pos))
        hi = min(lo + 1, n - 1)
        fr = pos - lo
        out.append(srt[:, lo] * (1 - fr) + srt[:, hi] * fr)
    return out


def _resample(u8: torch.Tensor, size: int) -> torch.Tensor:
    """uint8 [P, h, w] -> [P, size, size] with PIL's two-pass bicubic (horizontal first)."""
    P, h, w = u8.shape
    dev = u8.device
    st = _native.stream(dev)
    cur = u8.contiguous()
    if w != size:
        W, S = pil_bicubic_coeffs(w, size)
        Wt, St = torch.from_numpy(W).to(dev), torch.from_numpy(S).to(dev)
        out = torch.empty(P, h, size, dtype=torch.uint8, device=dev)
        _native.call("be_resample_u8", _native.ptr(cur), P, h, w, h, size, _native.ptr(Wt), _native.ptr(St), W.shape[1],
                     1, _native.ptr(out), st)
        cur = out
    if h != size:
        W, S = pil_bicubic_coeffs(h, size)
        Wt, St = torch.from_numpy(W).to(dev), torch.from_numpy(S).to(dev)
        out = torch.empty(P, size, size, dtype=torch.uint8, device=dev)
        _native.call("be_resample_u8", _native.ptr(cur), P, h, size, size, size, _native.ptr(Wt), _native.ptr(St),
                     W.shape[1], 0, _native.ptr(out), st)
        cur = out
    return cur


def batch_to_dinov2(crops: torch.Tensor, rgb_channels=None, plow: float = 1.0, phigh: float = 99.0,
                    size: int = 224, return_u8: bool = False):
    """crops [n, h, w, C] (any numeric dtype, GPU) -> bf16 [n, 3, size, size] ImageNet-normalised.
    ``return_u8`` also returns the stretched, resized uint8 RGB [n, 3, size, size] -- the reference's
    query thumbnail (``to_rgb_uint8`` + PIL bicubic resize to 224, reference main.py:1392-1397)."""
    n, h, w, C = crops.shape
    dev = crops.device
    if not crops.is_cuda:
        arr = crops.cpu().numpy()
        rgbs = [ref.to_rgb_uint8(a, rgb_channels, plow, phigh) for a in arr]
        out = torch.from_numpy(np.stack([ref.to_dinov2_array(r, size) for r in rgbs])).to(torch.bfloat16)
        if not return_u8:
            return out
        from PIL import Image

        u8 = np.stack([np.asarray(Image.fromarray(r).resize((size, size), Image.BICUBIC)) for r in rgbs])
        return out, torch.from_numpy(u8).permute(0, 3, 1, 2).contiguous()
    x = crops.float().contiguous()
    cm = ref.channel_map(C, rgb_channels)
    planes = torch.stack([x[..., c] if c >= 0 else (x[..., 0] + x[..., 1]) * 0.5 for c in cm], 1)  # n,3,h,w
    lo, hi = percentiles(planes.reshape(n * 3, h * w), (plow, phigh))
    chan = torch.tensor(cm, dtype=torch.int32, device=dev)
    u8 = torch.empty(n, 3, h, w, dtype=torch.uint8, device=dev)
    st = _native.stream(dev)
    lo, hi = lo.contiguous(), hi.contiguous()
    _native.call("be_stretch_u8", _native.ptr(x), n, h, w, C, _native.ptr(chan), _native.ptr(lo), _native.ptr(hi),
                 _native.ptr(u8), st)
    if (h, w) != (size, size):
        u8 = _resample(u8.view(n * 3, h, w), size).view(n, 3, size, size)
    out = torch.empty(n, 3, size, size, dtype=torch.bfloat16, device=dev)
    _native.call("be_imagenet_norm", _native.ptr(u8), n, size, _native.ptr(out), st)
    return (out, u8) if return_u8 else out
