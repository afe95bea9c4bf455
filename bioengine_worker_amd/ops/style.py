"""Cellpose style vector + folded style shifts.

``make_style``: global average pool of the deepest NHWC feature map, L2-normalised per image
(cellpose ``make_style``).  The pooled sum is a HIP reduction (``be_nhwc_channel_sum``).

``style_shifts``: every ``batchconvstyle.full`` Linear of the decoder stacked into ONE GEMM, then
folded with the following BatchNorm into a per-(image, channel) pre-activation shift consumed by
the fused conv prologue: ``shift = (style @ W^T + b) * s + t``.
"""
from __future__ import annotations

import torch

from . import _native

_native.register_hip_signatures({"be_nhwc_channel_sum": "ppiiiiis"})


def nhwc_channel_sum(x: torch.Tensor, square: bool = False) -> torch.Tensor:
    """Sum over H, W of an NHWC tensor -> fp32 [N, C]."""
    N = x.shape[0]
    C = x.shape[-1]
    HW = x.numel() // (N * C)
    if not x.is_cuda:
        xf = x.float().reshape(N, HW, C)
        return (xf * xf if square else xf).sum(1)
    assert x.dtype == torch.bfloat16 and x.is_contiguous()
    out = torch.zeros(N, C, device=x.device, dtype=torch.float32)
    split = max(1, min(64, HW // 256))
    _native.call("be_nhwc_channel_sum", _native.ptr(x), _native.ptr(out), N, HW, C, split, int(square),
                 _native.stream(x.device))
    return out


def make_style(x: torch.Tensor) -> torch.Tensor:
    N, H, W, C = x.shape
    s = nhwc_channel_sum(x) / float(H * W)
    return s / torch.sqrt(torch.sum(s * s, dim=1, keepdim=True))


def style_shifts(style: torch.Tensor, w: torch.Tensor, b: torch.Tensor, s: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    feat = torch.addmm(b, style, w.t())
    return torch.addcmul(t, feat, s)
