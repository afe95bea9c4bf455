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

_native.register_hip_signatures({"be_nhwc_channel_sum": "ppiiiiis", "be_style_shift": "piifppppiipps"})


def nhwc_channel_sum(x: torch.Tensor, square: bool = False) -> torch.Tensor:
    """Sum over H, W of an NHWC tensor -> fp32 [N, C]."""
    N = x.shape[0]
    C = x.shape[-1]
    HW = x.numel() // (N * C)
    if not x.is_cuda:
        xf = x.float().reshape(N, HW, C)
        return (xf * xf if square else xf).sum(1)
    assert x.dtype == torch.bfloat16 and x.is_contiguous()
    split = max(1, min(64, HW // 256))
    part = torch.empty(N, split, C, device=x.device, dtype=torch.float32)
    _native.call("be_nhwc_channel_sum", _native.ptr(x), _native.ptr(part), N, HW, C, split, int(square),
                 _native.stream(x.device))
    return part.sum(1) if split > 1 else part.view(N, C)  # fixed-order reduction: run-to-run identical


def make_style(x: torch.Tensor) -> torch.Tensor:
    N, H, W, C = x.shape
    s = nhwc_channel_sum(x) / float(H * W)
    return s / torch.sqrt(torch.sum(s * s, dim=1, keepdim=True))


def style_shifts(style: torch.Tensor, w: torch.Tensor, b: torch.Tensor, s: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    feat = torch.addmm(b, style, w.t())
    return torch.addcmul(t, feat, s)


def style_and_shifts(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, s: torch.Tensor, t: torch.Tensor,
                     style_on: bool = True) -> tuple[torch.Tensor, torch.Tensor]:
    """(make_style(x), style_shifts(style or 0, w, b, s, t)) for NHWC ``x``: on the GPU the pooled sum
    is one reduction launch and everything after it ONE kernel (``be_style_shift``)."""
    N, H, W_, C = x.shape
    J = w.shape[0]
    if not x.is_cuda or C % 4 or C > 1024:
        st = make_style(x)
        return st, style_shifts(st if style_on else torch.zeros_like(st), w, b, s, t)
    sums = nhwc_channel_sum(x)
    style = torch.empty(N, C, device=x.device, dtype=torch.float32)
    shifts = torch.empty(N, J, device=x.device, dtype=torch.float32)
    _native.call("be_style_shift", _native.ptr(sums), N, C, 1.0 / float(H * W_), _native.ptr(w), _native.ptr(b),
                 _native.ptr(s), _native.ptr(t), J, int(bool(style_on)), _native.ptr(style), _native.ptr(shifts),
                 _native.stream(x.device))
    return style, shifts
