"""Transformer building blocks on HIP kernels (``csrc/kernels/attention.hip``, ``layernorm.hip``).

* :func:`flash_attention` — fused MHA forward (head_dim 64) with optional SAM decomposed
  relative-position bias; differentiable (backward recomputes the probabilities from the saved
  log-sum-exp in fp32 PyTorch math — the HIP backward is future work, see docs).
* :func:`add_layernorm` — LayerScale residual update fused with the next LayerNorm.
* :func:`bias_gelu_` — bias + exact GELU on a GEMM output.

Plain GEMMs (qkv / proj / MLP) stay on hipBLASLt through ``torch.nn.functional.linear``.
Every op has a PyTorch reference (``*_ref``) used on CPU and by the numerics tests.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import _native


# ------------------------------------------------------------------ attention

def attention_ref(q, k, v, scale: float, rel_h=None, rel_w=None):
    """q, k, v: [B, N, H, D] -> [B, N, H, D] (fp32 math).  rel_h [B, H, N, Hg], rel_w [B, H, N, Wg]."""
    qf, kf, vf = (t.float().permute(0, 2, 1, 3) for t in (q, k, v))  # B H N D
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if rel_h is not None:
        B, H, N, Hg = rel_h.shape
        Wg = rel_w.shape[-1]
        bias = rel_h.float()[..., :, None] + rel_w.float()[..., None, :]  # B H N Hg Wg
        s = s + bias.reshape(B, H, N, Hg * Wg)
    p = torch.softmax(s, dim=-1)
    return torch.matmul(p, vf).permute(0, 2, 1, 3)


def _strides_ok(q, k, v):
    return (q.stride() == k.stride() == v.stride() and q.stride(-1) == 1 and q.shape[-1] == 64
            and all(t.dtype == torch.bfloat16 for t in (q, k, v)))


def _attn_fwd_hip(q, k, v, scale, rel_h, rel_w, want_lse: bool):
    B, N, H, D = q.shape
    out = torch.empty(B, N, H, D, device=q.device, dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device=q.device, dtype=torch.float32) if want_lse else None
    Hg = Wg = 0
    rh = rw = None
    if rel_h is not None:
        Hg, Wg = rel_h.shape[-1], rel_w.shape[-1]
        rh = rel_h.float().contiguous()
        rw = rel_w.float().contiguous()
    sb, st, sh = q.stride(0), q.stride(1), q.stride(2)
    _native.call("be_attn_fwd", _native.ptr(q), _native.ptr(k), _native.ptr(v), st, sh, sb,
                 _native.ptr(out), out.stride(1), out.stride(2), out.stride(0), _native.ptr(lse),
                 _native.ptr(rh), _native.ptr(rw), Hg, Wg, B, H, N, D, float(scale), 0, _native.stream(q.device))
    return out, lse


class _FlashAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale, rel_h, rel_w):
        out, lse = _attn_fwd_hip(q, k, v, scale, rel_h, rel_w, want_lse=True)
        ctx.save_for_backward(q, k, v, out, lse, rel_h if rel_h is not None else torch.empty(0),
                              rel_w if rel_w is not None else torch.empty(0))
        ctx.scale = scale
        ctx.has_rel = rel_h is not None
        return out

    @staticmethod
    def backward(ctx, go):
        q, k, v, out, lse, rel_h, rel_w = ctx.saved_tensors
        scale = ctx.scale
        qf, kf, vf = (t.float().permute(0, 2, 1, 3) for t in (q, k, v))
        of = out.float().permute(0, 2, 1, 3)
        gof = go.float().permute(0, 2, 1, 3)
        s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
        if ctx.has_rel:
            B, H, N, Hg = rel_h.shape
            s = s + (rel_h.float()[..., :, None] + rel_w.float()[..., None, :]).reshape(B, H, N, -1)
        p = torch.exp(s - lse[..., None])
        dv = torch.matmul(p.transpose(-1, -2), gof)
        dp = torch.matmul(gof, vf.transpose(-1, -2))
        delta = (gof * of).sum(-1, keepdim=True)
        ds = p * (dp - delta)
        dq = torch.matmul(ds, kf) * scale
        dk = torch.matmul(ds.transpose(-1, -2), qf) * scale
        drh = drw = None
        if ctx.has_rel:
            B, H, N, Hg = rel_h.shape
            Wg = rel_w.shape[-1]
            ds5 = ds.reshape(B, H, N, Hg, Wg)
            drh = ds5.sum(-1).to(rel_h.dtype)
            drw = ds5.sum(-2).to(rel_w.dtype)
        back = lambda t, ref: t.permute(0, 2, 1, 3).to(ref.dtype)
        return back(dq, q), back(dk, k), back(dv, v), None, drh, drw


def flash_attention(q, k, v, scale: float | None = None, rel_h=None, rel_w=None):
    """Multi-head attention.  q, k, v: [B, N, H, 64] (bf16 on GPU; views of one packed qkv buffer
    are fine).  rel_h [B, H, N, Hg] / rel_w [B, H, N, Wg]: SAM decomposed rel-pos terms (Hg*Wg == N).
    Returns [B, N, H, 64]."""
    D = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if q.is_cuda:
        if not _strides_ok(q, k, v):
            raise ValueError("flash_attention on GPU needs bf16 q/k/v with head_dim 64 and identical strides")
        if torch.is_grad_enabled() and any(t.requires_grad for t in (q, k, v, rel_h, rel_w) if t is not None):
            return _FlashAttn.apply(q, k, v, scale, rel_h, rel_w)
        return _attn_fwd_hip(q, k, v, scale, rel_h, rel_w, want_lse=False)[0]
    return attention_ref(q, k, v, scale, rel_h, rel_w).to(q.dtype).contiguous()


def flash_attention_mx(q, k, v, scale: float | None = None):
    """Multi-head attention with an MX-fp8 output for the next fp8 GEMM: returns (oq e4m3fn [B, N, H*64],
    os E8M0 uint8 [B*N, H*2]) -- one power-of-two scale per 32 head dims, quantised from the fp32
    accumulator in the kernel's epilogue (no bf16 output, no separate quantisation pass).  CPU: the
    PyTorch reference (fp32 attention, then ``mx_quantize_ref``)."""
    from .fp8 import FP8_DTYPE, mx_quantize_ref

    B, N, H, D = q.shape
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if not q.is_cuda:
        o = attention_ref(q, k, v, scale).float().reshape(B, N, H * D)
        oq, os_ = mx_quantize_ref(o)
        return oq, os_.reshape(B * N, H * D // 32)
    if not _strides_ok(q, k, v):
        raise ValueError("flash_attention_mx needs bf16 q/k/v with head_dim 64 and identical strides")
    oq = torch.empty(B, N, H * D, device=q.device, dtype=FP8_DTYPE)
    os_ = torch.empty(B * N, H * D // 32, device=q.device, dtype=torch.uint8)
    sb, st, sh = q.stride(0), q.stride(1), q.stride(2)
    _native.call("be_attn_fwd_mx", _native.ptr(q), _native.ptr(k), _native.ptr(v), st, sh, sb, _native.ptr(oq),
                 _native.ptr(os_), B, H, N, D, float(scale), _native.stream(q.device))
    return oq, os_


# ------------------------------------------------------------------ layer norm / residual

def add_layernorm_ref(x, y, gamma, w, b, eps: float = 1e-6):
    xn = x.float()
    if y is not None:
        yn = y.float() * (gamma.float() if gamma is not None else 1.0)
        xn = (xn + yn).to(x.dtype).float()
    out = F.layer_norm(xn, (x.shape[-1],), w.float() if w is not None else None, b.float() if b is not None else None,
                       eps)
    return xn.to(x.dtype), out.to(x.dtype)


def add_layernorm(x: torch.Tensor, y: torch.Tensor | None, gamma: torch.Tensor | None, w: torch.Tensor,
                  b: torch.Tensor, eps: float = 1e-6, inplace: bool = True):
    """``x <- x + gamma * y`` (in place when ``inplace``) and returns ``LN(x) * w + b``.

    Inference op (no autograd): training code composes the same math from torch ops."""
    if not x.is_cuda:
        xn, out = add_layernorm_ref(x, y, gamma, w, b, eps)
        if y is not None and inplace:
            x.copy_(xn)
        return out
    C = x.shape[-1]
    rows = x.numel() // C
    assert x.dtype == torch.bfloat16 and x.is_contiguous()
    if y is not None:
        assert y.shape == x.shape and y.dtype == torch.bfloat16
        y = y.contiguous()
    out = torch.empty_like(x)
    g = gamma.float().contiguous() if gamma is not None else None
    _native.call("be_add_layernorm", _native.ptr(x), _native.ptr(y), _native.ptr(g), _native.ptr(w.float().contiguous()),
                 _native.ptr(b.float().contiguous()), _native.ptr(out), None, rows, C, float(eps),
                 int(bool(inplace)), _native.stream(x.device))
    return out


def bias_gelu_(h: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    """In-place ``h = gelu(h + bias)`` (exact erf GELU) on a [..., C] GEMM output."""
    if not h.is_cuda:
        h.copy_(F.gelu(h.float() + bias.float()).to(h.dtype))
        return h
    C = h.shape[-1]
    assert h.dtype == torch.bfloat16 and h.is_contiguous()
    _native.call("be_bias_gelu", _native.ptr(h), _native.ptr(bias.float().contiguous()), h.numel() // C, C,
                 _native.stream(h.device))
    return h
