"""Two-group ping-pong 256 x 256 bf16 GEMM (``csrc/kernels/gemm_8p.hip``): the forward (``x W^T``)
layout with the bias / bias+GELU / bias+residual epilogues of :mod:`.gemm_mt`, for the Cellpose-SAM
linear layers.  On CPU every helper is the fp32 PyTorch op of the same math."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _native

E_NONE, E_BIAS, E_BIAS_GELU, E_BIAS_RES = 0, 1, 2, 6


def supported(M: int, N: int, K: int, lda: int | None = None) -> bool:
    return K % 64 == 0 and N % 4 == 0 and M * (lda or K) < 2 ** 32 and N * K < 2 ** 32


def _ok(*ts) -> bool:
    return all(t is None or (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous()) for t in ts)


def _bias(b):
    if b is None:
        return None, 0
    b = b.contiguous()
    if b.dtype == torch.bfloat16:
        return b, 1
    return b.float(), 0


def _call(x, w, C, C2, b, aux, epi):
    M, K = x.shape
    N = w.shape[0]
    bb, bf = _bias(b)
    _native.call("be_gemm_8p", _native.ptr(x), _native.ptr(w), _native.ptr(C), _native.ptr(C2), _native.ptr(bb), bf,
                 _native.ptr(aux), M, N, K, K, K, N, epi, _native.stream(x.device))


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    """x [M, K] @ w [N, K]^T (+ b[N]) -> bf16 [M, N]."""
    M, K = x.shape
    N = w.shape[0]
    if not (x.is_cuda and _ok(x, w) and supported(M, N, K)):
        return F.linear(x, w, None if b is None else b.to(x.dtype))
    out = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    _call(x, w, out, None, b, None, E_BIAS if b is not None else E_NONE)
    return out


def linear_res(x, w, b, r):
    """x w^T + b + r -> bf16 (residual fused in the epilogue)."""
    M, K = x.shape
    N = w.shape[0]
    if not (x.is_cuda and _ok(x, w, r) and supported(M, N, K)):
        return (F.linear(x.float(), w.float(), None if b is None else b.float()) + r.float()).to(x.dtype)
    out = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    _call(x, w, out, None, b, r, E_BIAS_RES)
    return out


def linear_gelu(x, w, b):
    """-> (g = gelu(f), f = x w^T + b), both bf16; g is the erf GELU of the bf16-rounded f."""
    M, K = x.shape
    N = w.shape[0]
    if not (x.is_cuda and _ok(x, w) and supported(M, N, K)):
        f = F.linear(x.float(), w.float(), b.float()).to(x.dtype)
        return F.gelu(f.float()).to(x.dtype), f
    f = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    g = torch.empty_like(f)
    _call(x, w, f, g, b, None, E_BIAS_GELU)
    return g, f


def linear_gelu_only(x, w, b):
    """gelu(x w^T + b) bf16 (inference: the pre-activation is not stored)."""
    M, K = x.shape
    N = w.shape[0]
    if not (x.is_cuda and _ok(x, w) and supported(M, N, K)):
        return F.gelu(F.linear(x.float(), w.float(), b.float()).to(x.dtype).float()).to(x.dtype)
    g = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    _call(x, w, None, g, b, None, E_BIAS_GELU)
    return g
