"""Ping-pong bf16 MFMA GEMM (``csrc/kernels/gemm_pp.hip``): large tiles, two staggered wave
groups and a 4-slot LDS-DMA ring of K-halves.  One main loop serves

* :func:`linear` / :func:`linear_gelu` -- ``x W^T (+ b)`` (and ``gelu``) for large M;
* :func:`conv3` -- the 3x3 / pad 1 conv on plain NHWC bf16 as an implicit GEMM over pixels with
  the CPnet epilogue (bias, residual, the consumer's BN + ReLU + style shift).

cfg: 0 = 256 x 256 tiles (8 waves of 128 x 64), 1 = 512 x 128, 2 = 256 x 128 (waves of 64 x 64).
On CPU every helper is the fp32 PyTorch op of the same math (the numerics oracle)."""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _native

P_NONE, P_BIAS, P_BIAS_GELU, P_DGELU = 0, 1, 2, 4
TILES = {0: (256, 256), 1: (512, 128), 2: (256, 128)}


def _forced() -> int | None:
    v = os.environ.get("BE_PP_CFG")
    return None if v is None else int(v)


def gemm_cfg(M: int, N: int) -> int:
    f = _forced()
    if f is not None:
        return f
    return 0 if N >= 256 else 2


def supported(M: int, N: int, K: int) -> bool:
    return K % 32 == 0 and N % 4 == 0 and K % 8 == 0


def _f32(b: torch.Tensor | None) -> torch.Tensor | None:
    """The epilogue reads an fp32 bias; the CPSAM engine's biases are bf16 views of its weight mirror."""
    if b is None or (b.dtype == torch.float32 and b.is_contiguous()):
        return b
    return b.float().contiguous()


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, cfg: int | None = None) -> torch.Tensor:
    """x [M, K] @ w [N, K]^T (+ b fp32 [N]) -> bf16 [M, N]."""
    M, K = x.shape
    N = w.shape[0]
    if not x.is_cuda or not supported(M, N, K) or not (x.is_contiguous() and w.is_contiguous()):
        return F.linear(x, w, None if b is None else b.to(x.dtype))
    out = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    b = _f32(b)
    _native.call("be_gemm_pp", _native.ptr(x), _native.ptr(w), _native.ptr(out), None, _native.ptr(b), None, None,
                 M, N, K, K, K, N, 0, P_BIAS if b is not None else P_NONE, gemm_cfg(M, N) if cfg is None else cfg,
                 _native.stream(x.device))
    return out


def linear_gelu(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, cfg: int | None = None):
    """-> (g = gelu(f), f = x w^T + b), both bf16; g is the GELU of the bf16-rounded f."""
    M, K = x.shape
    N = w.shape[0]
    if not x.is_cuda or not supported(M, N, K):
        f = F.linear(x.float(), w.float(), b.float()).to(x.dtype)
        return F.gelu(f.float()).to(x.dtype), f
    f = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    g = torch.empty_like(f)
    b = _f32(b)
    _native.call("be_gemm_pp", _native.ptr(x), _native.ptr(w), _native.ptr(f), _native.ptr(g), _native.ptr(b), None, None,
                 M, N, K, K, K, N, 0, P_BIAS_GELU, gemm_cfg(M, N) if cfg is None else cfg, _native.stream(x.device))
    return g, f


def _dgrad_cfg(M: int, N: int, cfg: int | None) -> int:
    if cfg is not None:
        return cfg
    f = _forced()
    if f is not None:
        return f
    return 0 if N % 256 == 0 and N >= 2048 else 2


def mm(x: torch.Tensor, w: torch.Tensor, cfg: int | None = None) -> torch.Tensor:
    """x [M, K] @ w [K, N] (the dgrad: W read as stored, transposed in LDS) -> bf16 [M, N]."""
    M, K = x.shape
    N = w.shape[1]
    c = _dgrad_cfg(M, N, cfg)
    if not x.is_cuda or not supported(M, N, K) or N % TILES[c][1] or not (x.is_contiguous() and w.is_contiguous()):
        return torch.mm(x, w)
    out = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    _native.call("be_gemm_pp", _native.ptr(x), _native.ptr(w), _native.ptr(out), None, None, None, None, M, N, K, K, N, N,
                 1, P_NONE, c, _native.stream(x.device))
    return out


def mm_dgelu(dm: torch.Tensor, w2: torch.Tensor, f: torch.Tensor, out_db: torch.Tensor | None = None,
             cfg: int | None = None) -> torch.Tensor:
    """df = gelu'(f) * (dm @ w2), dm [M, K], w2 [K, N], f [M, N]; out_db [N] fp32 = column sums of df."""
    M, K = dm.shape
    N = w2.shape[1]
    c = _dgrad_cfg(M, N, cfg)
    if not dm.is_cuda or not supported(M, N, K) or N % TILES[c][1]:
        x = f.float()
        gp = 0.5 * (1.0 + torch.erf(x * 0.7071067811865476)) + x * torch.exp(-0.5 * x * x) * 0.3989422804014327
        df = (gp * (dm.float() @ w2.float())).to(dm.dtype)
        if out_db is not None:
            torch.sum(df.float(), 0, out=out_db)
        return df
    df = torch.empty(M, N, device=dm.device, dtype=torch.bfloat16)
    if out_db is not None:
        out_db.zero_()
    _native.call("be_gemm_pp", _native.ptr(dm), _native.ptr(w2), _native.ptr(df), None, None, _native.ptr(f),
                 _native.ptr(out_db), M, N, K, K, N, N, 1, P_DGELU, c, _native.stream(dm.device))
    return df


def wgrad_split(M: int, N: int, K: int, cfg: int) -> int:
    """K slices for a [M, N] weight gradient over K tokens: enough blocks for 256 CUs while each slice
    keeps >= 16 K-halves (512 tokens)."""
    bm, bn = TILES[cfg]
    tiles = (M // bm) * (N // bn)
    split = 1
    while tiles * split < 256 and K % (64 * split) == 0 and K // (split * 2) >= 512:
        split *= 2
    return split


def wgrad(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor, cfg: int | None = None, split: int | None = None):
    """out (fp32 [n, k], in place) = dy^T x, dy [m, n], x [m, k] bf16 (both read as stored)."""
    out2 = out.view(out.shape[0], -1)
    m, n = dy.shape
    k = x.shape[1]
    c = (0 if n >= 2048 else 2) if cfg is None else cfg
    if _forced() is not None and cfg is None:
        c = _forced()
    bm, bn = TILES[c]
    if not dy.is_cuda or n % bm or k % bn or m % 32 or not (dy.is_contiguous() and x.is_contiguous()
                                                          and out2.is_contiguous()):
        torch.mm(dy.t().float(), x.float(), out=out2)
        return
    sp = wgrad_split(n, k, m, c) if split is None else split
    ws, wsb = None, 0
    if sp > 1:
        from .gemm_bf16 import _workspace

        ws = _workspace(dy.device, sp * n * k * 4)
        wsb = ws.numel()
    _native.call("be_wgrad_pp", _native.ptr(dy), _native.ptr(x), _native.ptr(out2), _native.ptr(ws), wsb, n, k, m, n, k,
                 k, c, sp, _native.stream(dy.device))


# ---------------------------------------------------------------------------------------------
# 3x3 conv


def pack_conv3(w: torch.Tensor) -> torch.Tensor:
    """[Cout, Cin, 3, 3] -> bf16 [Cout, 3, 3, Cin] (K = tap-major, channel-minor)."""
    return w.detach().permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)


def conv_cfg(cout: int) -> int:
    f = _forced()
    if f is not None:
        return f
    return 0 if cout >= 256 else 2


def conv3_supported(cin: int, cout: int) -> bool:
    return cin % 32 == 0 and cout % 4 == 0


def conv3_ref(x, wp, bias=None, residual=None, ascale=None, ashift=None, arelu=True, post_relu=False):
    """fp32 reference (bf16 operands, fp32 accumulation); x NHWC, wp = pack_conv3(w). -> (out, aout)."""
    w = wp.float().permute(0, 3, 1, 2)
    y = F.conv2d(x.float().permute(0, 3, 1, 2), w, None, padding=1).permute(0, 2, 3, 1)
    if bias is not None:
        y = y + bias.float()
    if residual is not None:
        y = y + residual.float()
    if post_relu:
        y = torch.relu(y)
    out = y.to(torch.bfloat16)
    aout = None
    if ascale is not None or ashift is not None:
        a = out.float()
        if ascale is not None:
            a = a * ascale.float()
        if ashift is not None:
            sh = ashift.float()
            a = a + (sh[:, None, None, :] if sh.dim() == 2 else sh)
        if arelu:
            a = torch.relu(a)
        aout = a.to(torch.bfloat16)
    return out, aout


def conv3(x: torch.Tensor, wp: torch.Tensor, bias: torch.Tensor | None = None, *, residual=None, want_out: bool = True,
          ascale=None, ashift=None, arelu: bool = True, post_relu: bool = False, out=None, aout=None,
          cfg: int | None = None):
    """x NHWC bf16 [N, H, W, Cin], wp = :func:`pack_conv3` -> ``(out, aout)`` (see module doc);
    ``ashift`` may be [Cout] or a row-strided [N, Cout] per-image shift."""
    N, H, W, C = x.shape
    cout = wp.shape[0]
    assert wp.shape[1:] == (3, 3, C), "wp must be pack_conv3(w)"
    act = ascale is not None or ashift is not None
    if not x.is_cuda:
        o, a = conv3_ref(x, wp, bias, residual, ascale, ashift, arelu, post_relu)
        return (o if want_out else None), a
    assert conv3_supported(C, cout), "Cin % 32 == 0 and Cout % 4 == 0"
    assert x.dtype == torch.bfloat16 and x.is_contiguous() and wp.is_contiguous() and wp.dtype == torch.bfloat16
    if want_out and out is None:
        out = torch.empty(N, H, W, cout, device=x.device, dtype=torch.bfloat16)
    if act and aout is None:
        aout = torch.empty(N, H, W, cout, device=x.device, dtype=torch.bfloat16)
    if residual is not None:
        assert residual.shape == (N, H, W, cout) and residual.dtype == torch.bfloat16 and residual.is_contiguous()
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.is_contiguous()
    at_ns = 0
    if ashift is not None:
        assert ashift.dtype == torch.float32
        if ashift.dim() == 2:
            assert ashift.shape == (N, cout) and ashift.stride(1) == 1
            at_ns = ashift.stride(0) if N > 1 else cout
            assert at_ns % 4 == 0 and ashift.data_ptr() % 16 == 0
        else:
            assert ashift.is_contiguous() and ashift.numel() == cout
    if ascale is not None:
        assert ascale.dtype == torch.float32 and ascale.is_contiguous() and ascale.numel() == cout
    _native.call("be_conv3_pp", _native.ptr(x), _native.ptr(wp), _native.ptr(bias), _native.ptr(residual),
                 _native.ptr(out if want_out else None), _native.ptr(aout if act else None), _native.ptr(ascale),
                 _native.ptr(ashift), at_ns, int(bool(arelu)), int(bool(post_relu)), N, H, W, C, cout,
                 conv_cfg(cout) if cfg is None else cfg, _native.stream(x.device))
    return (out if want_out else None), (aout if act else None)
