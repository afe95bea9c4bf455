"""FP8 (OCP e4m3fn) linear layers on the CDNA4 block-scaled MFMA (``csrc/kernels/gemm_fp8.hip``).

The reference embeds cells with DINOv2 ViT-B/14 in fp16 on CUDA (``apps/cell-image-search/
embedder.py:35-57``; ~500 img/s/A100, ``README.md:122``).  On MI355X the embedding GEMMs run in fp8:

* weights are quantised once per output channel (``sw[n] = amax_k |W[n,k]| / 448``);
* activations are quantised per token on the fly (``sx[m] = amax_k |x[m,k]| / 448``,
  ``be_quant_fp8_rows``);
* ``be_gemm_fp8`` multiplies the e4m3 operands on ``v_mfma_scale_f32_16x16x128_f8f6f4`` (unit block
  scales, 2x the bf16 MFMA rate) and applies ``sx * sw``, the bias and optionally GELU in its fp32
  epilogue, writing bf16;
* the fp8 activations come from fused producers: ``add_layernorm_fp8`` (residual + LayerNorm ->
  e4m3 + scale) and ``quantize_rows(x, gelu=True)`` (fc1 output -> GELU -> e4m3 + scale), so
  quantisation adds no pass over HBM of its own.

:class:`Fp8Linear` runs ``be_gemm_fp8`` by default (``gemm="hip"``).  With its epilogue operands
loaded before the K loop, the MX block scales staged next to each tile by LDS-DMA, and the
attention epilogue emitting MX-fp8 straight into proj's MFMA scale operand, the DINOv2 ViT-B/14
embedder at batch 64 runs 15,892 img/s on it against 15,662 on hipBLASLt's fp8 GEMM
(``profiles/r03/fp8/fp8_bench_s23.jsonl``); hipBLASLt stays selectable (``gemm="hipblaslt"``).

CPU tensors run the PyTorch reference of the same math (``torch.float8_e4m3fn`` round-to-nearest-even
quantisation, fp32 accumulation) — the oracle the GPU numerics tests compare against.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _native

FP8_MAX = 448.0
FP8_DTYPE = torch.float8_e4m3fn


def _row_scale(x: torch.Tensor) -> torch.Tensor:
    return x.float().abs().amax(dim=-1).clamp_min(1e-12) / FP8_MAX


def quantize_rows_ref(x: torch.Tensor, gelu: bool = False) -> tuple[torch.Tensor, torch.Tensor]:
    """[..., K] -> (e4m3fn [..., K], fp32 scale [...]) with per-row amax scaling (PyTorch math).
    ``gelu``: quantise the bf16-rounded exact GELU of x instead."""
    if gelu:
        x = F.gelu(x.float()).to(torch.bfloat16)
    s = _row_scale(x)
    q = (x.float() / s[..., None]).clamp(-FP8_MAX, FP8_MAX).to(FP8_DTYPE)
    return q, s


def quantize_weight(w: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Per-output-channel quantisation of a [N, K] weight (done once, at model load)."""
    return quantize_rows_ref(w.detach())


def quantize_rows(x: torch.Tensor, gelu: bool = False) -> tuple[torch.Tensor, torch.Tensor]:
    """Dynamic per-token quantisation of a bf16 [..., K] activation (optionally of GELU(x), fused)."""
    if not x.is_cuda:
        return quantize_rows_ref(x, gelu)
    K = x.shape[-1]
    assert x.dtype == torch.bfloat16 and x.is_contiguous() and K % 8 == 0 and K <= 4096, (x.dtype, x.shape)
    rows = x.numel() // K
    q = torch.empty(x.shape, dtype=FP8_DTYPE, device=x.device)
    s = torch.empty(x.shape[:-1], dtype=torch.float32, device=x.device)
    _native.call("be_quant_fp8_rows", _native.ptr(x), _native.ptr(q), _native.ptr(s), rows, K,
                 int(bool(gelu)), _native.stream(x.device))
    return q, s


def linear_fp8_ref(xq, sx, wq, sw, bias=None, gelu: bool = False) -> torch.Tensor:
    y = torch.matmul(xq.float(), wq.float().t()) * sx.float()[..., None] * sw.float()
    if bias is not None:
        y = y + bias.float()
    if gelu:
        y = F.gelu(y)
    return y.to(torch.bfloat16)


def linear_fp8(xq: torch.Tensor, sx: torch.Tensor, wq: torch.Tensor, sw: torch.Tensor,
               bias: torch.Tensor | None = None, gelu: bool = False, tile_cfg: int = 0) -> torch.Tensor:
    """``epi(xq . wq^T * sx * sw + bias)`` -> bf16 [..., N]; xq e4m3fn [..., K], wq e4m3fn [N, K].

    ``tile_cfg`` picks the kernel's block tile (0 = by shape; 1 = 128x128, 2 = 256x128, 3 = 128x256,
    4 = 256x256, 5 / 6 = 128x128 on 8 waves) — exposed for the tile sweep in ``tools/fp8_bench.py``."""
    if not xq.is_cuda:
        return linear_fp8_ref(xq, sx, wq, sw, bias, gelu)
    K = xq.shape[-1]
    N = wq.shape[0]
    M = xq.numel() // K
    assert xq.dtype == FP8_DTYPE and wq.dtype == FP8_DTYPE and wq.shape[1] == K
    assert K % 128 == 0 and N % 4 == 0, "fp8 GEMM needs K % 128 == 0 and N % 4 == 0"
    assert xq.is_contiguous() and wq.is_contiguous() and sx.numel() == M and sw.numel() == N
    y = torch.empty(*xq.shape[:-1], N, dtype=torch.bfloat16, device=xq.device)
    b = bias.float().contiguous() if bias is not None else None
    _native.call("be_gemm_fp8", _native.ptr(xq), _native.ptr(wq), _native.ptr(sx.contiguous()),
                 _native.ptr(sw.float().contiguous()), _native.ptr(b), _native.ptr(y), M, N, K, int(bool(gelu)),
                 int(tile_cfg), _native.stream(xq.device))
    return y


MX_BLOCK = 32


def mx_quantize_ref(x: torch.Tensor, gelu: bool = False) -> tuple[torch.Tensor, torch.Tensor]:
    """[..., K] -> MX-fp8 (e4m3fn [..., K], E8M0 uint8 [..., K/32]): one power-of-two scale 2^e per 32
    consecutive elements of a row, the smallest with amax / 2^e <= 448 (byte = e + 127).  ``gelu``:
    quantise the exact GELU of x (fp32) -- what the fused fc1 epilogue does."""
    xf = x.float()
    if gelu:
        xf = F.gelu(xf)
    K = xf.shape[-1]
    assert K % MX_BLOCK == 0
    blk = xf.reshape(*xf.shape[:-1], K // MX_BLOCK, MX_BLOCK)
    amax = blk.abs().amax(-1)
    e = torch.where(amax > 0, torch.ceil(torch.log2(amax / FP8_MAX)), torch.full_like(amax, -127.0))
    e = torch.where((amax > 0) & (amax * torch.exp2(-e) > FP8_MAX), e + 1, e).clamp(-127, 127)
    q = (blk * torch.exp2(-e)[..., None]).clamp(-FP8_MAX, FP8_MAX).to(FP8_DTYPE).reshape(xf.shape)
    return q, (e + 127).to(torch.uint8)


def mx_dequant_ref(q: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    K = q.shape[-1]
    blk = q.float().reshape(*q.shape[:-1], K // MX_BLOCK, MX_BLOCK)
    return (blk * torch.exp2(s.float() - 127.0)[..., None]).reshape(q.shape)


def linear_fp8_mx(x: tuple, wq: torch.Tensor, sw: torch.Tensor, bias: torch.Tensor | None = None,
                  gelu: bool = False, mx_out: bool = False):
    """fp8 GEMM whose input ``x = (xq, scales)`` carries either per-row fp32 scales ``[M]`` or MX block
    scales (uint8 E8M0 ``[M, K/32]``, applied inside ``v_mfma_scale_f32_16x16x128_f8f6f4``).
    ``mx_out`` (requires ``gelu``): the epilogue applies GELU and writes MX-fp8 ``(yq, ys)`` for the
    next GEMM instead of bf16 -- fc1 -> fc2 of a ViT MLP with no bf16 activation and no quantisation
    pass in between (``be_gemm_fp8_mx``)."""
    xq, xs = x
    mx_in = xs.dtype == torch.uint8
    assert not mx_out or gelu, "MX output is the fused GELU epilogue"
    if not xq.is_cuda:
        xf = mx_dequant_ref(xq, xs) if mx_in else xq.float() * xs.float()[..., None]
        y = torch.matmul(xf, wq.float().t()) * sw.float()
        if bias is not None:
            y = y + bias.float()
        if mx_out:
            return mx_quantize_ref(y, gelu=True)
        return (F.gelu(y) if gelu else y).to(torch.bfloat16)
    K = xq.shape[-1]
    N = wq.shape[0]
    M = xq.numel() // K
    assert xq.dtype == FP8_DTYPE and wq.dtype == FP8_DTYPE and wq.shape[1] == K and xq.is_contiguous()
    assert K % 128 == 0 and N % (MX_BLOCK if mx_out else 4) == 0
    if mx_in:
        assert xs.shape[-1] == K // MX_BLOCK and xs.numel() == M * (K // MX_BLOCK) and xs.is_contiguous()
    else:
        assert xs.numel() == M
    b = bias.float().contiguous() if bias is not None else None
    y = yq = ys = None
    if mx_out:
        yq = torch.empty(*xq.shape[:-1], N, dtype=FP8_DTYPE, device=xq.device)
        ys = torch.empty(*xq.shape[:-1], N // MX_BLOCK, dtype=torch.uint8, device=xq.device)
    else:
        y = torch.empty(*xq.shape[:-1], N, dtype=torch.bfloat16, device=xq.device)
    _native.call("be_gemm_fp8_mx", _native.ptr(xq), None if mx_in else _native.ptr(xs.float().contiguous()),
                 _native.ptr(xs) if mx_in else None, _native.ptr(wq), _native.ptr(sw.float().contiguous()),
                 _native.ptr(b), _native.ptr(y), _native.ptr(yq), _native.ptr(ys), M, N, K,
                 2 if mx_out else int(bool(gelu)), _native.stream(xq.device))
    return (yq, ys) if mx_out else y


def add_layernorm_fp8(x: torch.Tensor, y: torch.Tensor | None, gamma: torch.Tensor | None, w: torch.Tensor,
                      b: torch.Tensor, eps: float = 1e-6) -> tuple[torch.Tensor, torch.Tensor]:
    """``x <- x + gamma * y`` (in place) and returns ``quantize_rows(LN(x) * w + b)`` — the fused
    residual + LayerNorm of ``transformer.add_layernorm`` emitting the fp8 GEMM's input directly."""
    if not x.is_cuda:
        from .transformer import add_layernorm

        return quantize_rows_ref(add_layernorm(x, y, gamma, w, b, eps).float())
    C = x.shape[-1]
    rows = x.numel() // C
    assert x.dtype == torch.bfloat16 and x.is_contiguous()
    if y is not None:
        assert y.shape == x.shape and y.dtype == torch.bfloat16
        y = y.contiguous()
    q = torch.empty(x.shape, dtype=FP8_DTYPE, device=x.device)
    s = torch.empty(x.shape[:-1], dtype=torch.float32, device=x.device)
    g = gamma.float().contiguous() if gamma is not None else None
    _native.call("be_add_layernorm_fp8", _native.ptr(x), _native.ptr(y), _native.ptr(g),
                 _native.ptr(w.float().contiguous()), _native.ptr(b.float().contiguous()), _native.ptr(q),
                 _native.ptr(s), rows, C, float(eps), 1, _native.stream(x.device))
    return q, s


def add_layernorm_mx(x: torch.Tensor, y: torch.Tensor | None, gamma: torch.Tensor | None, w: torch.Tensor,
                     b: torch.Tensor, eps: float = 1e-6) -> tuple[torch.Tensor, torch.Tensor]:
    """``x <- x + gamma * y`` (in place) and returns ``mx_quantize(LN(x) * w + b)``: e4m3fn values and
    one E8M0 scale per 32 channels -- the block-scaled GEMM's A operand (``linear_fp8_mx``)."""
    if not x.is_cuda:
        from .transformer import add_layernorm

        return mx_quantize_ref(add_layernorm(x, y, gamma, w, b, eps).float())
    C = x.shape[-1]
    rows = x.numel() // C
    assert x.dtype == torch.bfloat16 and x.is_contiguous() and C % MX_BLOCK == 0
    if y is not None:
        assert y.shape == x.shape and y.dtype == torch.bfloat16
        y = y.contiguous()
    q = torch.empty(x.shape, dtype=FP8_DTYPE, device=x.device)
    s = torch.empty(*x.shape[:-1], C // MX_BLOCK, dtype=torch.uint8, device=x.device)
    g = gamma.float().contiguous() if gamma is not None else None
    _native.call("be_add_layernorm_mx", _native.ptr(x), _native.ptr(y), _native.ptr(g),
                 _native.ptr(w.float().contiguous()), _native.ptr(b.float().contiguous()), _native.ptr(q),
                 _native.ptr(s), rows, C, float(eps), 1, _native.stream(x.device))
    return q, s


def linear_fp8_hipblaslt(xq: torch.Tensor, sx: torch.Tensor, wq: torch.Tensor, sw: torch.Tensor,
                         bias: torch.Tensor | None = None) -> torch.Tensor:
    """The same row-wise-scaled fp8 GEMM as :func:`linear_fp8` (no GELU) through hipBLASLt
    (``torch._scaled_mm`` with per-token / per-channel scale vectors)."""
    K = xq.shape[-1]
    x2 = xq.reshape(-1, K)
    y = torch._scaled_mm(x2, wq.t(), scale_a=sx.reshape(-1, 1).float(), scale_b=sw.reshape(1, -1).float(),
                         bias=None if bias is None else bias.to(torch.bfloat16), out_dtype=torch.bfloat16)
    return y.view(*xq.shape[:-1], wq.shape[0])


class Fp8Linear:
    """A frozen linear layer holding e4m3 weights + per-channel scales (inference only).

    ``gemm`` picks the GEMM for GPU tensors: ``"hip"`` (default, our block-scaled MFMA kernel; faster
    end to end on the ViT-B/14 embedder, ``profiles/r03/fp8/fp8_bench_s23.jsonl``) or ``"hipblaslt"``
    (the plain row-wise-scaled library GEMM); ``be_gemm_fp8`` also fuses GELU / MX-fp8 output into
    its epilogue.  No silent fallback between them."""

    def __init__(self, weight: torch.Tensor, bias: torch.Tensor | None = None, gemm: str = "hip"):
        if gemm not in ("hipblaslt", "hip"):
            raise ValueError(f"gemm must be 'hipblaslt' or 'hip', got {gemm!r}")
        self.gemm = gemm
        self.wq, self.sw = quantize_weight(weight)
        self.bias = None if bias is None else bias.detach().float().contiguous()

    def to(self, device) -> "Fp8Linear":
        self.wq, self.sw = self.wq.to(device), self.sw.to(device)
        if self.bias is not None:
            self.bias = self.bias.to(device)
        return self

    def __call__(self, x, gelu: bool = False, mx_out: bool = False):
        """x: bf16 activations, or an already-quantised ``(xq, sx)`` pair (``add_layernorm_fp8``), or
        an MX pair ``(xq, uint8 block scales)`` (``mx_out`` of the previous layer; HIP GEMM only).
        ``mx_out``: GELU + MX-fp8 output ``(yq, ys)`` straight from the epilogue (HIP GEMM only)."""
        if mx_out or (isinstance(x, tuple) and x[1].dtype == torch.uint8):
            if self.gemm != "hip" and x[0].is_cuda:
                raise ValueError("MX-fp8 activations need Fp8Linear(gemm='hip')")
            return linear_fp8_mx(x if isinstance(x, tuple) else quantize_rows(x), self.wq, self.sw, self.bias,
                                 gelu=gelu or mx_out, mx_out=mx_out)
        xq, sx = x if isinstance(x, tuple) else quantize_rows(x)
        if xq.is_cuda and self.gemm == "hipblaslt":
            y = linear_fp8_hipblaslt(xq, sx, self.wq, self.sw, self.bias)
            return F.gelu(y) if gelu else y
        return linear_fp8(xq, sx, self.wq, self.sw, self.bias, gelu)
