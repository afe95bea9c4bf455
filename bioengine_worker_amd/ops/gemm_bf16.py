"""In-house bf16 MFMA GEMMs with fused epilogues (``csrc/kernels/gemm_bf16.hip``) for the CPSAM
training engine (``train/cpsam_engine.py``), same helper surface as :mod:`.gemm`:

* :func:`linear` -- ``x W^T (+ b)``;
* :func:`linear_gelu` -- ``f = x W^T + b`` and ``g = gelu(f)`` from ONE GEMM (pre-activation kept
  for the backward);
* :func:`mm` -- ``x W`` (dgrad; W read as stored, transposed in LDS);
* :func:`mm_dgelu` -- ``df = gelu'(f) * (dm W2)`` with the lin1 bias gradient ``sum_rows(df)``
  reduced in the same epilogue;
* :func:`wgrad` -- ``dy^T x`` in fp32, written in place (split-K over tokens with a slab sum).

The GELU is the erf form of the reference's ``nn.GELU`` in both directions.  On CPU every helper
is the plain fp32 PyTorch op (the reference math of the same call)."""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _native

E_NONE, E_BIAS, E_BIAS_GELU, E_DGELU, E_F32 = range(5)
_ws: dict = {}


def _workspace(dev: torch.device, nbytes: int) -> torch.Tensor:
    key = (dev.index, torch.cuda.current_stream(dev).stream_id)
    w = _ws.get(key)
    if w is None or w.numel() < nbytes:
        w = _ws[key] = torch.empty(max(nbytes, 64 << 20), dtype=torch.uint8, device=dev)
    return w


def _cfg(M: int, N: int) -> int:
    """256x128 tiles when they fill the chip, else 128x128 (``BE_GEMM_CFG`` forces one: 0 = 256x128 on
    8 waves, 1 = 128x128 on 4, 2 = 256x128 on 4 waves of 128x64, 3 = 128x256 on 4 waves of 64x128)."""
    return 0 if ((M + 255) // 256) * ((N + 127) // 128) >= 192 else 1


def _call(A, B, C, M, N, K, lda, ldb, ldc, ta, tb, epi, C2=None, bias=None, aux=None, dbias=None, split=1, cfg=None):
    if bias is not None and (bias.dtype != torch.float32 or not bias.is_contiguous()):
        bias = bias.float().contiguous()  # the epilogue reads fp32 (the engine's biases are bf16 mirror views)
    ws, wsb = None, 0
    if split > 1:
        ws = _workspace(A.device, split * M * ldc * 4)
        wsb = ws.numel()
    if cfg is None:
        cfg = _cfg(M, N)
        forced = os.environ.get("BE_GEMM_CFG")
        if forced is not None:
            cfg = int(forced)
        bm, bn = {0: (256, 128), 1: (128, 128), 2: (256, 128), 3: (128, 256)}[cfg]
        if (ta == 1 and M % bm) or (tb == 1 and N % bn):
            cfg = 1  # transposed tiles are read whole: 128 x 128 tiles
    _native.call("be_gemm_bf16", _native.ptr(A), _native.ptr(B), _native.ptr(C), _native.ptr(C2), _native.ptr(bias),
                 _native.ptr(aux), _native.ptr(dbias), _native.ptr(ws), wsb, M, N, K, lda, ldb, ldc, ta, tb, epi,
                 cfg, split, _native.stream(A.device))
    return C


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    """x [M, K] @ w [N, K]^T (+ b) -> bf16 [M, N]."""
    M, K = x.shape
    N = w.shape[0]
    if not x.is_cuda or not supported(M, N, K, "linear") or not (x.is_contiguous() and w.is_contiguous()):
        return F.linear(x, w, b)
    out = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    return _call(x, w, out, M, N, K, K, K, N, 0, 0, E_BIAS if b is not None else E_NONE, bias=b)


def linear_gelu(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """-> (g = gelu(f), f = x w^T + b)."""
    M, K = x.shape
    N = w.shape[0]
    if not x.is_cuda or not supported(M, N, K, "linear"):
        f = F.linear(x, w, b)
        return F.gelu(f), f
    f = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    g = torch.empty_like(f)
    _call(x, w, f, M, N, K, K, K, N, 0, 0, E_BIAS_GELU, C2=g, bias=b)
    return g, f


def mm(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """x [M, K] @ w [K, N] -> bf16 [M, N]."""
    M, K = x.shape
    N = w.shape[1]
    if not x.is_cuda or not supported(M, N, K, "mm") or not (x.is_contiguous() and w.is_contiguous()):
        return torch.mm(x, w)
    out = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    return _call(x, w, out, M, N, K, K, N, N, 0, 1, E_NONE)


def _gelu_grad(f: torch.Tensor) -> torch.Tensor:
    x = f.float()
    return 0.5 * (1.0 + torch.erf(x * 0.7071067811865476)) + x * torch.exp(-0.5 * x * x) * 0.3989422804014327


def mm_dgelu(dm: torch.Tensor, w2: torch.Tensor, f: torch.Tensor, out_db: torch.Tensor | None = None) -> torch.Tensor:
    """df = gelu'(f) * (dm @ w2), dm [M, K], w2 [K, N], f [M, N]; out_db [N] fp32 = sum_rows(df)."""
    if not dm.is_cuda or not supported(dm.shape[0], w2.shape[1], dm.shape[1], "mm"):
        df = (_gelu_grad(f) * (dm.float() @ w2.float())).to(dm.dtype)
        if out_db is not None:
            torch.sum(df.float(), 0, out=out_db)
        return df
    M, K = dm.shape
    N = w2.shape[1]
    df = torch.empty(M, N, device=dm.device, dtype=torch.bfloat16)
    if out_db is not None:
        out_db.zero_()
    return _call(dm, w2, df, M, N, K, K, N, N, 0, 1, E_DGELU, aux=f, dbias=out_db)


def wgrad_split(n_out: int, k_in: int, m: int) -> int:
    """Split-K factor for a [n_out, k_in] weight gradient over m tokens: enough blocks for the chip."""
    cfg = _cfg(n_out, k_in)
    tiles = ((n_out + (255 if cfg == 0 else 127)) // (256 if cfg == 0 else 128)) * ((k_in + 127) // 128)
    split = 1
    while tiles * split < 224 and m % (64 * split * 2) == 0 and m // (split * 2) >= 512:
        split *= 2
    return split


def wgrad(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor) -> None:
    """out (fp32 [n, k], in place) = dy^T x with dy [m, n], x [m, k]."""
    out2 = out.view(out.shape[0], -1)
    m, n = dy.shape
    k = x.shape[1]
    if not dy.is_cuda or dy.dtype != torch.bfloat16 or not supported(n, k, m, "wgrad") or not (
            dy.is_contiguous() and x.is_contiguous() and out2.is_contiguous()):
        if dy.is_cuda:
            from ..train.cpsam_engine import _wgrad

            _wgrad(dy, x, out)
        else:
            torch.mm(dy.t().to(out2.dtype), x.to(out2.dtype), out=out2)
        return
    assert out2.is_contiguous() and out2.dtype == torch.float32
    _call(dy, x, out2, n, k, m, n, k, k, 1, 1, E_F32, split=wgrad_split(n, k, m))


def supported(M: int, N: int, K: int, kind: str) -> bool:
    """Shapes the kernel takes as they are (transposed tiles are read whole)."""
    if K % 64 or N % 4:
        return False
    if kind == "mm":
        return N % 128 == 0
    if kind == "wgrad":
        return M % 128 == 0 and N % 128 == 0
    return True
