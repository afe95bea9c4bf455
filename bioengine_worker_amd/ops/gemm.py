"""Epilogue-fused, autotuned library GEMMs (``csrc/kernels/gemm_lt.hip`` over hipBLASLt).

Row-major helpers used by the CPSAM training engine (``train/cpsam_engine.py``):

* :func:`linear` -- ``x W^T (+ b)``, bf16 out;
* :func:`linear_gelu` -- MLP lin1 forward: ``f = x W^T + b`` (bias in the GEMM epilogue), then
  ``g = gelu(f)`` (one HIP pass); ``f`` is kept for the backward.  The GELU-with-aux-output epilogue
  that would produce both from the GEMM is not available in this hipBLASLt build for any layout or
  bias / aux type (``tools/lt_probe.py`` -> ``profiles/r03/cpsam/hipblaslt_epilogue_probe.jsonl``);
* :func:`mm_dgelu` -- lin2 dgrad fused with the GELU backward: ``df = gelu'(f) * (dm W2)`` and the
  lin1 bias gradient ``sum_rows(df)`` (fp32) from one GEMM;
* :func:`mm` -- ``x W`` (dgrad), :func:`wgrad` -- ``dy^T x`` with an fp32 result written in place
  (the parameter's view of the flat gradient buffer).

The forward GELU is the erf form of the reference's ``nn.GELU``; the epilogue's GELU derivative is
hipBLASLt's (tanh form), which differs from the erf derivative by < 2e-3 absolute -- below bf16
resolution of the gradients; the ViT-L numerics test (``tests/test_cpsam_numerics_gpu.py``) bounds
the whole step against fp32 autograd.

On CPU every helper runs the plain PyTorch op (fp32 reference math), so the engine's CPU test
covers the same call sequence.  On GPU with ``BE_LT=0`` the helpers run the round-2 path (bf16
``torch.mm`` / ``F.linear`` on PyTorch's hipBLASLt heuristics + the HIP GELU kernels of
``vit_train``), which is the A/B baseline of ``tools/cpsam_train_bench.py``.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _native

EPI_NONE, EPI_BIAS, EPI_GELU_AUX_BIAS, EPI_DGELU_BGRAD, EPI_GELU_BIAS, EPI_BGRAD, EPI_DGELU = range(7)
_WS_BYTES = 64 << 20
_ws: dict = {}
_zeros: dict = {}
_dgelu_mode: dict = {}  # (device, M, N, K) -> the GELU-backward variant that runs for that shape


def enabled(t: torch.Tensor) -> bool:
    """Opt-in (``BE_LT=1``): on the CPSAM B=8 step the tuned plans ended up on the same hipBLASLt
    kernels as PyTorch's heuristic -- identical per-kernel times in the step-window kernel traces
    (profiles/r03/cpsam/kt_step_b8_{lt,torch}.txt, 37.58 vs 37.57 ms kernel-busy per step)."""
    return t.is_cuda and os.environ.get("BE_LT", "0") == "1"


def _workspace(dev: torch.device) -> torch.Tensor:
    """One workspace per (device, stream): GEMMs on two streams (the CPSAM engine's side-stream
    weight gradients) must not share scratch."""
    key = (dev.index, torch.cuda.current_stream(dev).stream_id)
    w = _ws.get(key)
    if w is None:
        w = _ws[key] = torch.empty(_WS_BYTES, dtype=torch.uint8, device=dev)
    return w


def _gemm(x, y, out, M, N, K, tx, ty, epi=EPI_NONE, bias=None, aux=None, bgrad=None, bias_fp32=0, alpha=1.0,
          beta=0.0):
    assert x.dtype == torch.bfloat16 and y.dtype == torch.bfloat16
    assert x.is_contiguous() and y.is_contiguous() and out.is_contiguous()
    ws = _workspace(x.device)
    _native.call("be_lt_gemm", _native.ptr(x), _native.ptr(y), _native.ptr(out), _native.ptr(bias), _native.ptr(aux),
                 _native.ptr(bgrad), _native.ptr(ws), ws.numel(), M, N, K, tx, ty,
                 1 if out.dtype == torch.float32 else 0, epi, bias_fp32, float(alpha), float(beta),
                 _native.stream(x.device))
    return out


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    """x [M, K] @ w[N, K]^T (+ b[N]) -> [M, N] (x.dtype)."""
    if not enabled(x):
        return F.linear(x, w, b)
    M, K = x.shape
    N = w.shape[0]
    out = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    return _gemm(x, w, out, M, N, K, 0, 1, EPI_BIAS if b is not None else EPI_NONE, bias=b)


def linear_gelu(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """-> (g = gelu(x w^T + b), f = x w^T + b), both [M, N]."""
    from . import vit_train as vt

    if not enabled(x):
        f = F.linear(x, w, b)
        return (vt.gelu_fwd(f, _zero(f.device, f.shape[1])) if x.is_cuda else F.gelu(f)), f

    f = linear(x, w, b)
    return vt.gelu_fwd(f, _zero(f.device, f.shape[1])), f


def _zero(dev: torch.device, n: int) -> torch.Tensor:
    z = _zeros.get((dev.index, n))
    if z is None:
        z = _zeros[(dev.index, n)] = torch.zeros(n, device=dev)
    return z


def _gelu_grad(f: torch.Tensor) -> torch.Tensor:
    """d gelu(x) / dx of the erf GELU: Phi(x) + x phi(x)."""
    x = f.float()
    return 0.5 * (1.0 + torch.erf(x * 0.7071067811865476)) + x * torch.exp(-0.5 * x * x) * 0.3989422804014327


def mm_dgelu(dm: torch.Tensor, w2: torch.Tensor, f: torch.Tensor, out_db: torch.Tensor | None = None) -> torch.Tensor:
    """df = gelu'(f) * (dm @ w2) with dm [M, K], w2 [K, N], f [M, N]; out_db[N] (fp32) = df summed
    over rows (written in place when given).

    hipBLASLt's DGELU epilogues exist only for some shapes in this build, so the first (eager) call
    of each shape picks the first variant that runs, in order: DGELU + fp32 bias gradient in one
    GEMM; DGELU + bf16 bias gradient; DGELU GEMM + a column-sum pass; plain GEMM + the HIP GELU
    backward kernel.  A variant that is not available fails in the heuristic before anything is
    enqueued, so probing is safe inside a graph capture too."""
    if dm.is_cuda and not enabled(dm):
        return _mm_dgelu_mode("kernel", dm, w2, f, out_db, *dm.shape[:1], w2.shape[1], dm.shape[1])
    if not enabled(dm):
        df = (_gelu_grad(f) * (dm.float() @ w2.float())).to(dm.dtype)
        if out_db is not None:
            torch.sum(df.float(), 0, out=out_db)
        return df
    M, K = dm.shape
    N = w2.shape[1]
    key = (dm.device.index, M, N, K)
    if os.environ.get("BE_LT_DGELU", "0") != "1":
        # default: tuned GEMM + the HIP GELU-backward kernel.  Measured (profiles/r03/cpsam/gemm_ab_b*.jsonl):
        # the DGELU epilogue kernels of this hipBLASLt build are 2.2-2.8x slower than GEMM + pass
        # (8192x4096x1024: 364 vs ~125 us), and one B=1 run with the bgrad32 variant gave a NaN loss.
        _dgelu_mode[key] = "kernel"
        return _mm_dgelu_mode("kernel", dm, w2, f, out_db, M, N, K)
    modes = [_dgelu_mode[key]] if key in _dgelu_mode else ["bgrad32", "bgrad16", "dgelu", "kernel"]
    for mode in modes:
        try:
            df = _mm_dgelu_mode(mode, dm, w2, f, out_db, M, N, K)
        except RuntimeError:
            if len(modes) == 1:
                raise
            continue
        _dgelu_mode[key] = mode
        return df
    raise RuntimeError("no GELU-backward GEMM variant ran")


def _mm_dgelu_mode(mode, dm, w2, f, out_db, M, N, K):
    dev = dm.device
    df = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    if mode == "bgrad32":
        db = out_db if out_db is not None else torch.empty(N, device=dev, dtype=torch.float32)
        _gemm(dm, w2, df, M, N, K, 0, 0, EPI_DGELU_BGRAD, aux=f, bgrad=db, bias_fp32=1)
    elif mode == "bgrad16":
        db = torch.empty(N, device=dev, dtype=torch.bfloat16)
        _gemm(dm, w2, df, M, N, K, 0, 0, EPI_DGELU_BGRAD, aux=f, bgrad=db, bias_fp32=0)
        if out_db is not None:
            out_db.copy_(db)
    elif mode == "dgelu":
        _gemm(dm, w2, df, M, N, K, 0, 0, EPI_DGELU, aux=f)
        if out_db is not None:
            torch.sum(df, 0, dtype=torch.float32, out=out_db)
    else:
        from . import vit_train as vt

        dg = mm(dm, w2)
        z = _zero(dev, N)
        df, _ = vt.gelu_bwd(dg, f, z, out_db=out_db)
    return df


def mm(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """x [M, K] @ w [K, N] -> [M, N]."""
    if not enabled(x):
        return torch.mm(x, w)
    M, K = x.shape
    N = w.shape[1]
    out = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    return _gemm(x, w, out, M, N, K, 0, 0)


def wgrad(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor) -> None:
    """out (fp32 [n, k], in place) = dy^T x with dy [m, n], x [m, k]."""
    out2 = out.view(out.shape[0], -1)
    if dy.is_cuda and not enabled(dy):
        from ..train.cpsam_engine import _wgrad

        _wgrad(dy, x, out)
        return
    if not enabled(dy) or dy.dtype != torch.bfloat16:
        torch.mm(dy.t().to(out2.dtype), x.to(out2.dtype), out=out2)
        return
    m, n = dy.shape
    k = x.shape[1]
    if m >= 4096 and n * k <= 3072 * 1024:
        # <= 192 output tiles: PyTorch's batched split-K path is faster here (proj 38.7 vs 52.3 us)
        from ..train.cpsam_engine import _wgrad

        _wgrad(dy, x, out)
        return
    _gemm(dy, x, out2, n, k, m, 1, 0)


def plans() -> list[dict]:
    """The autotuned GEMM table of this process (shape, layout, epilogue, candidates, best us)."""
    import ctypes

    cap = 256
    buf = (ctypes.c_longlong * (10 * cap))()
    n = _native.hip().be_lt_plans(buf, cap)
    rows = []
    for i in range(min(n, cap)):
        r = buf[10 * i:10 * i + 10]
        rows.append({"M": r[0], "N": r[1], "K": r[2], "tx": r[3], "ty": r[4], "fp32_out": r[5], "epi": r[6],
                     "accum": r[7], "candidates": r[8] // 1000, "rejected": r[8] % 1000, "best_us": r[9] / 1000.0})
    return rows


def dgelu_modes() -> dict:
    """{"MxNxK": variant} of the GELU-backward GEMMs this process has run."""
    return {f"{k[1]}x{k[2]}x{k[3]}": v for k, v in _dgelu_mode.items()}
