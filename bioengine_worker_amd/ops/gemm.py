"""Library GEMMs (PyTorch -> hipBLASLt) for the CPSAM training engine (``train/cpsam_engine.py``),
with the same row-major helper surface as the in-house kernels (:mod:`.gemm_bf16`, :mod:`.gemm_pp`):

* :func:`linear` -- ``x W^T (+ b)``, bf16 out;
* :func:`linear_gelu` -- MLP lin1 forward: ``f = x W^T + b``, then ``g = gelu(f)`` (one HIP pass of
  ``vit_train``); ``f`` is kept for the backward;
* :func:`mm_dgelu` -- lin2 dgrad + the GELU backward: ``df = gelu'(f) * (dm W2)`` and the lin1 bias
  gradient ``sum_rows(df)`` (fp32) from the HIP GELU-backward kernel;
* :func:`mm` -- ``x W`` (dgrad); :func:`wgrad` -- ``dy^T x`` with an fp32 result written in place
  (the parameter's view of the flat gradient buffer; split-K below 192 output tiles).

This is the engine's default backend: on the whole graphed step it measured faster than the
in-house kernels (``profiles/r04/cpsam/``).  The GELU is the erf form of the reference's
``nn.GELU`` in both directions.  On CPU every helper runs the plain fp32 PyTorch op (the reference
math), so the engine's CPU test covers the same call sequence.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

_zeros: dict = {}


def _zero(dev: torch.device, n: int) -> torch.Tensor:
    z = _zeros.get((dev.index, n))
    if z is None:
        z = _zeros[(dev.index, n)] = torch.zeros(n, device=dev)
    return z


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    """x [M, K] @ w[N, K]^T (+ b[N]) -> [M, N] (x.dtype)."""
    return F.linear(x, w, b)


def linear_gelu(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """-> (g = gelu(x w^T + b), f = x w^T + b), both [M, N]."""
    f = F.linear(x, w, b)
    if not x.is_cuda:
        return F.gelu(f), f
    from . import vit_train as vt

    return vt.gelu_fwd(f, _zero(f.device, f.shape[1])), f


def _gelu_grad(f: torch.Tensor) -> torch.Tensor:
    """d gelu(x) / dx of the erf GELU: Phi(x) + x phi(x)."""
    x = f.float()
    return 0.5 * (1.0 + torch.erf(x * 0.7071067811865476)) + x * torch.exp(-0.5 * x * x) * 0.3989422804014327


def mm_dgelu(dm: torch.Tensor, w2: torch.Tensor, f: torch.Tensor, out_db: torch.Tensor | None = None) -> torch.Tensor:
    """df = gelu'(f) * (dm @ w2) with dm [M, K], w2 [K, N], f [M, N]; out_db[N] (fp32) = df summed
    over rows (written in place when given)."""
    if not dm.is_cuda:
        df = (_gelu_grad(f) * (dm.float() @ w2.float())).to(dm.dtype)
        if out_db is not None:
            torch.sum(df.float(), 0, out=out_db)
        return df
    from . import vit_train as vt

    df, _ = vt.gelu_bwd(torch.mm(dm, w2), f, _zero(dm.device, w2.shape[1]), out_db=out_db)
    return df


def mm(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """x [M, K] @ w [K, N] -> [M, N]."""
    return torch.mm(x, w)


def wgrad(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor) -> None:
    """out (fp32 [n, k], in place) = dy^T x with dy [m, n], x [m, k]."""
    if dy.is_cuda:
        from ..train.cpsam_engine import _wgrad

        _wgrad(dy, x, out)
        return
    out2 = out.view(out.shape[0], -1)
    torch.mm(dy.t().to(out2.dtype), x.to(out2.dtype), out=out2)
