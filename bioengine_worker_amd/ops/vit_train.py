"""ViT training ops (``csrc/kernels/vit_train.hip``, ``attention_bwd.hip``, ``layernorm.hip``).

The autograd-free Cellpose-SAM training engine (``train/cpsam_engine.py``) is built from these plus
hipBLASLt GEMMs:

* :func:`ln_fwd` — ``xo = x + rs[b] * y`` then ``LayerNorm(xo)`` with saved (mean, rstd).
* :func:`ln_bwd` — LayerNorm backward fused with the residual-gradient accumulation and the column
  partials of dw / db / sum(dx).
* :func:`gelu_fwd` / :func:`gelu_bwd` — bias + exact GELU (pre-activation kept) and its backward
  with the bias-gradient partials.
* :func:`scale_cast` — per-sample scaled fp32 -> bf16 cast + column sums (bias gradients).
* :func:`attn_bwd` — flash-attention backward with the SAM decomposed rel-pos bias gradients.

GPU tensors run the HIP kernels; CPU tensors run the fp32 PyTorch reference of the same math (the
oracle of the CPU engine test and of the GPU numerics tests).
"""
from __future__ import annotations

import math

import os

import torch
import torch.nn.functional as F

from . import _native


_ROWCOL_BLOCKS = int(os.environ.get("BE_ROWCOL_BLOCKS", "512"))


def _rpb(rows: int, target_blocks: int | None = None) -> int:
    return max(4, -(-rows // (target_blocks or _ROWCOL_BLOCKS)))


class ColsumDeferral:
    """Collects the fp32 partial -> ``out`` column reductions of the backward kernels and runs them
    all in :meth:`flush` (``be_colsum_batched``: one launch per 48 reductions instead of one each).
    Only reductions with a caller-supplied ``out`` (gradient views read after the backward) are
    deferred; the partials stay referenced until the flush."""

    def __init__(self):
        self.items: list[tuple[torch.Tensor, torch.Tensor]] = []

    def add(self, p: torch.Tensor, out: torch.Tensor) -> None:
        self.items.append((p, out))

    def flush(self) -> None:
        if not self.items:
            return
        desc = torch.tensor([[p.data_ptr(), o.data_ptr(), p.shape[0], p.shape[1]] for p, o in self.items],
                            dtype=torch.int64)
        dev = self.items[0][0].device
        _native.call("be_colsum_batched", desc.data_ptr(), len(self.items), _native.stream(dev))
        self.items.clear()


_DEFER: ColsumDeferral | None = None


class defer_colsums:
    """``with defer_colsums() as d: ...; d.flush()`` -- see :class:`ColsumDeferral` (GPU only; the
    flush also runs on exit)."""

    def __enter__(self) -> ColsumDeferral:
        global _DEFER
        self._prev, _DEFER = _DEFER, ColsumDeferral()
        return _DEFER

    def __exit__(self, *exc) -> None:
        global _DEFER
        d, _DEFER = _DEFER, self._prev
        if exc[0] is None:
            d.flush()


def _deferrable(p: torch.Tensor, out: torch.Tensor | None) -> bool:
    return (_DEFER is not None and out is not None and p.is_cuda and p.dtype == torch.float32 and p.dim() == 2
            and p.is_contiguous() and out.is_contiguous() and out.dtype == torch.float32
            and out.numel() == p.shape[1])


def _colsum(p: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Column sums of [rows, C] (fp32), written into ``out`` when given (no extra copy).  On the GPU
    the kernels' fp32 partials go through ``be_colsum`` (one small launch, ~3x faster than torch's
    dim-0 reduction at these shapes), or are deferred to a batched launch (:class:`defer_colsums`)."""
    if _deferrable(p, out):
        _DEFER.add(p, out)
        return out.view(-1)
    if p.is_cuda and p.dtype == torch.float32 and p.dim() == 2 and p.is_contiguous():
        o = torch.empty(p.shape[1], device=p.device, dtype=torch.float32) if out is None else out.view(-1)
        if o.is_contiguous():
            _native.call("be_colsum", _native.ptr(p), _native.ptr(o), p.shape[0], p.shape[1], _native.stream(p.device))
            return o
    if out is None:
        return p.sum(0, dtype=torch.float32)
    return torch.sum(p, 0, dtype=torch.float32, out=out.view(-1))


def colsum_bf16(x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out (fp32 [C]) = column sums of x [rows, C] (bf16 on GPU: per-16-row fp32 partials by
    ``be_colpart_bf16``, 16 rows each, then the (deferrable) partial reduction)."""
    C = x.shape[-1]
    rows = x.numel() // C
    if x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and C % 8 == 0:
        part = torch.empty(-(-rows // 16), C, device=x.device, dtype=torch.float32)
        _native.call("be_colpart_bf16", _native.ptr(x), _native.ptr(part), rows, C, _native.stream(x.device))
        return _colsum(part, out)
    return torch.sum(x.reshape(rows, C), 0, dtype=torch.float32, out=out.view(-1))


def sum_slabs(ws: torch.Tensor, out: torch.Tensor) -> None:
    """out = ws.sum(0) for fp32 split-K slabs ws [S, ...] (one vectorised pass on the GPU)."""
    n = out.numel()
    if ws.is_cuda and ws.is_contiguous() and out.is_contiguous() and n % 4 == 0 and ws.numel() == ws.shape[0] * n:
        _native.call("be_sum_slabs", _native.ptr(ws), _native.ptr(out), ws.shape[0], n, _native.stream(ws.device))
    else:
        torch.sum(ws, 0, out=out.view(ws.shape[1:]))


def _rowscale(rs: torch.Tensor | None, rows: int, rpn: int):
    if rs is None:
        return None
    return rs.float().repeat_interleave(rpn)[:rows, None]


# ------------------------------------------------------------------ LayerNorm
def ln_fwd(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, y: torch.Tensor | None = None,
           rs: torch.Tensor | None = None, rpn: int = 1, xo: torch.Tensor | None = None, eps: float = 1e-6):
    """Returns (xo, out, stats): xo = x + rs[row // rpn] * y (None when y is None), out = LN(xo or x)."""
    C = x.shape[-1]
    rows = x.numel() // C
    if x.is_cuda:
        assert x.dtype == torch.bfloat16 and x.is_contiguous()
        out = torch.empty_like(x)
        stats = torch.empty(rows, 2, device=x.device, dtype=torch.float32)
        if y is not None:
            assert y.shape == x.shape and y.dtype == torch.bfloat16 and y.is_contiguous()
            xo = torch.empty_like(x) if xo is None else xo
        else:
            xo = None
        _native.call("be_add_layernorm_train", _native.ptr(x), _native.ptr(y),
                     _native.ptr(rs.float().contiguous() if rs is not None else None), int(rpn), _native.ptr(xo),
                     _native.ptr(w), _native.ptr(b), _native.ptr(out), _native.ptr(stats), rows, C, float(eps),
                     _native.stream(x.device))
        return xo, out, stats
    xf = x.float().reshape(rows, C)
    if y is not None:
        sc = _rowscale(rs, rows, rpn)
        yf = y.float().reshape(rows, C)
        xf = xf + (yf * sc if sc is not None else yf)
        xf = xf.to(x.dtype).float()
        if xo is None:
            xo = xf.to(x.dtype).reshape(x.shape)
        else:
            xo.copy_(xf.reshape(x.shape))
    else:
        xo = None
    mean = xf.mean(-1)
    rstd = torch.rsqrt(xf.var(-1, unbiased=False) + eps)
    out = ((xf - mean[:, None]) * rstd[:, None] * w.float() + b.float()).to(x.dtype).reshape(x.shape)
    return xo, out, torch.stack([mean, rstd], 1)


def ln_bwd(dh: torch.Tensor, x: torch.Tensor, stats: torch.Tensor, w: torch.Tensor,
           r1: torch.Tensor | None = None, s1: torch.Tensor | None = None, r2: torch.Tensor | None = None,
           s2: torch.Tensor | None = None, rpn: int = 1, want_dx: bool = True, want_dxb: bool = False,
           want_col: bool = False, out_dw: torch.Tensor | None = None, out_db: torch.Tensor | None = None,
           out_col: torch.Tensor | None = None):
    """LayerNorm backward.  Returns (dx fp32 | None, dx bf16 | None, dw, db, colsum(dx) | None) with
    dx = LN'(dh) + s1[b] r1 + s2[b] r2.  ``out_*``: write the reduced sums straight into these (e.g.
    the parameters' views of the flat gradient buffer)."""
    C = x.shape[-1]
    rows = x.numel() // C
    if x.is_cuda:
        rpb = _rpb(rows)
        nblk = -(-rows // rpb)
        dev = x.device
        dx = torch.empty(rows, C, device=dev, dtype=torch.float32) if want_dx else None
        dxb = torch.empty(rows, C, device=dev, dtype=torch.bfloat16) if want_dxb else None
        pdw = torch.empty(nblk, C, device=dev, dtype=torch.float32)
        pdb = torch.empty(nblk, C, device=dev, dtype=torch.float32)
        pcol = torch.empty(nblk, C, device=dev, dtype=torch.float32) if want_col else None
        f = lambda t: None if t is None else t.float().contiguous()
        _native.call("be_ln_bwd", _native.ptr(dh.contiguous()), _native.ptr(x), _native.ptr(stats),
                     _native.ptr(w.float().contiguous()), _native.ptr(f(r1)), _native.ptr(f(s1)), _native.ptr(f(r2)),
                     _native.ptr(f(s2)), int(rpn), _native.ptr(dx), _native.ptr(dxb), _native.ptr(pdw),
                     _native.ptr(pdb), _native.ptr(pcol), rows, C, rpb, _native.stream(dev))
        if _deferrable(pdw, out_dw) and _deferrable(pdb, out_db):
            dw, db = _colsum(pdw, out_dw), _colsum(pdb, out_db)
        elif out_dw is not None and out_db is not None and out_dw.is_contiguous() and out_db.is_contiguous():
            _native.call("be_colsum2", _native.ptr(pdw), _native.ptr(out_dw), _native.ptr(pdb), _native.ptr(out_db),
                         nblk, C, _native.stream(dev))  # dw and db partials in one launch
            dw, db = out_dw.view(-1), out_db.view(-1)
        else:
            dw, db = _colsum(pdw, out_dw), _colsum(pdb, out_db)
        return dx, dxb, dw, db, (_colsum(pcol, out_col) if want_col else None)
    xf = x.float().reshape(rows, C)
    d = dh.float().reshape(rows, C)
    mean, rstd = stats[:, 0:1], stats[:, 1:2]
    xh = (xf - mean) * rstd
    g = d * w.float()
    o = rstd * (g - g.mean(-1, keepdim=True) - xh * (g * xh).mean(-1, keepdim=True))
    for r, s in ((r1, s1), (r2, s2)):
        if r is not None:
            sc = _rowscale(s, rows, rpn)
            rf = r.float().reshape(rows, C)
            o = o + (rf * sc if sc is not None else rf)
    dw, db = _colsum(d * xh, out_dw), _colsum(d, out_db)
    return (o if want_dx else None, o.to(dh.dtype) if want_dxb else None, dw, db,
            _colsum(o, out_col) if want_col else None)


# ------------------------------------------------------------------ GELU / casts
def gelu_fwd(f: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    C = f.shape[-1]
    rows = f.numel() // C
    if f.is_cuda:
        g = torch.empty_like(f)
        _native.call("be_gelu_fwd", _native.ptr(f), _native.ptr(bias.float().contiguous()), _native.ptr(g), rows, C,
                     _rpb(rows), _native.stream(f.device))
        return g
    return F.gelu(f.float() + bias.float()).to(f.dtype)


def gelu_bwd(dg: torch.Tensor, f: torch.Tensor, bias: torch.Tensor, out_db: torch.Tensor | None = None):
    """(df, dbias) for g = gelu(f + bias)."""
    C = f.shape[-1]
    rows = f.numel() // C
    if f.is_cuda:
        rpb = _rpb(rows)
        df = torch.empty_like(f)
        pcol = torch.empty(-(-rows // rpb), C, device=f.device, dtype=torch.float32)
        _native.call("be_gelu_bwd", _native.ptr(dg.contiguous()), _native.ptr(f), _native.ptr(bias.float().contiguous()),
                     _native.ptr(df), _native.ptr(pcol), rows, C, rpb, _native.stream(f.device))
        return df, _colsum(pcol, out_db)
    t = f.float() + bias.float()
    d = 0.5 * (1 + torch.erf(t / math.sqrt(2))) + t * torch.exp(-0.5 * t * t) / math.sqrt(2 * math.pi)
    df = dg.float() * d
    return df.to(f.dtype), _colsum(df.reshape(rows, C), out_db)


def scale_cast(x: torch.Tensor, rs: torch.Tensor | None = None, rpn: int = 1, dtype=torch.bfloat16,
               out_col: torch.Tensor | None = None):
    """(rs[row // rpn] * x in ``dtype``, column sums of it in fp32)."""
    C = x.shape[-1]
    rows = x.numel() // C
    if x.is_cuda:
        rpb = _rpb(rows)
        y = torch.empty(x.shape, device=x.device, dtype=torch.bfloat16)
        pcol = torch.empty(-(-rows // rpb), C, device=x.device, dtype=torch.float32)
        _native.call("be_scale_cast", _native.ptr(x.float().contiguous()),
                     _native.ptr(rs.float().contiguous() if rs is not None else None), int(rpn), _native.ptr(y),
                     _native.ptr(pcol), rows, C, rpb, _native.stream(x.device))
        return y, _colsum(pcol, out_col)
    sc = _rowscale(rs, rows, rpn)
    yf = x.float().reshape(rows, C)
    if sc is not None:
        yf = yf * sc
    return yf.to(dtype).reshape(x.shape), _colsum(yf, out_col)


# ------------------------------------------------------------------ attention
def attn_fwd(q, k, v, scale: float, rel_h=None, rel_w=None):
    """(out [B, N, H, 64], lse [B, H, N] natural log).  q/k/v [B, N, H, 64]."""
    if q.is_cuda:
        from .transformer import _attn_fwd_hip

        return _attn_fwd_hip(q, k, v, scale, rel_h, rel_w, want_lse=True)
    qf, kf, vf = (t.float().permute(0, 2, 1, 3) for t in (q, k, v))
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if rel_h is not None:
        B, H, N, Hg = rel_h.shape
        s = s + (rel_h.float()[..., :, None] + rel_w.float()[..., None, :]).reshape(B, H, N, -1)
    lse = torch.logsumexp(s, -1)
    o = torch.matmul(torch.exp(s - lse[..., None]), vf).permute(0, 2, 1, 3)
    return o.to(q.dtype).contiguous(), lse


def attn_bwd(q, k, v, o, do, lse, scale: float, rel_h=None, rel_w=None, dk=None, dv=None):
    """Flash-attention backward.  q/k/v [B, N, H, 64] (views of a packed qkv are fine), o / do
    [B, N, H, 64] contiguous, lse [B, H, N].  Returns (dq fp32 [B, N, H, 64], dk, dv, drel_h, drel_w);
    ``dk``/``dv`` may be passed in as views of a packed gradient buffer (written in place)."""
    B, N, H, D = q.shape
    if q.is_cuda:
        assert D == 64 and q.stride() == k.stride() == v.stride() and q.stride(-1) == 1
        o = o.contiguous()
        do = do.contiguous().to(torch.bfloat16)
        dq = torch.empty(B, N, H, D, device=q.device, dtype=torch.float32)
        if dk is None:
            dk = torch.empty(B, N, H, D, device=q.device, dtype=torch.bfloat16)
        if dv is None:
            dv = torch.empty(B, N, H, D, device=q.device, dtype=torch.bfloat16)
        assert dk.stride() == dv.stride() and dk.stride(-1) == 1
        delta = torch.empty(B * H * N, device=q.device, dtype=torch.float32)
        Hg = Wg = 0
        rh = rw = drh = drw = None
        if rel_h is not None:
            Hg, Wg = rel_h.shape[-1], rel_w.shape[-1]
            rh, rw = rel_h.float().contiguous(), rel_w.float().contiguous()
            drh, drw = torch.empty_like(rh), torch.empty_like(rw)
        _native.call("be_attn_bwd", _native.ptr(q), _native.ptr(k), _native.ptr(v), q.stride(1), q.stride(2),
                     q.stride(0), _native.ptr(o), _native.ptr(do), o.stride(1), o.stride(2), o.stride(0),
                     _native.ptr(lse.contiguous()), _native.ptr(delta), _native.ptr(rh), _native.ptr(rw), Hg, Wg,
                     _native.ptr(dq), _native.ptr(drh), _native.ptr(drw), _native.ptr(dk), _native.ptr(dv),
                     dk.stride(1), dk.stride(2), dk.stride(0), B, H, N, D, float(scale), 0, _native.stream(q.device))
        return dq, dk, dv, drh, drw
    qf, kf, vf = (t.float().permute(0, 2, 1, 3) for t in (q, k, v))
    of, gf = o.float().permute(0, 2, 1, 3), do.float().permute(0, 2, 1, 3)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if rel_h is not None:
        s = s + (rel_h.float()[..., :, None] + rel_w.float()[..., None, :]).reshape(B, H, N, -1)
    p = torch.exp(s - lse[..., None].float())
    dvf = torch.matmul(p.transpose(-1, -2), gf)
    dp = torch.matmul(gf, vf.transpose(-1, -2))
    ds = p * (dp - (gf * of).sum(-1, keepdim=True))
    dqf = torch.matmul(ds, kf) * scale
    dkf = torch.matmul(ds.transpose(-1, -2), qf) * scale
    drh = drw = None
    if rel_h is not None:
        ds5 = ds.reshape(B, H, N, rel_h.shape[-1], rel_w.shape[-1])
        drh, drw = ds5.sum(-1), ds5.sum(-2)
    back = lambda t: t.permute(0, 2, 1, 3)
    dkt, dvt = back(dkf).to(k.dtype), back(dvf).to(v.dtype)
    if dk is not None:
        dk.copy_(dkt)
        dv.copy_(dvt)
    else:
        dk, dv = dkt, dvt
    return back(dqf).contiguous(), dk, dv, drh, drw


# ---------------------------------------------------------------------------- SAM rel-pos terms
def relpos_fwd_ref(q, Rh, Rw):
    """q [B, N, H, c] (N = g*g), Rh / Rw [g, g, c] -> rel_h, rel_w [B, H, N, g] fp32 (oracle)."""
    B, N, H, c = q.shape
    g = Rh.shape[0]
    q5 = q.float().reshape(B, g, g, H, c)
    rh = torch.einsum("byxhc,ykc->bhyxk", q5, Rh.float()).reshape(B, H, N, g)
    rw = torch.einsum("byxhc,xkc->bhyxk", q5, Rw.float()).reshape(B, H, N, g)
    return rh.contiguous(), rw.contiguous()


def _rel_table_idx(g: int, device) -> torch.Tensor:
    ar = torch.arange(g, device=device)
    return (ar[:, None] - ar[None, :] + (g - 1)).long()


def relpos_fwd(q, tab_h, tab_w):
    """rel_h / rel_w from the [2g-1, c] rel-pos TABLES (get_rel_pos gather done inside the kernel) on
    MFMA (``relpos.hip``) for the 32 x 32 grid / head_dim 64; torch oracle otherwise."""
    B, N, H, c = q.shape
    g = (tab_h.shape[0] + 1) // 2
    if not (q.is_cuda and g == 32 and c == 64 and N == g * g and q.dtype == torch.bfloat16 and q.stride(-1) == 1):
        idx = _rel_table_idx(g, tab_h.device)
        return relpos_fwd_ref(q, tab_h[idx], tab_w[idx])
    rh = torch.empty(B, H, N, g, device=q.device, dtype=torch.float32)
    rw = torch.empty_like(rh)
    _native.call("be_relpos_fwd", _native.ptr(q), q.stride(1), q.stride(2), q.stride(0),
                 _native.ptr(tab_h.float().contiguous()), _native.ptr(tab_w.float().contiguous()), _native.ptr(rh),
                 _native.ptr(rw), B, H, g, c, _native.stream(q.device))
    return rh, rw


def relpos_bwd_ref(q, Rh, Rw, drh, drw):
    """-> (dq_rel [B, N, H, c] fp32, dRh [g, g, c], dRw [g, g, c]) (oracle)."""
    B, N, H, c = q.shape
    g = Rh.shape[0]
    q5 = q.float().reshape(B, g, g, H, c)
    dh = drh.float().reshape(B, H, g, g, g)
    dw = drw.float().reshape(B, H, g, g, g)
    dq = torch.einsum("bhyxk,ykc->byxhc", dh, Rh.float()) + torch.einsum("bhyxk,xkc->byxhc", dw, Rw.float())
    dRh = torch.einsum("bhyxk,byxhc->ykc", dh, q5)
    dRw = torch.einsum("bhyxk,byxhc->xkc", dw, q5)
    return dq.reshape(B, N, H, c), dRh, dRw


def relpos_bwd_(q, tab_h, tab_w, drh, drw, dq, out_q, grad_rh, grad_rw, rel_idx):
    """Fused backward of the rel-pos terms (tables ``tab_h`` / ``tab_w`` [2g-1, c]): ``out_q`` (bf16
    view, e.g. the q slot of a packed dqkv gradient) = dq + dq_rel; ``grad_rh`` / ``grad_rw`` (the
    table gradients) overwritten with the gathered dRh / dRw (rel_idx [g, g] = y - k + g - 1).
    ``dq`` (fp32) is clobbered."""
    B, N, H, c = q.shape
    g = rel_idx.shape[0]
    if q.is_cuda and g == 32 and c == 64 and N == g * g and q.stride(-1) == 1 and dq.stride(-1) == 1 \
            and out_q.stride(-1) == 1 and grad_rh.is_contiguous() and grad_rw.is_contiguous():
        _native.call("be_relpos_bwd", _native.ptr(drh), _native.ptr(drw), _native.ptr(tab_h.float().contiguous()),
                     _native.ptr(tab_w.float().contiguous()), _native.ptr(dq), dq.stride(1), dq.stride(2), dq.stride(0),
                     _native.ptr(out_q), out_q.stride(1), out_q.stride(2), out_q.stride(0), _native.ptr(q),
                     q.stride(1), q.stride(2), q.stride(0), _native.ptr(grad_rh), _native.ptr(grad_rw), B, H, g, c,
                     _native.stream(q.device))
        return
    dq_rel, dRh, dRw = relpos_bwd_ref(q, tab_h[rel_idx], tab_w[rel_idx], drh, drw)
    out_q.copy_((dq.float() + dq_rel).to(out_q.dtype))
    for dR, out in ((dRh, grad_rh), (dRw, grad_rw)):
        out.zero_()
        out.index_add_(0, rel_idx.reshape(-1), dR.reshape(-1, dR.shape[-1]).to(out.dtype))
