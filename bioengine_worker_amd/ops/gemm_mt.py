"""Macro-tile bf16 MFMA GEMMs (``csrc/kernels/gemm_mt.hip``) with the row-major helper surface of
:mod:`.gemm` (the library backend), so the Cellpose-SAM engines can run every linear layer on the
framework's own kernel:

* :func:`linear` -- ``x W^T (+ b)``; :func:`linear_res` -- ``x W^T + b + r`` (residual fused);
* :func:`linear_gelu` -- ``f = x W^T + b`` and ``g = gelu(f)`` from one epilogue;
* :func:`mm` -- ``x W`` (data gradient, W as stored); :func:`mm_dgelu` -- ``gelu'(f) * (dm W2)`` with
  the lin1 bias gradient (column sums) from the same epilogue;
* :func:`wgrad` -- ``dy^T x`` in fp32 straight into the parameter's view of the flat gradient buffer;
  split-K slices are summed inside the same launch (no separate slab-sum kernel).

The tile configuration of each call comes from a static table keyed by the GEMM's shape
(:data:`TABLE`, measured per shape on an MI355X: ``profiles/r05/gemm_mt/``), with a deterministic
fall-back rule for shapes outside it -- nothing is timed at run time, so the kernels a step runs are
the same on every box.  On CPU every helper is the fp32 PyTorch op of the same math.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _native

E_NONE, E_BIAS, E_BIAS_GELU, E_DGELU, E_F32, E_BIAS_RES = 0, 1, 2, 4, 5, 6
#: cfg -> (BM, BN): 0 256x256 (8 waves), 1 256x192 (8 waves, K-contiguous B only), 2 256x128,
#: 3 128x256, 4 128x128 (4 waves)
TILES = {0: (256, 256), 1: (256, 192), 2: (256, 128), 3: (128, 256), 4: (128, 128)}
NCU = 256

#: (kind, M, N, K) -> (cfg, split).  kind: "nt" forward, "nn" data gradient, "tn" weight gradient.
#: The fastest configuration per Cellpose-SAM shape in the per-shape sweep of tools/gemm_mt_bench.py
#: on an MI355X (profiles/r05/gemm/gemm_mt_sweep_s23.jsonl, graph-replayed, median of 5 rounds).
TABLE: dict = {
    ("nn", 1024, 1024, 1024): (4, 1), ("nn", 1024, 1024, 3072): (4, 1), ("nn", 1024, 1024, 4096): (4, 1),
    ("nn", 1024, 4096, 1024): (4, 1), ("nn", 8192, 1024, 1024): (2, 1), ("nn", 8192, 1024, 3072): (2, 1),
    ("nn", 8192, 1024, 4096): (2, 1), ("nn", 8192, 4096, 1024): (0, 1),
    ("nt", 1024, 1024, 1024): (4, 1), ("nt", 1024, 1024, 4096): (4, 1), ("nt", 1024, 3072, 1024): (4, 1),
    ("nt", 1024, 4096, 1024): (4, 1), ("nt", 8192, 1024, 1024): (2, 1), ("nt", 8192, 1024, 4096): (3, 1),
    ("nt", 8192, 3072, 1024): (1, 1), ("nt", 8192, 4096, 1024): (0, 1),
    ("tn", 1024, 1024, 1024): (4, 1), ("tn", 1024, 1024, 8192): (4, 4), ("tn", 1024, 4096, 1024): (4, 1),
    ("tn", 1024, 4096, 8192): (0, 4), ("tn", 3072, 1024, 1024): (4, 1), ("tn", 3072, 1024, 8192): (0, 5),
    ("tn", 4096, 1024, 1024): (4, 1), ("tn", 4096, 1024, 8192): (0, 4),
}


def _forced():
    v = os.environ.get("BE_GEMM_MT_CFG")
    if not v:
        return None
    c, _, sp = v.partition(",")
    return int(c), int(sp or 1)


def _valid(kind: str, cfg: int, M: int, N: int) -> bool:
    """M / N-contiguous operands (the data gradient's W, both weight-gradient operands) are staged in
    whole 16-byte chunks by power-of-two tile widths: M / N multiples of 8, no 192-wide tiles."""
    if kind == "nn":
        return cfg != 1 and N % 8 == 0
    if kind == "tn":
        return cfg != 1 and M % 8 == 0 and N % 8 == 0
    return True


def choose(kind: str, M: int, N: int, K: int) -> tuple[int, int]:
    """Tile configuration and split-K count of one GEMM: the static table, else the candidate with
    the fewest rounds of one-block-per-CU waves, larger tiles first (fewer bytes staged per FLOP)."""
    f = _forced()
    if f is not None:
        return f
    hit = TABLE.get((kind, M, N, K))
    if hit is not None:
        return hit
    best = None
    nkt = K // 64
    for cfg in (0, 1, 2, 3, 4):
        if not _valid(kind, cfg, M, N):
            continue
        bm, bn = TILES[cfg]
        tiles = -(-M // bm) * -(-N // bn)
        split = 1
        if kind == "tn":
            # split-K until the slices fill the chip, keeping >= 8 K-tiles per slice
            while tiles * split * 2 <= NCU and nkt // (split * 2) >= 8:
                split *= 2
        blocks = tiles * split
        rounds = -(-blocks // NCU)
        # work per CU in units of 128x128x64 tile-steps, plus a per-block fixed cost
        per_block = (bm * bn / 16384.0) * (nkt / split) + 6.0
        cost = rounds * per_block
        if best is None or cost < best[0] - 1e-9:
            best = (cost, cfg, split)
    return best[1], best[2]


_ws: dict = {}
_cnt: dict = {}


def _stream_key(dev: torch.device) -> tuple:
    """Split-K scratch is private to a (device, stream) pair: two split-K launches in flight on two
    streams (the CPSAM step's side-stream weight gradients beside a main-stream one) would otherwise
    overwrite each other's slabs and bump the same tile counters.  Work on ONE stream is ordered, so
    it can share."""
    return (dev.index, torch.cuda.current_stream(dev).cuda_stream)


def _workspace(dev: torch.device, nbytes: int) -> torch.Tensor:
    """fp32 split-K slab workspace, grown but never freed: a captured HIP graph keeps its address."""
    key = _stream_key(dev)
    cur = _ws.get(key)
    if cur is None or cur[-1].numel() * 4 < nbytes:
        t = torch.empty((nbytes + 3) // 4, device=dev, dtype=torch.float32)
        _ws.setdefault(key, []).append(t)
        cur = _ws[key]
    return cur[-1]


def _counters(dev: torch.device) -> torch.Tensor:
    key = _stream_key(dev)
    c = _cnt.get(key)
    if c is None:
        # per-tile arrival counters; the last arriving slice resets its tile's counter to 0
        c = _cnt[key] = torch.zeros(65536, device=dev, dtype=torch.int32)
    return c


def _bias(b: torch.Tensor | None):
    if b is None:
        return None, 0
    if not b.is_contiguous():
        b = b.contiguous()
    if b.dtype == torch.bfloat16:
        return b, 1
    if b.dtype != torch.float32:
        b = b.float()
    return b, 0


def _call(A, B, C, C2, bias, bias_bf16, aux, dbias, Cf, M, N, K, lda, ldb, ldc, ta, tb, epi, cfg, split, dev):
    ws = cnt = None
    ws_bytes = 0
    if split > 1:
        bm, bn = TILES[cfg]
        tiles = (-(-M // bm)) * (-(-N // bn))
        if tiles > 65536:
            raise ValueError("too many output tiles for the split-K arrival counters")
        ws_bytes = tiles * split * bm * bn * 4
        ws = _workspace(dev, ws_bytes)
        ws_bytes = ws.numel() * 4
        cnt = _counters(dev)
    _native.call("be_gemm_mt", _native.ptr(A), _native.ptr(B), _native.ptr(C), _native.ptr(C2), _native.ptr(bias),
                 int(bias_bf16), _native.ptr(aux), _native.ptr(dbias), _native.ptr(Cf), _native.ptr(ws), int(ws_bytes),
                 _native.ptr(cnt), M, N, K, lda, ldb, ldc, ta, tb, epi, cfg, split, _native.stream(dev))


def supported(M: int, N: int, K: int) -> bool:
    return K % 64 == 0 and N % 4 == 0


def _ok(*ts) -> bool:
    return all(t is None or (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous()) for t in ts)


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    """x [M, K] @ w [N, K]^T (+ b[N]) -> bf16 [M, N]."""
    M, K = x.shape
    N = w.shape[0]
    if not (x.is_cuda and _ok(x, w) and supported(M, N, K)):
        return F.linear(x, w, None if b is None else b.to(x.dtype))
    out = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    bb, bf = _bias(b)
    cfg, _ = choose("nt", M, N, K)
    _call(x, w, out, None, bb, bf, None, None, None, M, N, K, K, K, N, 0, 0, E_BIAS if b is not None else E_NONE,
          cfg, 1, x.device)
    return out


def linear_res(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None, r: torch.Tensor) -> torch.Tensor:
    """x [M, K] @ w [N, K]^T + b[N] + r [M, N] -> bf16 [M, N] (the residual add fused in the epilogue)."""
    M, K = x.shape
    N = w.shape[0]
    if not (x.is_cuda and _ok(x, w, r) and supported(M, N, K)):
        y = F.linear(x.float(), w.float(), None if b is None else b.float()) + r.float()
        return y.to(x.dtype)
    out = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    bb, bf = _bias(b)
    cfg, _ = choose("nt", M, N, K)
    _call(x, w, out, None, bb, bf, r, None, None, M, N, K, K, K, N, 0, 0, E_BIAS_RES, cfg, 1, x.device)
    return out


def linear_gelu(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """-> (g = gelu(f), f = x w^T + b), both bf16 [M, N]; g is the (erf) GELU of the bf16-rounded f."""
    M, K = x.shape
    N = w.shape[0]
    if not (x.is_cuda and _ok(x, w) and supported(M, N, K)):
        f = F.linear(x.float(), w.float(), b.float()).to(x.dtype)
        return F.gelu(f.float()).to(x.dtype), f
    f = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    g = torch.empty_like(f)
    bb, bf = _bias(b)
    cfg, _ = choose("nt", M, N, K)
    _call(x, w, f, g, bb, bf, None, None, None, M, N, K, K, K, N, 0, 0, E_BIAS_GELU, cfg, 1, x.device)
    return g, f


def linear_gelu_only(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """gelu(x w^T + b) bf16 [M, N] (inference: the pre-activation is not stored)."""
    M, K = x.shape
    N = w.shape[0]
    if not (x.is_cuda and _ok(x, w) and supported(M, N, K)):
        f = F.linear(x.float(), w.float(), b.float()).to(x.dtype)
        return F.gelu(f.float()).to(x.dtype)
    g = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    bb, bf = _bias(b)
    cfg, _ = choose("nt", M, N, K)
    _call(x, w, None, g, bb, bf, None, None, None, M, N, K, K, K, N, 0, 0, E_BIAS_GELU, cfg, 1, x.device)
    return g


def _gelu_grad(f: torch.Tensor) -> torch.Tensor:
    x = f.float()
    return 0.5 * (1.0 + torch.erf(x * 0.7071067811865476)) + x * torch.exp(-0.5 * x * x) * 0.3989422804014327


def mm(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """x [M, K] @ w [K, N] -> bf16 [M, N] (w read as stored: the data gradient's weight)."""
    M, K = x.shape
    N = w.shape[1]
    cfg, _ = choose("nn", M, N, K)
    if not (x.is_cuda and _ok(x, w) and supported(M, N, K) and _valid("nn", cfg, M, N)):
        return torch.mm(x, w)
    out = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    _call(x, w, out, None, None, 0, None, None, None, M, N, K, K, N, N, 0, 1, E_NONE, cfg, 1, x.device)
    return out


def mm_dgelu(dm: torch.Tensor, w2: torch.Tensor, f: torch.Tensor, out_db: torch.Tensor | None = None) -> torch.Tensor:
    """df = gelu'(f) * (dm @ w2) with dm [M, K], w2 [K, N], f [M, N]; out_db[N] (fp32) = column sums of
    df (written in place when given)."""
    M, K = dm.shape
    N = w2.shape[1]
    cfg, _ = choose("nn", M, N, K)
    if not (dm.is_cuda and _ok(dm, w2, f) and supported(M, N, K) and _valid("nn", cfg, M, N)):
        df = (_gelu_grad(f) * (dm.float() @ w2.float())).to(dm.dtype)
        if out_db is not None:
            torch.sum(df.float(), 0, out=out_db)
        return df
    df = torch.empty(M, N, device=dm.device, dtype=torch.bfloat16)
    if out_db is not None:
        out_db.zero_()
    _call(dm, w2, df, None, None, 0, f, out_db, None, M, N, K, K, N, N, 0, 1, E_DGELU, cfg, 1, dm.device)
    return df


def wgrad(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor) -> None:
    """out (fp32 [n, k], in place) = dy^T x with dy [m, n], x [m, k] (m = tokens)."""
    m, n = dy.shape
    k = x.shape[1]
    out2 = out.view(out.shape[0], -1)
    cfg, split = choose("tn", n, k, m)
    if not (dy.is_cuda and _ok(dy, x) and out2.is_contiguous() and out2.dtype == torch.float32
            and m % 64 == 0 and _valid("tn", cfg, n, k)):
        torch.mm(dy.t().to(out2.dtype), x.to(out2.dtype), out=out2)
        return
    _call(dy, x, None, None, None, 0, None, None, out2, n, k, m, n, k, k, 1, 1, E_F32, cfg, split, dy.device)
