"""Per-shape choice between the in-house bf16 MFMA GEMMs -- the two-barrier kernel
(:mod:`.gemm_bf16`, small tiles, best at batch 1) and the ping-pong kernel (:mod:`.gemm_pp`, large
tiles, staggered wave groups, best at large M) -- and the library GEMM (:mod:`.gemm`, hipBLASLt
through PyTorch) for the CPSAM training engine.

None wins everywhere (``profiles/r04/gemm/``).  The first EAGER call of each (op, shape) runs every
eligible implementation (median of 3 replays of a HIP graph of 10 calls, after one warm-up each:
kernel time, not launch overhead), keeps the fastest and
writes its result last; later calls -- and every call inside a HIP-graph capture, whose shapes the
eager warm-up steps of the engine have already decided -- go straight to the winner.
``BE_GEMM_AUTO=hip`` / ``pp`` / ``lib`` pins one side (A/B), and :func:`choices` reports the table."""
from __future__ import annotations

import os

import torch

from . import gemm as lib
from . import gemm_bf16 as hip
from . import gemm_pp as pp

_choice: dict = {}


def _capturing() -> bool:
    try:
        return torch.cuda.is_current_stream_capturing()
    except Exception:  # noqa: BLE001
        return False


def _time(fn, reps: int = 10) -> float:
    """GPU time of one call, in ms.  The calls are captured into a HIP graph and replayed, so the
    figure is kernel time: bracketing single eager launches with events (the first version) timed
    the host launch path instead -- ~40 us per call against ~17-22 us on the GPU at batch 1 -- and
    picked kernels that then lost inside the graphed step (profiles/r04/cpsam/)."""
    fn()
    torch.cuda.synchronize()
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        ts = []
        for _ in range(3):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            g.replay()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) / reps)
        del g
    except Exception:  # noqa: BLE001  (a path that cannot be captured: time it eagerly)
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                fn()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) / reps)
    ts.sort()
    return ts[len(ts) // 2]


def _pick(key, cands: dict):
    """cands: name -> zero-arg callable (ineligible implementations left out)."""
    mode = os.environ.get("BE_GEMM_AUTO", "auto")
    if mode in cands:
        return cands[mode]()
    if mode != "auto":
        return cands["lib"]()
    c = _choice.get(key)
    if c is None:
        if _capturing() or not torch.cuda.is_available():
            return cands["lib"]()
        t = {name: _time(fn) for name, fn in cands.items()}
        best = min(t, key=t.get)
        c = _choice[key] = (best, t)
    return cands[c[0]]()


def linear(x, w, b=None):
    if not x.is_cuda:
        return hip.linear(x, w, b)
    M, K = x.shape
    c = {"hip": lambda: hip.linear(x, w, b), "lib": lambda: lib.linear(x, w, b)}
    if pp.supported(M, w.shape[0], K) and M >= 2048:
        c["pp"] = lambda: pp.linear(x, w, b)
    return _pick(("linear", tuple(x.shape), tuple(w.shape), b is not None), c)


def linear_gelu(x, w, b):
    if not x.is_cuda:
        return hip.linear_gelu(x, w, b)
    M, K = x.shape
    c = {"hip": lambda: hip.linear_gelu(x, w, b), "lib": lambda: lib.linear_gelu(x, w, b)}
    if pp.supported(M, w.shape[0], K) and M >= 2048:
        c["pp"] = lambda: pp.linear_gelu(x, w, b)
    return _pick(("linear_gelu", tuple(x.shape), tuple(w.shape)), c)


def mm(x, w):
    if not x.is_cuda:
        return hip.mm(x, w)
    M, K = x.shape
    N = w.shape[1]
    c = {"hip": lambda: hip.mm(x, w), "lib": lambda: lib.mm(x, w)}
    if pp.supported(M, N, K) and M >= 2048 and N % pp.TILES[pp._dgrad_cfg(M, N, None)][1] == 0:
        c["pp"] = lambda: pp.mm(x, w)
    return _pick(("mm", tuple(x.shape), tuple(w.shape)), c)


def mm_dgelu(dm, w2, f, out_db=None):
    if not dm.is_cuda:
        return hip.mm_dgelu(dm, w2, f, out_db=out_db)
    M, K = dm.shape
    N = w2.shape[1]
    c = {"hip": lambda: hip.mm_dgelu(dm, w2, f, out_db=out_db), "lib": lambda: lib.mm_dgelu(dm, w2, f, out_db=out_db)}
    if pp.supported(M, N, K) and M >= 2048 and N % pp.TILES[pp._dgrad_cfg(M, N, None)][1] == 0:
        c["pp"] = lambda: pp.mm_dgelu(dm, w2, f, out_db=out_db)
    return _pick(("mm_dgelu", tuple(dm.shape), tuple(w2.shape)), c)


def wgrad(dy, x, out):
    if not dy.is_cuda:
        return hip.wgrad(dy, x, out)
    m, n = dy.shape
    k = x.shape[1]
    c = {"hip": lambda: hip.wgrad(dy, x, out), "lib": lambda: lib.wgrad(dy, x, out)}
    cfg = 0 if n >= 2048 else 2
    bm, bn = pp.TILES[cfg]
    if n % bm == 0 and k % bn == 0 and m % 32 == 0 and dy.is_contiguous() and x.is_contiguous():
        c["pp"] = lambda: pp.wgrad(dy, x, out)
    return _pick(("wgrad", tuple(dy.shape), tuple(x.shape)), c)


def choices() -> list[dict]:
    """The decided table: one row per (op, shapes) with every candidate's timing (ms)."""
    return [{"op": k[0], "shapes": [list(s) for s in k[1:3]], "impl": v[0],
             **{f"{name}_ms": round(t, 4) for name, t in v[1].items()}} for k, v in _choice.items()]
