"""Per-shape choice between the in-house bf16 MFMA GEMM (:mod:`.gemm_bf16`) and the library GEMM
(:mod:`.gemm`, hipBLASLt through PyTorch) for the CPSAM training engine.

Neither wins everywhere (``profiles/r04/gemm/``): the in-house kernel with its fused epilogues is
faster on the weight gradients at batch 1 and on the square 1024x1024 projections, the library on
the large forward / data-gradient shapes at batch 8.  The first EAGER call of each (op, shape) runs
both implementations (HIP-event median of 3, after one warm-up each), keeps the faster and writes its
result last; later calls -- and every call inside a HIP-graph capture, whose shapes the eager
warm-up steps of the engine have already decided -- go straight to the winner.  ``BE_GEMM_AUTO=hip``
/ ``lib`` pins one side (A/B), and :func:`choices` reports the table."""
from __future__ import annotations

import os

import torch

from . import gemm as lib
from . import gemm_bf16 as hip

_choice: dict = {}


def _capturing() -> bool:
    try:
        return torch.cuda.is_current_stream_capturing()
    except Exception:  # noqa: BLE001
        return False


def _time(fn, reps: int = 3) -> float:
    fn()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def _pick(key, f_hip, f_lib):
    mode = os.environ.get("BE_GEMM_AUTO", "auto")
    if mode == "hip":
        return f_hip()
    if mode == "lib":
        return f_lib()
    c = _choice.get(key)
    if c is None:
        if _capturing() or not torch.cuda.is_available():
            return f_lib()
        th, tl = _time(f_hip), _time(f_lib)
        c = _choice[key] = ("hip", th, tl) if th < tl else ("lib", th, tl)
    return f_hip() if c[0] == "hip" else f_lib()


def linear(x, w, b=None):
    if not x.is_cuda:
        return hip.linear(x, w, b)
    return _pick(("linear", tuple(x.shape), tuple(w.shape), b is not None), lambda: hip.linear(x, w, b),
                 lambda: lib.linear(x, w, b))


def linear_gelu(x, w, b):
    if not x.is_cuda:
        return hip.linear_gelu(x, w, b)
    return _pick(("linear_gelu", tuple(x.shape), tuple(w.shape)), lambda: hip.linear_gelu(x, w, b),
                 lambda: lib.linear_gelu(x, w, b))


def mm(x, w):
    if not x.is_cuda:
        return hip.mm(x, w)
    return _pick(("mm", tuple(x.shape), tuple(w.shape)), lambda: hip.mm(x, w), lambda: lib.mm(x, w))


def mm_dgelu(dm, w2, f, out_db=None):
    if not dm.is_cuda:
        return hip.mm_dgelu(dm, w2, f, out_db=out_db)
    return _pick(("mm_dgelu", tuple(dm.shape), tuple(w2.shape)), lambda: hip.mm_dgelu(dm, w2, f, out_db=out_db),
                 lambda: lib.mm_dgelu(dm, w2, f, out_db=out_db))


def wgrad(dy, x, out):
    if not dy.is_cuda:
        return hip.wgrad(dy, x, out)
    return _pick(("wgrad", tuple(dy.shape), tuple(x.shape)), lambda: hip.wgrad(dy, x, out),
                 lambda: lib.wgrad(dy, x, out))


def choices() -> list[dict]:
    """The decided table: one row per (op, shapes) with both timings (ms)."""
    return [{"op": k[0], "shapes": [list(s) for s in k[1:3]], "impl": v[0], "hip_ms": round(v[1], 4),
             "lib_ms": round(v[2], 4)} for k, v in _choice.items()]
