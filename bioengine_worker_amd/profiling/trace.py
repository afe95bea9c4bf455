"""Request tracing → Chrome trace JSON (SURVEY.md §5 "Tracing / profiling": the reference has only
ad-hoc timing logs; the rebuild records per-request spans — router queue, replica call, batch,
kernels, post-processing — and exports them for chrome://tracing / Perfetto).

* :func:`span` — context manager (sync and async code) recording a complete event ("ph": "X") on
  the current process/thread with the current request id attached.
* GPU stages: ``span(..., cuda=True)`` additionally brackets the block with HIP events on the
  current stream and records the device time as a separate "gpu" track (resolved lazily when the
  trace is exported, so tracing never adds a device synchronisation to the hot path).
* :func:`request` — starts a request scope (id propagated through ``contextvars`` into spawned
  tasks and threads started with ``contextvars.copy_context``).

Enable with ``BIOENGINE_TRACE=1`` (or :func:`enable`); export with :func:`export` /
``BIOENGINE_TRACE_FILE=path.json`` (written at interpreter exit).  Disabled tracing costs one
attribute check per span.
"""
from __future__ import annotations

import atexit
import contextlib
import contextvars
import itertools
import json
import os
import threading
import time
from typing import Any

from ..runtime import faults as _faults

_enabled = os.environ.get("BIOENGINE_TRACE", "0") not in ("0", "", "false")
_events: list[dict] = []
_gpu_pending: list = []
_lock = threading.Lock()
_req = contextvars.ContextVar("bioengine_request_id", default=None)
_ids = itertools.count(1)
_t0 = time.perf_counter()
MAX_EVENTS = 1_000_000


def enable(on: bool = True) -> None:
    global _enabled
    _enabled = on


def enabled() -> bool:
    return _enabled


def clear() -> None:
    with _lock:
        _events.clear()
        _gpu_pending.clear()


def _us(t: float) -> float:
    return (t - _t0) * 1e6


@contextlib.contextmanager
def request(name: str = "request", **args):
    """Request scope: every span inside carries the same ``req`` id."""
    if not _enabled:
        yield None
        return
    rid = f"r{next(_ids)}"
    tok = _req.set(rid)
    try:
        with span(name, cat="request", **args):
            yield rid
    finally:
        _req.reset(tok)


@contextlib.contextmanager
def span(name: str, cat: str = "stage", cuda: bool = False, **args):
    _faults.point(name)  # stage boundary: deadline check + fault-injection hook (runtime/faults.py)
    if not _enabled:
        yield
        return
    ev_start = ev_end = None
    if cuda:
        try:
            import torch

            if torch.cuda.is_available():
                ev_start = torch.cuda.Event(enable_timing=True)
                ev_end = torch.cuda.Event(enable_timing=True)
                ev_start.record()
        except Exception:  # noqa: BLE001
            ev_start = None
    t = time.perf_counter()
    try:
        yield
    finally:
        dur = time.perf_counter() - t
        rid = _req.get()
        a = dict(args)
        if rid:
            a["req"] = rid
        ev = {"name": name, "cat": cat, "ph": "X", "ts": _us(t), "dur": dur * 1e6, "pid": os.getpid(),
              "tid": threading.get_ident() % 100000, "args": a}
        with _lock:
            if len(_events) < MAX_EVENTS:
                _events.append(ev)
            if ev_start is not None:
                ev_end.record()
                _gpu_pending.append((name, ev["ts"], ev_start, ev_end, a))


def instant(name: str, **args) -> None:
    if not _enabled:
        return
    with _lock:
        _events.append({"name": name, "ph": "i", "s": "p", "ts": _us(time.perf_counter()), "pid": os.getpid(),
                        "tid": threading.get_ident() % 100000, "args": args})


def counter(name: str, **values) -> None:
    if not _enabled:
        return
    with _lock:
        _events.append({"name": name, "ph": "C", "ts": _us(time.perf_counter()), "pid": os.getpid(), "args": values})


def _resolve_gpu() -> list[dict]:
    out = []
    pend = list(_gpu_pending)
    _gpu_pending.clear()
    for name, ts, s, e, a in pend:
        try:
            e.synchronize()
            ms = s.elapsed_time(e)
        except Exception:  # noqa: BLE001
            continue
        out.append({"name": name, "cat": "gpu", "ph": "X", "ts": ts, "dur": ms * 1e3, "pid": os.getpid(),
                    "tid": "gpu", "args": dict(a, device_ms=round(ms, 4))})
    return out


def events() -> list[dict]:
    with _lock:
        gpu = _resolve_gpu()
        _events.extend(gpu)
        return list(_events)


def export(path: str | None = None) -> dict[str, Any]:
    """Chrome trace document; written to ``path`` when given."""
    doc = {"traceEvents": events(), "displayTimeUnit": "ms",
           "otherData": {"producer": "bioengine-worker-amd", "pid": os.getpid()}}
    if path:
        with open(path, "w") as f:
            json.dump(doc, f)
    return doc


def summary() -> dict[str, dict]:
    """Per-span-name count / total / mean / p50 / p95 (ms) — the router-metrics view of a trace."""
    by: dict[str, list[float]] = {}
    for e in events():
        if e.get("ph") == "X":
            by.setdefault(f"{e.get('cat')}:{e['name']}", []).append(e["dur"] / 1e3)
    out = {}
    for k, v in by.items():
        s = sorted(v)
        out[k] = {"count": len(s), "total_ms": round(sum(s), 3), "mean_ms": round(sum(s) / len(s), 4),
                  "p50_ms": round(s[len(s) // 2], 4), "p95_ms": round(s[min(len(s) - 1, int(0.95 * (len(s) - 1)))], 4)}
    return out


if os.environ.get("BIOENGINE_TRACE_FILE"):
    # "{pid}" in the path gives every process (router, replicas) its own file
    atexit.register(lambda: export(os.environ["BIOENGINE_TRACE_FILE"].replace("{pid}", str(os.getpid()))))
