"""Per-replica execution context (``serve.get_replica_context()``), multiplexed model id, and
per-replica log capture.

Several in-process replicas share one interpreter, so the "current replica" is a ContextVar set
around ``__init__`` and every request.  Output written while a replica is current (print, logging)
is copied into that replica's ring buffer, which ``get_app_status(logs_tail=...)`` reports
(reference surfaces per-replica Ray logs: ``bioengine/cluster/proxy_actor.py:563-738``).
"""
from __future__ import annotations

import collections
import contextvars
import io
import logging
import sys
import threading
from dataclasses import dataclass, field


@dataclass
class ReplicaContext:
    app_name: str
    deployment: str
    replica_tag: str
    servable_object: object = None
    gpu_ids: list = field(default_factory=list)

    @property
    def replica_id(self):  # newer Ray API
        return _ReplicaID(self.replica_tag, self.deployment, self.app_name)


@dataclass
class _ReplicaID:
    unique_id: str
    deployment_name: str
    app_name: str

    def __str__(self):
        return self.unique_id


_current: contextvars.ContextVar[ReplicaContext | None] = contextvars.ContextVar("be_replica", default=None)
_model_id: contextvars.ContextVar[str] = contextvars.ContextVar("be_model_id", default="")
_buffers: dict[str, collections.deque] = {}
_buf_lock = threading.Lock()
_installed = False


def get_replica_context() -> ReplicaContext:
    ctx = _current.get()
    if ctx is None:
        raise RuntimeError("`serve.get_replica_context()` may only be called from within a deployment replica")
    return ctx


def current() -> ReplicaContext | None:
    return _current.get()


def set_current(ctx: ReplicaContext | None):
    return _current.set(ctx)


def reset_current(token):
    _current.reset(token)


def get_multiplexed_model_id() -> str:
    return _model_id.get()


def set_model_id(mid: str):
    return _model_id.set(mid or "")


def reset_model_id(tok):
    _model_id.reset(tok)


def log_buffer(tag: str, maxlen: int = 5000) -> collections.deque:
    with _buf_lock:
        if tag not in _buffers:
            _buffers[tag] = collections.deque(maxlen=maxlen)
        return _buffers[tag]


def drop_log_buffer(tag: str, keep: bool = True):
    if not keep:
        with _buf_lock:
            _buffers.pop(tag, None)


class _Tee(io.TextIOBase):
    def __init__(self, orig):
        self.orig = orig
        self._partial: dict[str, str] = {}

    def write(self, s):
        ctx = _current.get()
        if ctx is not None:
            buf = log_buffer(ctx.replica_tag)
            pending = self._partial.get(ctx.replica_tag, "") + s
            *lines, rest = pending.split("\n")
            buf.extend(lines)
            self._partial[ctx.replica_tag] = rest
        return self.orig.write(s)

    def flush(self):
        return self.orig.flush()

    def isatty(self):
        return False

    def fileno(self):
        return self.orig.fileno()


class _ReplicaLogHandler(logging.Handler):
    def emit(self, record):
        ctx = _current.get()
        if ctx is not None:
            try:
                log_buffer(ctx.replica_tag).append(self.format(record))
            except Exception:
                pass


def install_log_capture():
    global _installed
    if _installed:
        return
    _installed = True
    sys.stdout = _Tee(sys.stdout)
    sys.stderr = _Tee(sys.stderr)
    h = _ReplicaLogHandler()
    h.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s - %(message)s"))
    logging.getLogger().addHandler(h)
    logging.getLogger("ray.serve").addHandler(h)
    logging.getLogger("ray.serve").setLevel(logging.INFO)
