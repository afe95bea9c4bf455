"""Failure detection and fault injection for the serving runtime (SURVEY.md §5 "Failure detection /
elastic recovery / fault injection"; the reference only has ``DemoDeployment.set_fail_health_check``,
``apps/demo-app/demo_deployment.py:232-237``).

* **Per-request deadlines** — :func:`deadline_scope` sets an absolute wall-clock deadline in a
  ``contextvar``; the router (``serve/controller.py``) derives one from the deployment's
  ``request_timeout_s`` (or the caller's), cancels the request when it passes (raising
  :class:`DeadlineExceeded`) and ships it to process replicas with the call, where every traced
  stage boundary (:func:`point`) re-checks it, so work past its deadline stops at the next stage.
* **Replica watchdog** — :class:`InflightTable` records each in-flight call with its deadline; a
  replica whose call overran its deadline by ``BIOENGINE_WATCHDOG_GRACE_S`` fails its health check
  and the controller replaces it (process replicas are killed, which also tears down a wedged HIP
  context).
* **GPU-hang watchdog** — :func:`gpu_wait` polls a HIP event with a timeout instead of a blocking
  ``synchronize``; :func:`gpu_probe` launches a tiny kernel on a private stream and waits on it,
  which the replica's built-in health check runs so a hung device marks the replica UNHEALTHY.
* **Fault injection** — :func:`inject` (or ``BIOENGINE_FAULTS``) arms rules ``stage-glob ->
  error | delay | hang | oom`` with a probability and a count; :func:`point` is called at every
  ``trace.span`` stage (router admission, replica call, cellpose tiles/cpnet/blend/masks, training
  augment/forward/backward/all-reduce/AdamW) and at replica call entry.

``BIOENGINE_FAULTS`` format: ``stage=kind[:prob[:count[:delay_s]]]`` items separated by ``;``,
e.g. ``replica.infer=error:1:2;cellpose.masks=delay:1:-1:0.5``.
"""
from __future__ import annotations

import contextlib
import contextvars
import fnmatch
import os
import random
import threading
import time
from dataclasses import dataclass, field


class InjectedFault(RuntimeError):
    """Raised by an armed ``error`` rule."""


class DeadlineExceeded(TimeoutError):
    """The request's deadline passed (router timeout or a stage boundary after it)."""


class GpuHangError(RuntimeError):
    """A HIP event did not complete within the watchdog timeout."""


# ---------------------------------------------------------------------------- deadlines
_deadline: contextvars.ContextVar[float | None] = contextvars.ContextVar("bioengine_deadline", default=None)


def current_deadline() -> float | None:
    """Absolute ``time.time()`` deadline of the current request, or None."""
    return _deadline.get()


def remaining() -> float | None:
    d = _deadline.get()
    return None if d is None else d - time.time()


@contextlib.contextmanager
def deadline_scope(timeout_s: float | None = None, deadline: float | None = None):
    """Tighten the current deadline to ``now + timeout_s`` / ``deadline`` (the earlier one wins)."""
    cands = [d for d in (_deadline.get(), deadline, None if timeout_s is None else time.time() + timeout_s)
             if d is not None]
    tok = _deadline.set(min(cands) if cands else None)
    try:
        yield _deadline.get()
    finally:
        _deadline.reset(tok)


def check_deadline(stage: str = "") -> None:
    d = _deadline.get()
    if d is not None and time.time() > d:
        raise DeadlineExceeded(f"deadline exceeded{' at ' + stage if stage else ''} "
                               f"({time.time() - d:.3f}s late)")


# ---------------------------------------------------------------------------- fault injection
@dataclass
class Rule:
    stage: str
    kind: str = "error"  # error | delay | hang | oom
    prob: float = 1.0
    count: int = -1  # remaining firings (-1 = unlimited)
    delay_s: float = 0.0
    fired: int = 0
    seed_rng: random.Random = field(default_factory=lambda: random.Random(0))


_rules: list[Rule] = []
_rules_lock = threading.Lock()
_active = False
KINDS = ("error", "delay", "hang", "oom")


def inject(stage: str, kind: str = "error", prob: float = 1.0, count: int = -1, delay_s: float = 0.0,
           seed: int = 0) -> Rule:
    """Arm a rule; ``stage`` is an fnmatch glob over stage names (``"cellpose.*"``)."""
    global _active
    if kind not in KINDS:
        raise ValueError(f"fault kind must be one of {KINDS}")
    r = Rule(stage, kind, float(prob), int(count), float(delay_s), seed_rng=random.Random(seed))
    with _rules_lock:
        _rules.append(r)
        _active = True
    return r


def clear() -> None:
    global _active
    with _rules_lock:
        _rules.clear()
        _active = False


def rules() -> list[Rule]:
    with _rules_lock:
        return list(_rules)


def _parse_env(spec: str) -> None:
    for item in filter(None, (s.strip() for s in spec.split(";"))):
        stage, _, rhs = item.partition("=")
        parts = rhs.split(":")
        inject(stage.strip(), parts[0] or "error", float(parts[1]) if len(parts) > 1 else 1.0,
               int(parts[2]) if len(parts) > 2 else -1, float(parts[3]) if len(parts) > 3 else 0.0)


def _fire(stage: str) -> Rule | None:
    with _rules_lock:
        for r in _rules:
            if r.count == 0 or not fnmatch.fnmatchcase(stage, r.stage):
                continue
            if r.prob < 1.0 and r.seed_rng.random() >= r.prob:
                continue
            if r.count > 0:
                r.count -= 1
            r.fired += 1
            return r
    return None


def point(stage: str) -> None:
    """Stage boundary: deadline check + fault-injection hook.  Costs two global reads when idle."""
    if _deadline.get() is not None:
        check_deadline(stage)
    if not _active:
        return
    r = _fire(stage)
    if r is None:
        return
    if r.kind == "error":
        raise InjectedFault(f"injected fault at {stage}")
    if r.kind == "oom":
        try:
            import torch

            raise torch.cuda.OutOfMemoryError(f"injected HIP out of memory at {stage}")
        except ImportError:  # pragma: no cover
            raise MemoryError(f"injected out of memory at {stage}") from None
    if r.kind == "delay":
        time.sleep(r.delay_s)
    elif r.kind == "hang":  # a wedged stage: sleeps until its deadline (or delay_s, or ~forever)
        end = time.time() + (r.delay_s if r.delay_s > 0 else 3600.0)
        while time.time() < end:
            d = _deadline.get()
            if d is not None and time.time() > d + _grace():
                break
            time.sleep(0.01)
    check_deadline(stage)


if os.environ.get("BIOENGINE_FAULTS"):
    _parse_env(os.environ["BIOENGINE_FAULTS"])


# ---------------------------------------------------------------------------- replica watchdog
def _grace() -> float:
    return float(os.environ.get("BIOENGINE_WATCHDOG_GRACE_S", "30"))


class InflightTable:
    """In-flight calls of one replica: ``{call id: (method, start, deadline)}``."""

    def __init__(self):
        self._calls: dict[int, tuple[str, float, float | None]] = {}
        self._ids = iter(range(1, 1 << 62))
        self._lock = threading.Lock()

    @contextlib.contextmanager
    def track(self, method: str, deadline: float | None):
        with self._lock:
            cid = next(self._ids)
            self._calls[cid] = (method, time.time(), deadline)
        try:
            yield cid
        finally:
            with self._lock:
                self._calls.pop(cid, None)

    def overdue(self, grace_s: float | None = None) -> list[tuple[str, float]]:
        """Calls past deadline + grace, as (method, seconds overdue)."""
        g = _grace() if grace_s is None else grace_s
        now = time.time()
        with self._lock:
            return [(m, now - d) for m, _, d in self._calls.values() if d is not None and now > d + g]

    def __len__(self) -> int:
        return len(self._calls)

    def check(self, grace_s: float | None = None) -> None:
        late = self.overdue(grace_s)
        if late:
            m, s = max(late, key=lambda x: x[1])
            raise RuntimeError(f"watchdog: call '{m}' is {s:.1f}s past its deadline (replica wedged)")


# ---------------------------------------------------------------------------- GPU watchdog
def gpu_wait(event=None, timeout_s: float = 60.0, stream=None) -> float:
    """Wait for ``event`` (recorded now on ``stream`` if None) by polling; returns seconds waited,
    raises :class:`GpuHangError` after ``timeout_s``.  Never blocks inside the HIP runtime, so the
    calling thread stays responsive to deadlines."""
    import torch

    if event is None:
        event = torch.cuda.Event()
        event.record(stream)
    t0 = time.perf_counter()
    spin_until = t0 + 0.002
    sleep = 50e-6
    while not event.query():
        now = time.perf_counter()
        if now - t0 > timeout_s:
            raise GpuHangError(f"GPU work did not complete within {timeout_s:.1f}s")
        if now > spin_until:
            time.sleep(sleep)
            sleep = min(sleep * 2, 0.01)
    return time.perf_counter() - t0


_probe_streams: dict = {}


def gpu_probe(device=None, timeout_s: float = 10.0) -> float:
    """Launch a one-element kernel on a private stream of ``device`` and wait for it with the
    watchdog; returns the round-trip seconds (raises :class:`GpuHangError`)."""
    import torch

    dev = torch.device("cuda", torch.cuda.current_device() if device is None else torch.device(device).index or 0)
    s = _probe_streams.get(dev.index)
    if s is None:
        s = _probe_streams[dev.index] = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):
        x = torch.ones(1, device=dev)
        x.add_(1)
        ev = torch.cuda.Event()
        ev.record(s)
    return gpu_wait(ev, timeout_s)
