"""Continuous request batching inside a replica (``@serve.batch``).

Requests arriving one at a time (each RPC carries one image) are coalesced into batches for the
GPU.  Unlike a fixed-window batcher this loop is *continuous*: while a batch is executing, new
requests queue; the instant the device frees up the next batch is formed from everything queued
(up to ``max_batch_size``).  The ``batch_wait_timeout_s`` window is only spent when the device is
idle and the queue is short — so latency at low load stays ~one batch-of-1, and throughput at high
load approaches the full-batch rate.  The reference has no cross-request batching at all
(model-runner runtime ``max_ongoing_requests=1``, ``apps/model-runner/runtime_deployment.py:40``).

With ``max_concurrent_batches=2`` a second batch is dispatched only when a FULL batch is queued, so
at saturation the host side of one batch overlaps the GPU side of the next while moderate load
still forms one well-filled batch at a time.

Per-batch statistics (size histogram, queue wait) are kept for router metrics.
"""
from __future__ import annotations

import asyncio
import collections
import contextvars
import functools
import inspect
import os
import time

_current: contextvars.ContextVar = contextvars.ContextVar("bioengine_batch", default=None)


class _BatchQueue:
    def __init__(self, fn, owner, max_batch_size: int, timeout: float, max_concurrent_batches: int):
        self.fn = fn
        self.owner = owner
        self.max_batch_size = max_batch_size
        self.timeout = timeout
        self.queue: collections.deque = collections.deque()
        self.event = asyncio.Event()
        self.sem = asyncio.Semaphore(max_concurrent_batches)
        self.inflight = 0
        self.task = asyncio.get_running_loop().create_task(self._loop())
        self.stats = {"batches": 0, "requests": 0, "hist": collections.Counter(), "wait_s": 0.0}
        self.gap_ewma = float("inf")  # smoothed inter-arrival time (s)
        self.last_batch = 1
        self._last_arrival = None

    def submit(self, args, kwargs) -> asyncio.Future:
        fut = asyncio.get_running_loop().create_future()
        now = time.perf_counter()
        if self._last_arrival is not None:
            gap = now - self._last_arrival
            self.gap_ewma = gap if self.gap_ewma == float("inf") else 0.8 * self.gap_ewma + 0.2 * gap
        self._last_arrival = now
        self.queue.append((args, kwargs, fut, now))
        self.event.set()
        return fut

    def fill_target(self) -> int:
        """How many requests an idle device waits for (at most ``batch_wait_timeout_s``).

        * Requests arriving faster than half the timeout (open-loop load): a full batch.
        * Otherwise the previous batch's size: clients whose results just went out are on their way
          back (closed loop), so forming a batch from the one request that slipped in meanwhile
          would alternate 1-image and N-image batches.
        * A lone client never waits: a closed loop of one client with a fast service also arrives
          faster than half the timeout, but its batches stay at 1 (open-loop load grows the
          batch by itself, since requests queue while the device is busy)."""
        if self.last_batch > 1 and self.gap_ewma < 0.5 * self.timeout:
            return self.max_batch_size
        return min(self.max_batch_size, self.last_batch)

    async def _loop(self):
        while True:
            if not self.queue:
                self.event.clear()
                await self.event.wait()
            await self.sem.acquire()
            # A second concurrent batch only starts full: it overlaps the running batch's host work
            # (stacking, D2H, result encoding) at high load, but at moderate load two half-empty
            # batches would cost more GPU time than one full one.
            while self.inflight > 0 and len(self.queue) < self.max_batch_size:
                self.event.clear()
                await self.event.wait()
            # Device idle and queue short: give stragglers a bounded window to join.
            target = self.fill_target()
            if self.inflight == 0 and len(self.queue) < target and self.timeout > 0:
                deadline = time.perf_counter() + self.timeout
                while len(self.queue) < target:
                    rem = deadline - time.perf_counter()
                    if rem <= 0:
                        break
                    self.event.clear()
                    try:
                        await asyncio.wait_for(self.event.wait(), rem)
                    except asyncio.TimeoutError:
                        break
            items = []
            while self.queue and len(items) < self.max_batch_size:
                items.append(self.queue.popleft())
            if not items:
                self.sem.release()
                continue
            self.inflight += 1
            self.last_batch = len(items)
            asyncio.get_running_loop().create_task(self._run(items))

    async def _run(self, items):
        try:
            now = time.perf_counter()
            self.stats["batches"] += 1
            self.stats["requests"] += len(items)
            self.stats["hist"][len(items)] += 1
            self.stats["wait_s"] += sum(now - t for *_, t in items)
            nargs = len(items[0][0])
            cols = [[it[0][i] for it in items] for i in range(nargs)]
            kw = {}
            for k in items[0][1]:
                kw[k] = [it[1].get(k) for it in items]
            tok = _current.set((self, len(items)))
            try:
                res = self.fn(self.owner, *cols, **kw) if self.owner is not None else self.fn(*cols, **kw)
                if inspect.isawaitable(res):
                    res = await res
                res = list(res)
                if len(res) != len(items):
                    raise RuntimeError(f"batched function returned {len(res)} results for {len(items)} inputs")
                for (_, _, fut, _), r in zip(items, res):
                    if not fut.done():
                        if isinstance(r, BaseException):  # a per-request failure inside the batch
                            fut.set_exception(r)
                        else:
                            fut.set_result(r)
            except BaseException as e:  # noqa: BLE001
                for (_, _, fut, _) in items:
                    if not fut.done():
                        fut.set_exception(e)
            finally:
                _current.reset(tok)
        finally:
            self.inflight -= 1
            self.sem.release()
            self.event.set()  # wake a dispatcher waiting for a full queue or an idle device


#: ``BIOENGINE_BATCH_INLINE=0`` always offloads to a thread (A/B switch for :func:`offload`)
_INLINE = os.environ.get("BIOENGINE_BATCH_INLINE", "1") != "0"


async def offload(fn, *args, **kwargs):
    """Run blocking (GPU) work of a batched function.  A lone request on an idle queue -- batch of
    one, nothing queued behind it, no other batch in flight -- runs inline on the event loop: the
    two thread hand-offs of ``asyncio.to_thread`` are the largest serving cost left at concurrency
    1, and there is nothing for the loop to do meanwhile (a request arriving during the call
    would wait for the device anyway).  Everything else goes to a worker thread so the loop keeps
    forming the next batch."""
    cur = _current.get()
    if cur is not None and _INLINE:
        q, n = cur
        if n == 1 and not q.queue and q.inflight == 1:
            return fn(*args, **kwargs)
    return await asyncio.to_thread(fn, *args, **kwargs)


def batch(_func=None, *, max_batch_size: int = 10, batch_wait_timeout_s: float = 0.01, max_concurrent_batches: int = 1):
    def deco(fn):
        if not inspect.iscoroutinefunction(fn):
            raise TypeError("@serve.batch requires an async function")
        params = list(inspect.signature(fn).parameters)
        is_method = bool(params) and params[0] == "self"
        attr = f"__be_batch_{fn.__name__}"

        @functools.wraps(fn)
        async def wrapper(*args, **kwargs):
            if is_method:
                owner, args = args[0], args[1:]
                q = owner.__dict__.get(attr)
                if q is None or q.task.done():
                    q = _BatchQueue(fn, owner, max_batch_size, batch_wait_timeout_s, max_concurrent_batches)
                    owner.__dict__[attr] = q
            else:
                q = wrapper.__dict__.get("_q")
                if q is None or q.task.done():
                    q = _BatchQueue(fn, None, max_batch_size, batch_wait_timeout_s, max_concurrent_batches)
                    wrapper._q = q
            return await q.submit(args, kwargs)

        wrapper.__be_batch__ = (max_batch_size, batch_wait_timeout_s)
        return wrapper

    if _func is not None:
        return deco(_func)
    return deco


def batch_stats(owner, method_name: str) -> dict | None:
    q = owner.__dict__.get(f"__be_batch_{method_name}")
    if q is None:
        return None
    s = q.stats
    return {"batches": s["batches"], "requests": s["requests"], "mean_batch": s["requests"] / max(1, s["batches"]),
            "hist": dict(s["hist"]), "mean_wait_ms": 1e3 * s["wait_s"] / max(1, s["requests"])}
