"""Deployment replicas: in-process asyncio replicas and one-OS-process-per-replica (GPU pinned).

Replaces Ray actors hosting Serve replicas (every request crossed >= 3 process
boundaries and pickled full ndarrays through the object store).

* :class:`LocalReplica` — the user class lives in the worker process; requests are direct awaits
  (zero copies).  Used for CPU-only deployments (entry/orchestration deployments, demo apps).
* :class:`ProcessReplica` — the user class lives in a child Python process started with
  ``HIP_VISIBLE_DEVICES``/``ROCR_VISIBLE_DEVICES`` set to its reserved GPU(s), so each GPU replica
  owns its device and its HIP context.  Requests travel over a Unix-socket connection as
  pickle-protocol-5 frames with out-of-band buffers (ndarrays are sent as raw buffers, not
  re-encoded).  Child stdout/stderr go to a per-replica log file that status calls tail.

Both expose: ``start()``, ``call(method, args, kwargs, model_id)``, ``check_health()``,
``stop()``, ``ongoing`` (in-flight requests) and ``logs(tail)``.
"""
from __future__ import annotations

import asyncio
import inspect
import itertools
import os
import pickle
import secrets
import subprocess
import sys
import tempfile
import threading
import time
import uuid
from pathlib import Path

from ..runtime import faults
from . import context as rctx

STARTING, RUNNING, UNHEALTHY, STOPPING, DEAD = "STARTING", "RUNNING", "UNHEALTHY", "STOPPING", "DEAD"


def _new_tag(app: str, dep: str) -> str:
    return f"{app}#{dep}#{uuid.uuid4().hex[:6]}"


async def _resolve_result(res):
    from .tasks import ObjectRef

    if inspect.isawaitable(res) and not isinstance(res, ObjectRef):
        res = await res
    if isinstance(res, ObjectRef):
        res = await res
    return res


class ReplicaBase:
    def __init__(self, app: str, dep: str, cls, args, kwargs, gpu_ids: list[int], env: dict | None = None):
        self.app = app
        self.dep = dep
        self.cls = cls
        self.args = args
        self.kwargs = kwargs
        self.gpu_ids = list(gpu_ids)
        self.env = dict(env or {})
        self.tag = _new_tag(app, dep)
        self.state = STARTING
        self.ongoing = 0
        self.started_at = time.time()
        self.error: str | None = None
        self.health_failures = 0
        self.node_id = "head"
        self.inflight = faults.InflightTable()  # watchdog: calls and their deadlines

    @property
    def replica_id(self) -> str:
        return self.tag

    def info(self) -> dict:
        return {"replica_id": self.tag, "state": self.state, "ongoing_requests": self.ongoing,
                "gpu_ids": self.gpu_ids, "start_time": self.started_at, "node_id": self.node_id,
                "error": self.error, "pid": getattr(self, "pid", os.getpid())}


class LocalReplica(ReplicaBase):
    async def start(self):
        rctx.install_log_capture()
        ctx = rctx.ReplicaContext(self.app, self.dep, self.tag, None, self.gpu_ids)
        self._ctx = ctx

        def build():
            tok = rctx.set_current(ctx)
            try:
                # in-process replicas share the worker's environment: temp-dir variables would
                # redirect every later tempfile/AF_UNIX socket of the host process, so they are
                # only honoured by process replicas
                os.environ.update({k: str(v) for k, v in self.env.items() if k not in ("TMPDIR", "TEMP", "TMP")})
                obj = self.cls(*self.args, **self.kwargs)
            finally:
                rctx.reset_current(tok)
            return obj

        try:
            tok = rctx.set_current(ctx)
            try:
                self.obj = await asyncio.to_thread(build)
            finally:
                rctx.reset_current(tok)
            ctx.servable_object = self.obj
            self.state = RUNNING
        except BaseException as e:  # noqa: BLE001
            self.state = DEAD
            self.error = f"{type(e).__name__}: {e}"
            raise

    async def call(self, method: str, args, kwargs, model_id: str = ""):
        fn = getattr(self.obj, method)
        self.ongoing += 1
        tok = rctx.set_current(self._ctx)
        mtok = rctx.set_model_id(model_id)
        try:
            faults.point(f"replica_entry.{method}")
            return await self._invoke(fn, method, model_id, args, kwargs)
        finally:
            rctx.reset_model_id(mtok)
            rctx.reset_current(tok)
            self.ongoing -= 1

    async def _invoke(self, fn, method, model_id, args, kwargs):
        if inspect.iscoroutinefunction(fn) or inspect.iscoroutinefunction(getattr(fn, "__func__", None)):
            res = await fn(*args, **kwargs)  # cancelled at the deadline
        else:
            # a thread cannot be cancelled: the thread itself holds the watchdog entry, so a call
            # still running after the router gave up on it keeps counting as wedged
            deadline = faults.current_deadline()

            def tracked(*a, **k):
                with self.inflight.track(method, deadline):
                    return fn(*a, **k)

            res = await asyncio.to_thread(_run_with_ctx, self._ctx, model_id, tracked, args, kwargs)
        return await _resolve_result(res)

    async def check_health(self):
        self.inflight.check()
        if self.gpu_ids:
            await asyncio.to_thread(builtin_gpu_check)
        fn = getattr(self.obj, "check_health", None)
        if fn is None:
            return True
        await self.call("check_health", [], {})
        return True

    async def stop(self, timeout: float = 20.0):
        self.state = STOPPING
        t0 = time.time()
        while self.ongoing > 0 and time.time() - t0 < timeout:
            await asyncio.sleep(0.05)
        obj = getattr(self, "obj", None)
        if obj is not None:
            for hook in ("__del__",):
                pass
            self.obj = None
        self.state = DEAD

    def logs(self, tail: int = 100) -> list[str]:
        buf = rctx.log_buffer(self.tag)
        return list(buf)[-tail:] if tail > 0 else list(buf)


def builtin_gpu_check(timeout_s: float | None = None) -> None:
    """GPU-hang watchdog of the replica health check: a tiny kernel on a private stream must finish
    within ``BIOENGINE_GPU_PROBE_TIMEOUT_S``.  Only probes a process that already initialised HIP
    (never brings up a GPU context in a CPU-only replica)."""
    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_available() or not torch.cuda.is_initialized():
        return
    faults.gpu_probe(timeout_s=timeout_s or float(os.environ.get("BIOENGINE_GPU_PROBE_TIMEOUT_S", "10")))


def _run_with_ctx(ctx, model_id, fn, args, kwargs):
    tok = rctx.set_current(ctx)
    mtok = rctx.set_model_id(model_id)
    try:
        return fn(*args, **kwargs)
    finally:
        rctx.reset_model_id(mtok)
        rctx.reset_current(tok)


# ====================================================================== process replicas


#: strings at least this long (base64 images and thumbnails in request / response dicts) travel as
#: out-of-band UTF-8 buffers -- through the shared-memory ring with the arrays -- instead of inside
#: the pickle header that crosses the socket (pickle's C fast path never offers str to a reducer)
BIG_STR = 16 << 10


def _big_str(buf) -> str:
    # the received bytes stay attached: a consumer that wants them (base64 decoding, a re-send)
    # reads .utf8 instead of encoding the string again
    return Utf8Str(str(buf, "utf-8"), buf)


class _BigStr:
    __slots__ = ("b",)

    def __init__(self, b: bytes):
        self.b = b

    def __reduce_ex__(self, protocol):
        return _big_str, (pickle.PickleBuffer(self.b),)


class Utf8Str(str):
    """A ``str`` that carries its UTF-8 bytes (``.utf8``): long strings a server returns again and
    again -- pre-encoded base64 thumbnails -- cross the process boundary without a per-message
    ``encode``.  Behaves as a plain ``str`` everywhere else (JSON, msgpack, comparisons)."""

    __slots__ = ("utf8",)

    def __new__(cls, s: str, utf8: bytes | None = None):
        o = super().__new__(cls, s)
        o.utf8 = utf8 if utf8 is not None else s.encode("utf-8")
        return o

    def __reduce__(self):
        return str, (str(self),)


def _lift_strings(o, depth: int = 0):
    """Copy of the plain dict / list / tuple skeleton of ``o`` with long strings wrapped as
    :class:`_BigStr`; ``o`` itself when nothing qualifies (no copy)."""
    t = type(o)
    if t is Utf8Str:
        return _BigStr(o.utf8) if len(o.utf8) >= BIG_STR else o
    if t is str:
        if len(o) >= BIG_STR:
            try:
                return _BigStr(o.encode("utf-8"))
            except UnicodeEncodeError:
                return o
        return o
    if depth >= 6:
        return o
    if t is dict:
        out = None
        for k, v in o.items():
            w = _lift_strings(v, depth + 1)
            if w is not v:
                if out is None:
                    out = dict(o)
                out[k] = w
        return o if out is None else out
    if t is list or t is tuple:
        items = None
        for i, v in enumerate(o):
            w = _lift_strings(v, depth + 1)
            if w is not v:
                if items is None:
                    items = list(o)
                items[i] = w
        return o if items is None else (items if t is list else tuple(items))
    return o


def dumps(obj) -> list:
    """Pickle-5 header + the out-of-band buffers (arrays, long strings) as zero-copy memoryviews."""
    import cloudpickle

    bufs: list = []
    head = cloudpickle.dumps(_lift_strings(obj), protocol=5, buffer_callback=bufs.append)
    return [head] + [b.raw() if hasattr(b, "raw") else memoryview(b) for b in bufs]


def loads(frames: list):
    return pickle.loads(frames[0], buffers=frames[1:])


#: out-of-band payloads at least this large travel through the shared-memory ring (one memcpy in,
#: one out) instead of being streamed through the socket buffer in ~200 KB chunks, each chunk a
#: sender/reader wake-up
RING_MIN_BYTES = 64 << 10
#: messages whose socket part is at most this large are sent straight from the event loop (no
#: worker-thread hop); anything that could block on a full socket or ring goes through a thread
INLINE_MAX_BYTES = 128 << 10


def _ring_bytes(lens) -> int:
    return sum(8 + ((int(n) + 7) & ~7) for n in lens)


def _send_locked(conn, frames, ring) -> None:
    if ring is not None:
        ring.write(frames[1:])
        conn.send(("ring", len(frames)))
        conn.send_bytes(frames[0])
        return
    conn.send(len(frames))
    for f in frames:
        conn.send_bytes(f)


def _route(frames, ring):
    """(ring to use or None, bytes that would cross the socket)."""
    bufs = frames[1:]
    lens = [b.nbytes for b in bufs]
    if ring is not None and bufs and sum(lens) >= RING_MIN_BYTES and ring.fits(lens):
        return ring, len(frames[0]), lens
    return None, len(frames[0]) + sum(lens), lens


def _send_prepared(conn, lock, frames, ring):
    with lock:
        _send_locked(conn, frames, ring)


def send_frames(conn, lock: threading.Lock, obj, ring=None):
    """Send ``obj``; with a ``ring`` (:class:`~bioengine_worker_amd.runtime.shm_ring.ShmRing`) the
    out-of-band buffers go through shared memory and only the pickle header crosses the socket.
    Ring write and socket send happen under the same lock, so both lanes stay in message order."""
    frames = dumps(obj)
    use, _, _ = _route(frames, ring)
    _send_prepared(conn, lock, frames, use)


async def send_async(conn, lock: threading.Lock, obj, ring=None):
    """:func:`send_frames` from an event loop.  A message that cannot block -- small socket part
    and, for ring payloads, room in the ring right now -- is written inline (saves two thread
    wake-ups per message, the dominant cost of a small request); the rest goes through a thread."""
    frames = dumps(obj)
    use, sock_bytes, lens = _route(frames, ring)
    inline = sock_bytes <= INLINE_MAX_BYTES
    if inline and use is not None:
        st = use.stats()
        inline = st["capacity"] - st["queued_bytes"] >= _ring_bytes(lens)
    if inline and lock.acquire(blocking=False):
        try:
            _send_locked(conn, frames, use)
        finally:
            lock.release()
        return
    await asyncio.to_thread(_send_prepared, conn, lock, frames, use)


def recv_frames(conn, ring=None):
    n = conn.recv()
    if isinstance(n, tuple):  # ("ring", n_frames): header on the socket, buffers in the ring
        head = conn.recv_bytes()
        return loads([head] + [ring.read() for _ in range(n[1] - 1)])
    frames = [conn.recv_bytes() for _ in range(n)]
    return loads(frames)


def reader_mode() -> str:
    """``BE_REPLICA_READER``: ``loop`` (default; fd readiness on the event loop) or ``thread``."""
    return os.environ.get("BE_REPLICA_READER", "loop")


def ring_capacity() -> int:
    """Per-direction ring size (``BE_REPLICA_RING_MB``, default 128; 0 disables the rings)."""
    return int(float(os.environ.get("BE_REPLICA_RING_MB", "128")) * (1 << 20))


class ProcessReplica(ReplicaBase):
    _ids = itertools.count(1)

    def __init__(self, *a, log_dir: str | Path | None = None, python: str | None = None, **k):
        super().__init__(*a, **k)
        self.log_dir = Path(log_dir or tempfile.gettempdir()) / "bioengine_replicas"
        self.log_dir.mkdir(parents=True, exist_ok=True)
        self.log_file = self.log_dir / f"{self.tag.replace('#', '_')}.log"
        self.python = python or sys.executable
        self.pending: dict[int, asyncio.Future] = {}
        self.rids = itertools.count(1)
        self.send_lock = threading.Lock()
        self.proc = None
        self.conn = None
        self.tx = self.rx = None  # shared-memory bulk lanes (router->replica, replica->router)

    def _make_rings(self, env: dict) -> None:
        cap = ring_capacity()
        if cap <= 0:
            return
        try:
            from ..runtime.shm_ring import ShmRing, tune_malloc

            tune_malloc("router")
            self.tx, self.rx = ShmRing.create(cap), ShmRing.create(cap)
        except Exception:  # runtime library unavailable or /dev/shm exhausted: socket-only
            self._drop_rings()
            return
        env["BE_REPLICA_RING_RX"] = self.tx.name  # the child's receive lane is our transmit lane
        env["BE_REPLICA_RING_TX"] = self.rx.name

    def _drop_rings(self) -> None:
        for r in (self.tx, self.rx):
            if r is not None:
                r.unlink()
                r.shutdown()
        self.tx = self.rx = None

    async def start(self):
        from multiprocessing.connection import Listener

        self.loop = asyncio.get_running_loop()
        sock = str(Path(tempfile.gettempdir()) / f"be-rep-{os.getpid()}-{next(self._ids)}-{uuid.uuid4().hex[:6]}.sock")
        key = secrets.token_bytes(16)
        listener = Listener(sock, family="AF_UNIX", authkey=key)
        env = dict(os.environ)
        env.update({k: str(v) for k, v in self.env.items()})
        if self.gpu_ids:
            # indices are relative to the parent's visible set; the child sees exactly its GPUs
            env["HIP_VISIBLE_DEVICES"] = ",".join(str(g) for g in self.gpu_ids)
        env["BE_REPLICA_SOCK"] = sock
        env["BE_REPLICA_KEY"] = key.hex()
        env["BE_REPLICA_TAG"] = self.tag
        self._make_rings(env)
        root = str(Path(__file__).resolve().parents[2])
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        logf = open(self.log_file, "ab", buffering=0)
        self.proc = subprocess.Popen([self.python, "-u", "-m", "bioengine_worker_amd.serve.replica_worker"], env=env,
                                     stdout=logf, stderr=subprocess.STDOUT, close_fds=True)
        self.pid = self.proc.pid
        logf.close()
        try:
            self.conn = await asyncio.wait_for(asyncio.to_thread(listener.accept), timeout=120)
        except Exception as e:
            self._kill()
            self._drop_rings()
            self.state = DEAD
            self.error = f"replica process failed to connect: {e}"
            raise RuntimeError(self.error) from e
        finally:
            listener.close()
            try:
                os.unlink(sock)
            except OSError:
                pass
        for r in (self.tx, self.rx):  # the child opened both before connecting: drop the names
            if r is not None:
                r.unlink()
        if self.rx is not None and reader_mode() == "loop":
            # bulk payloads ride the ring, so socket messages are small: read them on the event loop
            # when the fd turns readable (no reader-thread -> loop hand-off per message)
            self._reader = None
            self.loop.add_reader(self.conn.fileno(), self._on_readable)
        else:
            self._reader = threading.Thread(target=self._read_loop, daemon=True)
            self._reader.start()
        fut = self.loop.create_future()
        self.pending[0] = fut
        await asyncio.to_thread(send_frames, self.conn, self.send_lock,
                                ("init", self.cls, self.args, self.kwargs, self.app, self.dep, self.tag, self.gpu_ids),
                                self.tx)
        ok, err = await fut
        if not ok:
            self.state = DEAD
            self.error = err
            self._kill()
            raise RuntimeError(f"replica {self.tag} failed to initialize: {err}")
        self.state = RUNNING

    def _read_loop(self):
        while True:
            try:
                msg = recv_frames(self.conn, self.rx)
            except (EOFError, OSError):
                break
            except Exception as e:  # undecodable result: fail the request that produced it
                msg = ("fatal", repr(e))
            self.loop.call_soon_threadsafe(self._dispatch, msg)
        self.loop.call_soon_threadsafe(self._on_exit)

    def _on_readable(self):
        try:
            while self.conn.poll():
                try:
                    msg = recv_frames(self.conn, self.rx)
                except (EOFError, OSError):
                    raise
                except Exception as e:  # undecodable result
                    msg = ("fatal", repr(e))
                self._dispatch(msg)
        except (EOFError, OSError):
            try:
                self.loop.remove_reader(self.conn.fileno())
            except (OSError, ValueError):
                pass
            self._on_exit()

    def _dispatch(self, msg):
        kind = msg[0]
        if kind == "ready":
            fut = self.pending.pop(0, None)
            if fut and not fut.done():
                fut.set_result((msg[1], msg[2]))
        elif kind == "result":
            _, rid, ok, val = msg
            fut = self.pending.pop(rid, None)
            if fut and not fut.done():
                if ok:
                    fut.set_result(val)
                else:
                    fut.set_exception(val if isinstance(val, BaseException) else RuntimeError(str(val)))
        elif kind == "hcall":
            _, rid, app, dep, method, args, kwargs, model_id, deadline = msg
            asyncio.ensure_future(self._serve_hcall(rid, app, dep, method, args, kwargs, model_id, deadline))

    async def _serve_hcall(self, rid, app, dep, method, args, kwargs, model_id, deadline=None):
        from .controller import get_router

        try:
            with faults.deadline_scope(deadline=deadline):
                val = await get_router().call(app, dep, method, args, kwargs, model_id)
            out = ("hresult", rid, True, val)
        except BaseException as e:  # noqa: BLE001
            out = ("hresult", rid, False, e)
        try:
            await send_async(self.conn, self.send_lock, out, self.tx)
        except Exception:
            pass

    def _on_exit(self):
        if self.state not in (STOPPING, DEAD):
            self.state = DEAD
            self.error = self.error or f"replica process exited (code {self.proc.poll() if self.proc else None})"
        for fut in self.pending.values():
            if not fut.done():
                fut.set_exception(RuntimeError(f"replica {self.tag} died: {self.error}"))
        self.pending.clear()
        for r in (self.tx, self.rx):  # release a sender blocked on a ring the dead child no longer drains
            if r is not None:
                r.shutdown()

    async def call(self, method: str, args, kwargs, model_id: str = ""):
        if self.state == DEAD:
            raise RuntimeError(f"replica {self.tag} is dead: {self.error}")
        rid = next(self.rids)
        fut = self.loop.create_future()
        self.pending[rid] = fut
        self.ongoing += 1
        try:
            with self.inflight.track(method, faults.current_deadline()):
                await send_async(self.conn, self.send_lock,
                                 ("call", rid, method, args, kwargs, model_id, faults.current_deadline()), self.tx)
                return await fut
        finally:
            self.ongoing -= 1

    async def check_health(self):
        if self.proc is None or self.proc.poll() is not None:
            raise RuntimeError(f"replica process is not running (exit code {self.proc.poll() if self.proc else None})")
        self.inflight.check()
        await self.call("__be_check_health__", [], {})
        return True

    def _kill(self):
        if self.proc is not None and self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(5)
            except subprocess.TimeoutExpired:
                self.proc.kill()

    async def stop(self, timeout: float = 20.0):
        self.state = STOPPING
        t0 = time.time()
        while self.ongoing > 0 and time.time() - t0 < timeout:
            await asyncio.sleep(0.05)
        try:
            if self.conn is not None:
                await asyncio.to_thread(send_frames, self.conn, self.send_lock, ("stop",))
        except Exception:
            pass
        if self.proc is not None:
            try:
                await asyncio.wait_for(asyncio.to_thread(self.proc.wait), timeout=5)
            except asyncio.TimeoutError:
                self._kill()
        self.state = DEAD

    def logs(self, tail: int = 100) -> list[str]:
        try:
            lines = self.log_file.read_text(errors="replace").splitlines()
        except OSError:
            return []
        return lines[-tail:] if tail > 0 else lines
