"""Child-process side of a :class:`~bioengine_worker_amd.serve.replica.ProcessReplica`.

Started as ``python -m bioengine_worker_amd.serve.replica_worker`` with ``HIP_VISIBLE_DEVICES`` set to
the replica's GPU(s).  Connects back to the parent over a Unix socket, instantiates the user
deployment class, and serves requests concurrently on its own asyncio loop.  Calls on
``DeploymentHandle`` objects made inside the replica are forwarded to the parent's router.
"""
from __future__ import annotations

import asyncio
import inspect
import itertools
import os
import sys
import threading
import traceback


class _ChildRouter:
    def __init__(self, conn, lock, loop, ring=None):
        self.conn = conn
        self.ring = ring
        self.lock = lock
        self.loop = loop
        self.rids = itertools.count(1)
        self.pending: dict[int, asyncio.Future] = {}

    async def call(self, app, dep, method, args, kwargs, model_id=""):
        from ..runtime import faults as _faults
        from .replica import send_async

        rid = next(self.rids)
        fut = self.loop.create_future()
        self.pending[rid] = fut
        await send_async(self.conn, self.lock, ("hcall", rid, app, dep, method, args, kwargs, model_id,
                                                                    _faults.current_deadline()),
                                self.ring)
        return await fut


async def _main():
    from multiprocessing.connection import Client

    from . import context as rctx
    from . import controller as ctrl_mod
    from .replica import _resolve_result, reader_mode, recv_frames, send_async, send_frames

    # GPU replicas run their device work on worker threads that hold the GIL between launches; a
    # 0.5 ms switch interval (default 5 ms) keeps the request reader and event loop responsive
    sys.setswitchinterval(float(os.environ.get("BE_REPLICA_SWITCH_INTERVAL_S", "0.0005")))
    sock = os.environ["BE_REPLICA_SOCK"]
    key = bytes.fromhex(os.environ["BE_REPLICA_KEY"])
    rx = tx = None
    if os.environ.get("BE_REPLICA_RING_RX"):  # open both lanes before connecting (parent unlinks after)
        from ..runtime.shm_ring import ShmRing

        rx, tx = ShmRing.open(os.environ["BE_REPLICA_RING_RX"]), ShmRing.open(os.environ["BE_REPLICA_RING_TX"])
    conn = Client(sock, family="AF_UNIX", authkey=key)
    lock = threading.Lock()
    loop = asyncio.get_running_loop()
    router = _ChildRouter(conn, lock, loop, tx)
    ctrl_mod._set_child_router(router)
    inbox: asyncio.Queue = asyncio.Queue()

    def reader():
        while True:
            try:
                msg = recv_frames(conn, rx)
            except (EOFError, OSError):
                loop.call_soon_threadsafe(inbox.put_nowait, ("stop",))
                return
            except Exception as e:  # noqa: BLE001
                print(f"replica: undecodable message: {e!r}", flush=True)
                continue
            loop.call_soon_threadsafe(inbox.put_nowait, msg)

    obj = None
    ctx = None

    from ..profiling import trace
    from ..runtime import faults
    from .replica import builtin_gpu_check

    inflight = faults.InflightTable()
    nonlocal_state = {"health_ok": 0}

    async def handle_call(rid, method, args, kwargs, model_id, deadline=None):
        # never cancelled in the child: the entry stays until the user code returns
        with faults.deadline_scope(deadline=deadline):
            with inflight.track(method, deadline), trace.span(f"child.{method}", cat="replica"):
                await _handle_call(rid, method, args, kwargs, model_id)

    async def _handle_call(rid, method, args, kwargs, model_id):
        tok = rctx.set_current(ctx)
        mtok = rctx.set_model_id(model_id)
        try:
            if method == "__be_check_health__":
                inflight.check()  # a call wedged past its deadline fails the replica
                await asyncio.to_thread(builtin_gpu_check)  # GPU-hang watchdog
                fn = getattr(obj, "check_health", None)
                res = None
                if fn is not None:
                    res = fn()
                    if inspect.isawaitable(res):
                        res = await res
                nonlocal_state["health_ok"] += 1
                if nonlocal_state["health_ok"] in (1, 3):  # lazy async_init has built the app by now
                    from ..runtime.gcpolicy import refreeze

                    refreeze()
            else:
                faults.point(f"replica_entry.{method}")
                fn = getattr(obj, method)
                if inspect.iscoroutinefunction(fn):
                    res = await fn(*args, **kwargs)
                else:
                    from .replica import _run_with_ctx

                    res = await asyncio.to_thread(_run_with_ctx, ctx, model_id, fn, args, kwargs)
                res = await _resolve_result(res)
            out = ("result", rid, True, res)
        except BaseException as e:  # noqa: BLE001
            traceback.print_exc()
            out = ("result", rid, False, _picklable_exc(e))
        finally:
            rctx.reset_model_id(mtok)
            rctx.reset_current(tok)
        try:
            await send_async(conn, lock, out, tx)
        except Exception as e:  # result not picklable
            await send_async(conn, lock, ("result", rid, False, RuntimeError(f"unpicklable result: {e}")), tx)

    def dispatch(msg):
        kind = msg[0]
        if kind == "call":
            _, rid, method, args, kwargs, model_id, deadline = msg
            asyncio.ensure_future(handle_call(rid, method, args, kwargs, model_id, deadline))
        elif kind == "hresult":
            _, rid, ok, val = msg
            fut = router.pending.pop(rid, None)
            if fut is not None and not fut.done():
                if ok:
                    fut.set_result(val)
                else:
                    fut.set_exception(val if isinstance(val, BaseException) else RuntimeError(str(val)))
        else:
            inbox.put_nowait(msg)

    def on_readable():
        # bulk payloads ride the ring, so socket messages are small: decode them on the loop as the
        # fd turns readable and start calls directly (no reader-thread and inbox hand-offs)
        try:
            while conn.poll():
                try:
                    msg = recv_frames(conn, rx)
                except (EOFError, OSError):
                    raise
                except Exception as e:  # noqa: BLE001
                    print(f"replica: undecodable message: {e!r}", flush=True)
                    continue
                dispatch(msg)
        except (EOFError, OSError):
            loop.remove_reader(conn.fileno())
            inbox.put_nowait(("stop",))

    if rx is not None and reader_mode() == "loop":
        loop.add_reader(conn.fileno(), on_readable)
    else:
        threading.Thread(target=reader, daemon=True).start()

    while True:
        msg = await inbox.get()
        kind = msg[0]
        if kind == "init":
            _, cls, args, kwargs, app, dep, tag, gpu_ids = msg
            ctx = rctx.ReplicaContext(app, dep, tag, None, gpu_ids)
            tok = rctx.set_current(ctx)
            try:
                obj = await asyncio.to_thread(_construct, ctx, cls, args, kwargs)
                ctx.servable_object = obj
                from ..runtime.gcpolicy import serving_gc

                serving_gc()  # app constructed: freeze startup objects out of the GC scans
                await asyncio.to_thread(send_frames, conn, lock, ("ready", True, None))
            except BaseException as e:  # noqa: BLE001
                traceback.print_exc()
                await asyncio.to_thread(send_frames, conn, lock, ("ready", False, f"{type(e).__name__}: {e}"))
            finally:
                rctx.reset_current(tok)
        elif kind == "call":
            _, rid, method, args, kwargs, model_id, deadline = msg
            asyncio.ensure_future(handle_call(rid, method, args, kwargs, model_id, deadline))
        elif kind == "hresult":
            _, rid, ok, val = msg
            fut = router.pending.pop(rid, None)
            if fut is not None and not fut.done():
                if ok:
                    fut.set_result(val)
                else:
                    fut.set_exception(val if isinstance(val, BaseException) else RuntimeError(str(val)))
        elif kind == "stop":
            break
    try:
        loop.remove_reader(conn.fileno())
    except (OSError, ValueError):
        pass
    try:
        conn.close()
    except Exception:
        pass


def _construct(ctx, cls, args, kwargs):
    from . import context as rctx

    tok = rctx.set_current(ctx)
    try:
        return cls(*args, **kwargs)
    finally:
        rctx.reset_current(tok)


def _picklable_exc(e: BaseException) -> BaseException:
    import pickle

    try:
        pickle.dumps(e)
        return e
    except Exception:
        return RuntimeError(f"{type(e).__name__}: {e}")


def main():
    sys.path.insert(0, os.getcwd())
    from ..runtime.shm_ring import tune_malloc

    tune_malloc()
    from ..compat import install

    install()
    prof_path = os.environ.get("BE_REPLICA_PROFILE")  # cProfile of the replica's event-loop thread
    if not prof_path:
        asyncio.run(_main())
        return
    import cProfile
    import pstats

    prof = cProfile.Profile()
    prof.enable()
    try:
        asyncio.run(_main())
    finally:
        prof.disable()
        with open(prof_path.replace("{pid}", str(os.getpid())), "w") as f:
            pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(40)
            pstats.Stats(prof, stream=f).sort_stats("cumulative").print_stats(80)


if __name__ == "__main__":
    main()
