"""Remote tasks (``ray.remote`` compatible) on the node's resource pool.

Reference call sites: code execution (``bioengine/worker/code_executor.py:19-93,471-497``),
cell-image-search ingestion fan-out with ``@ray.remote(num_gpus=1, num_cpus=2)``
(``apps/cell-image-search/ingestion.py:451-531``), model-runner's isolated test runs
(``apps/model-runner/runtime_deployment.py:132-141``).  SURVEY.md §2.6 C6.

* Tasks that need a GPU (or ask for isolation) run in a fresh child Python process with
  ``HIP_VISIBLE_DEVICES`` set to the GPU reserved for them; arguments and results travel as
  pickle-5 frames through temp files.  They queue FIFO until resources free up.
* Other tasks run on a thread pool in the worker process.

``remote(fn).options(...).remote(*args)`` returns an :class:`ObjectRef` (awaitable, ``ray.get``-able).
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import os
import pickle
import subprocess
import sys
import tempfile
import threading
import uuid
from pathlib import Path

_POOL = concurrent.futures.ThreadPoolExecutor(max_workers=max(4, (os.cpu_count() or 4)), thread_name_prefix="be-task")
_RES_LOCK = threading.Condition()


class GetTimeoutError(TimeoutError):
    pass


class RayTaskError(RuntimeError):
    """Raised by ``get`` when the task raised; ``cause`` holds the original exception."""

    def __init__(self, function_name: str = "", traceback_str: str = "", cause: BaseException | None = None, *a):
        super().__init__(f"{function_name} failed: {cause!r}" if cause else function_name)
        self.function_name = function_name
        self.traceback_str = traceback_str
        self.cause = cause

    def as_instanceof_cause(self):
        return self.cause or self


class ObjectRef:
    def __init__(self, fut: concurrent.futures.Future, name: str = ""):
        self._f = fut
        self.name = name

    def __await__(self):
        return asyncio.wrap_future(self._f).__await__()

    def future(self):
        return self._f

    def done(self) -> bool:
        return self._f.done()

    def result(self, timeout=None):
        return self._f.result(timeout)

    def hex(self):
        return f"{id(self):x}"


def _resources():
    from .controller import get_controller

    return get_controller().resources


def _run_isolated(fn, args, kwargs, gpu_ids, env_vars: dict, runtime_env: dict | None = None) -> object:
    import cloudpickle

    from ..apps.requirements import runtime_env_path

    pip_path = runtime_env_path(runtime_env)  # raises MissingRequirementsError before anything runs

    d = Path(tempfile.mkdtemp(prefix="be-task-"))
    inp, out = d / "in.pkl", d / "out.pkl"
    inp.write_bytes(cloudpickle.dumps((fn, args, kwargs)))
    env = dict(os.environ)
    env.update({k: str(v) for k, v in (env_vars or {}).items()})
    if gpu_ids:
        env["HIP_VISIBLE_DEVICES"] = ",".join(map(str, gpu_ids))
    root = str(Path(__file__).resolve().parents[2])
    if pip_path:
        root = pip_path + os.pathsep + root
    env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    p = subprocess.run([sys.executable, "-m", "bioengine_worker_amd.serve.task_worker", str(inp), str(out)], env=env,
                       capture_output=True, text=True)
    try:
        if not out.exists():
            raise RayTaskError(getattr(fn, "__name__", "task"), p.stderr[-4000:],
                               RuntimeError(f"task process exited with {p.returncode}: {p.stderr[-2000:]}"))
        ok, val, tb = pickle.loads(out.read_bytes())
        if p.stdout:
            sys.stdout.write(p.stdout)
        if not ok:
            raise RayTaskError(getattr(fn, "__name__", "task"), tb, val)
        return val
    finally:
        for f in (inp, out):
            try:
                f.unlink()
            except OSError:
                pass
        try:
            d.rmdir()
        except OSError:
            pass


class RemoteFunction:
    def __init__(self, fn, **opts):
        self._fn = fn
        self._opts = opts

    def options(self, **opts) -> "RemoteFunction":
        o = dict(self._opts)
        o.update(opts)
        return RemoteFunction(self._fn, **o)

    def remote(self, *args, **kwargs) -> ObjectRef:
        fn = self._fn
        num_gpus = float(self._opts.get("num_gpus", 0) or 0)
        num_cpus = float(self._opts.get("num_cpus", 1) if self._opts.get("num_cpus") is not None else 1)
        rt = self._opts.get("runtime_env") or {}
        isolate = num_gpus > 0 or bool(rt.get("pip")) or self._opts.get("isolate", False)
        env_vars = rt.get("env_vars") or {}
        # resolve ObjectRef arguments
        def resolve(v):
            return v.result() if isinstance(v, ObjectRef) else v

        def run():
            a = [resolve(x) for x in args]
            k = {kk: resolve(vv) for kk, vv in kwargs.items()}
            if not isolate:
                try:
                    return fn(*a, **k)
                except BaseException as e:  # noqa: BLE001
                    import traceback

                    raise RayTaskError(getattr(fn, "__name__", "task"), traceback.format_exc(), e) from e
            res = _resources()
            with _RES_LOCK:
                while not res.can_fit(min(num_cpus, res.total_cpu), num_gpus, 0):
                    _RES_LOCK.wait(0.2)
                ids = res.reserve(min(num_cpus, res.total_cpu), num_gpus, 0)
            try:
                return _run_isolated(fn, a, k, ids, env_vars, rt)
            finally:
                with _RES_LOCK:
                    res.release(min(num_cpus, res.total_cpu), num_gpus, 0, ids)
                    _RES_LOCK.notify_all()

        return ObjectRef(_POOL.submit(run), getattr(fn, "__name__", "task"))

    def __call__(self, *a, **k):
        raise TypeError("Remote functions cannot be called directly; use .remote()")


def remote(*args, **kwargs):
    if len(args) == 1 and callable(args[0]) and not kwargs:
        return RemoteFunction(args[0])

    def deco(fn):
        return RemoteFunction(fn, **kwargs)

    return deco


def get(refs, timeout: float | None = None):
    if isinstance(refs, (list, tuple)):
        return [get(r, timeout) for r in refs]
    if isinstance(refs, ObjectRef):
        try:
            return refs.result(timeout)
        except concurrent.futures.TimeoutError as e:
            raise GetTimeoutError(str(e)) from e
    return refs


def put(value) -> ObjectRef:
    f = concurrent.futures.Future()
    f.set_result(value)
    return ObjectRef(f, "put")


def wait(refs, num_returns: int = 1, timeout: float | None = None, fetch_local: bool = True):
    fs = {r.future(): r for r in refs}
    done, not_done = concurrent.futures.wait(list(fs), timeout=timeout, return_when=concurrent.futures.FIRST_COMPLETED
                                             if num_returns == 1 else concurrent.futures.ALL_COMPLETED)
    d = [fs[f] for f in fs if f in done][:num_returns]
    return d, [r for r in refs if r not in d]
