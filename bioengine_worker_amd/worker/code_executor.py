"""CodeExecutor: admin-only remote Python execution (``run_code``).

Reference: ``bioengine/worker/code_executor.py:19-93,303-517`` — source (``exec``) or
cloudpickle mode, ``remote_options`` (num_cpus/num_gpus/memory/runtime_env), timeout, stdout /
stderr capture, result dict ``{"result", "stdout", "stderr"}`` or ``{"error", "traceback",
"stdout", "stderr"}``.

Execution happens in a fresh child Python process with ``HIP_VISIBLE_DEVICES`` set to the GPU(s)
reserved from the node's resource pool.  Source-mode code is only *compiled* (dedented, like the
reference's ``textwrap.dedent`` at ``code_executor.py:258``) in the worker to report syntax errors
early; it is executed -- module-level statements included -- only in the child, so user code never
runs on the worker's event loop or in its process.  Unlike the
reference (which replays captured output after the task finished), stdout/stderr lines are
streamed to ``write_stdout``/``write_stderr`` *while* the code runs, and a timeout kills the child.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import pickle
import sys
import tempfile
import textwrap
import time
import traceback
from pathlib import Path
from typing import Any

from pydantic import Field

from ..transport.schema import schema_method
from ..utils.permissions import check_permissions, user_identity


def compile_source(code: str):
    return compile(textwrap.dedent(code), "<run_code>", "exec")


def load_func_from_source(code: str, function_name: str):
    """Exec ``code`` (dedented) and return ``function_name`` from it.  Called in the child."""
    ns: dict[str, Any] = {"__name__": "__bioengine_run_code__"}
    exec(compile_source(code), ns)  # noqa: S102 - admin-only by design
    if function_name not in ns:
        raise ValueError(f"Function '{function_name}' not defined in the provided code")
    if not callable(ns[function_name]):
        raise ValueError(f"Object '{function_name}' is not callable")
    return ns[function_name]


class CodeExecutor:
    def __init__(self, cluster=None, admin_users: list[str] | None = None, logger: logging.Logger | None = None,
                 default_timeout: float = 3600.0):
        self.cluster = cluster
        self.admin_users = list(admin_users or [])
        self.log = logger or logging.getLogger("bioengine.code_executor")
        self.default_timeout = default_timeout
        self._lock = asyncio.Condition()

    async def initialize(self, admin_users: list[str]):
        self.admin_users = list(admin_users)

    async def _reserve(self, cpus, gpus, mem):
        res = self.cluster.resources if self.cluster is not None else None
        if res is None:
            return None
        async with self._lock:
            t0 = time.time()
            while not res.can_fit(min(cpus, res.total_cpu), gpus, 0):
                if gpus > res.total_gpu:
                    raise RuntimeError(f"requested num_gpus={gpus} but the node has {res.total_gpu:g} GPU(s)")
                if self.cluster.mode == "slurm":
                    await self.cluster.monitor_cluster()
                try:
                    await asyncio.wait_for(self._lock.wait(), 1.0)
                except asyncio.TimeoutError:
                    pass
                if time.time() - t0 > 3600:
                    raise TimeoutError("resources never became available")
            return res.reserve(min(cpus, res.total_cpu), gpus, 0)

    async def _release(self, cpus, gpus, ids):
        res = self.cluster.resources if self.cluster is not None else None
        if res is None or ids is None:
            return
        async with self._lock:
            res.release(min(cpus, res.total_cpu), gpus, 0, ids)
            self._lock.notify_all()

    @schema_method
    async def run_code(
        self,
        code: str | None = Field(None, description="Python source defining `function_name` (mode='source')."),
        function_name: str | None = Field("analyze", description="Function to call."),
        func_bytes: bytes | None = Field(None, description="cloudpickle.dumps(function) (mode='pickle')."),
        mode: str = Field("source", description="'source' or 'pickle'."),
        args: list | None = Field(None, description="Positional arguments."),
        kwargs: dict | None = Field(None, description="Keyword arguments."),
        remote_options: dict | None = Field(None, description="{'num_cpus', 'num_gpus', 'memory', 'runtime_env'}"),
        write_stdout: Any = Field(None, description="Callback receiving stdout lines as they are produced."),
        write_stderr: Any = Field(None, description="Callback receiving stderr lines as they are produced."),
        timeout: float | None = Field(None, description="Seconds before the execution is killed."),
        context: dict = Field(..., description="Authentication context (injected)."),
    ) -> dict:
        """Execute a Python function in an isolated child process on the worker node (admin only)."""
        check_permissions(context, self.admin_users, "execute code on the BioEngine worker")
        uid, _ = user_identity(context)
        import cloudpickle

        try:
            if mode == "pickle":
                if func_bytes is None:
                    raise ValueError("func_bytes is required in pickle mode")
                job = ("pickle", bytes(func_bytes), None)
            elif mode == "source":
                if not code:
                    raise ValueError("code is required in source mode")
                compile_source(code)  # syntax check only; the child executes it
                job = ("source", code, function_name or "analyze")
            else:
                raise ValueError(f"invalid mode '{mode}'")
        except Exception as e:  # noqa: BLE001
            return {"error": str(e), "traceback": traceback.format_exc()}
        opts = dict(remote_options or {})
        bad = set(opts) - {"num_cpus", "num_gpus", "memory", "runtime_env", "resources", "name"}
        if bad:
            return {"error": f"unsupported remote_options {sorted(bad)}", "traceback": ""}
        cpus = float(opts.get("num_cpus", 1) or 0)
        gpus = float(opts.get("num_gpus", 0) or 0)
        env_vars = dict((opts.get("runtime_env") or {}).get("env_vars") or {})
        try:  # runtime_env.pip: installed from the local wheelhouse into a shared per-set directory
            from ..apps.requirements import runtime_env_path

            pip_path = await asyncio.to_thread(runtime_env_path, opts.get("runtime_env"))
        except Exception as e:  # noqa: BLE001
            return {"error": f"runtime_env pip requirements: {e}", "traceback": traceback.format_exc()}
        self.log.info(f"User '{uid}' runs '{function_name}' (remote_options={json.dumps(opts, default=str)})")
        try:
            ids = await self._reserve(cpus, gpus, 0)
        except Exception as e:  # noqa: BLE001
            return {"error": str(e), "traceback": traceback.format_exc()}
        d = Path(tempfile.mkdtemp(prefix="be-run-"))
        inp, out = d / "in.pkl", d / "out.pkl"
        try:
            inp.write_bytes(cloudpickle.dumps((job, list(args or []), dict(kwargs or {}))))
            env = dict(os.environ)
            env.update({k: str(v) for k, v in env_vars.items()})
            if ids:
                env["HIP_VISIBLE_DEVICES"] = ",".join(map(str, ids))
            root = str(Path(__file__).resolve().parents[2])
            if pip_path:
                root = pip_path + os.pathsep + root
            env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
            proc = await asyncio.create_subprocess_exec(sys.executable, "-u", "-m", "bioengine_worker_amd.worker.exec_child",
                                                        str(inp), str(out), env=env, stdout=asyncio.subprocess.PIPE,
                                                        stderr=asyncio.subprocess.PIPE)
            so, se = [], []

            async def pump(stream, sink, cb):
                while True:
                    line = await stream.readline()
                    if not line:
                        return
                    s = line.decode(errors="replace").rstrip("\n")
                    sink.append(s)
                    if cb is not None:
                        try:
                            r = cb(s)
                            if asyncio.iscoroutine(r):
                                await r
                        except Exception:
                            pass

            pumps = asyncio.gather(pump(proc.stdout, so, write_stdout), pump(proc.stderr, se, write_stderr))
            tmo = timeout if timeout is not None else self.default_timeout
            try:
                await asyncio.wait_for(asyncio.gather(pumps, proc.wait()), timeout=tmo)
            except asyncio.TimeoutError:
                proc.kill()
                await proc.wait()
                return {"error": f"Function execution timed out after {tmo} seconds.",
                        "traceback": "TimeoutError: Function execution exceeded maximum allowed time.",
                        "stdout": "\n".join(so), "stderr": "\n".join(se)}
            stdout, stderr = "\n".join(so) + ("\n" if so else ""), "\n".join(se) + ("\n" if se else "")
            if not out.exists():
                return {"error": f"execution process exited with code {proc.returncode}", "traceback": stderr[-4000:],
                        "stdout": stdout, "stderr": stderr}
            ok, val, tb = pickle.loads(out.read_bytes())
            if ok:
                return {"result": val, "stdout": stdout, "stderr": stderr}
            return {"error": str(val), "traceback": tb, "stdout": stdout, "stderr": stderr}
        finally:
            await self._release(cpus, gpus, ids)
            for f in (inp, out):
                try:
                    f.unlink()
                except OSError:
                    pass
            try:
                d.rmdir()
            except OSError:
                pass
