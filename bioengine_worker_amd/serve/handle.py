"""DeploymentHandle / DeploymentResponse (``ray.serve.handle`` compatible).

``handle.method.remote(*args)`` issues the request immediately and returns an awaitable
:class:`DeploymentResponse`; ``handle.options(multiplexed_model_id=...)`` routes the request's model
id to ``serve.get_multiplexed_model_id()`` inside the replica.  Handles are picklable: inside a
per-process replica they route back through the parent controller.
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import threading


class DeploymentResponse:
    def __init__(self, coro_factory):
        self._fut: asyncio.Future | concurrent.futures.Future
        try:
            loop = asyncio.get_running_loop()
            self._fut = loop.create_task(coro_factory())
            self._mode = "task"
        except RuntimeError:
            from .controller import get_controller

            loop = get_controller().loop
            self._fut = asyncio.run_coroutine_threadsafe(coro_factory(), loop)
            self._mode = "cf"

    def __await__(self):
        if self._mode == "task":
            return self._fut.__await__()
        return asyncio.wrap_future(self._fut).__await__()

    def result(self, timeout_s: float | None = None):
        if self._mode == "cf":
            return self._fut.result(timeout_s)
        if self._fut.done():
            return self._fut.result()
        raise RuntimeError("DeploymentResponse.result() called on the event loop thread; use `await` instead")

    def cancel(self):
        self._fut.cancel()

    def _to_object_ref(self):
        return self


class _MethodHandle:
    def __init__(self, handle: "DeploymentHandle", method: str):
        self._h = handle
        self._m = method

    def remote(self, *args, **kwargs) -> DeploymentResponse:
        return self._h._call(self._m, args, kwargs)

    def options(self, **opts) -> "_MethodHandle":
        return _MethodHandle(self._h.options(**opts), self._m)


class DeploymentHandle:
    def __init__(self, app_name: str, deployment_name: str, opts: dict | None = None):
        self.app_name = app_name
        self.deployment_name = deployment_name
        self._opts = dict(opts or {})

    def options(self, method_name: str | None = None, multiplexed_model_id: str | None = None, stream: bool = False,
                **_ignored) -> "DeploymentHandle":
        o = dict(self._opts)
        if method_name is not None:
            o["method_name"] = method_name
        if multiplexed_model_id is not None:
            o["multiplexed_model_id"] = multiplexed_model_id
        return DeploymentHandle(self.app_name, self.deployment_name, o)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return _MethodHandle(self, name)

    def remote(self, *args, **kwargs) -> DeploymentResponse:
        return self._call(self._opts.get("method_name", "__call__"), args, kwargs)

    def _call(self, method, args, kwargs) -> DeploymentResponse:
        from .controller import get_router

        model_id = self._opts.get("multiplexed_model_id", "")
        app, dep = self.app_name, self.deployment_name

        async def go():
            return await get_router().call(app, dep, method, list(args), dict(kwargs), model_id)

        return DeploymentResponse(go)

    def __reduce__(self):
        return (DeploymentHandle, (self.app_name, self.deployment_name, self._opts))

    def __repr__(self):
        return f"DeploymentHandle(app={self.app_name!r}, deployment={self.deployment_name!r})"
