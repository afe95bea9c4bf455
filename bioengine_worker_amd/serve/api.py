"""Ray-Serve-compatible deployment API on the native serving runtime.

App code written for the reference keeps working unchanged: ``from ray import serve`` resolves to
this module's namespace (see :mod:`.ray_compat`) and provides ``serve.deployment`` (+ ``.options``
/ ``.bind``), ``serve.multiplexed``, ``serve.get_multiplexed_model_id``,
``serve.get_replica_context``, ``serve.batch``, ``serve.run``/``delete``/``status``/``shutdown``
and ``DeploymentHandle`` (reference call sites: every app, e.g.
``apps/model-runner/runtime_deployment.py:31-55,187``, ``apps/composition-demo/entry_deployment.py``;
SURVEY.md §7.4 hard part 4).  Underneath there is no Ray: deployments run as replicas managed by
:class:`~.controller.ServeController` (in-process asyncio replicas, or one OS process per replica
pinned to its GPU).
"""
from __future__ import annotations

import asyncio
import collections
import copy
import functools
import inspect
from dataclasses import dataclass, field
from typing import Any

from . import context as _ctx
from .batching import batch  # noqa: F401
from .context import get_multiplexed_model_id, get_replica_context  # noqa: F401

DEFAULT_MAX_ONGOING = 5


@dataclass
class DeploymentConfig:
    name: str
    num_replicas: int | str | None = 1
    max_ongoing_requests: int = DEFAULT_MAX_ONGOING
    max_queued_requests: int = -1
    ray_actor_options: dict = field(default_factory=dict)
    autoscaling_config: dict | None = None
    health_check_period_s: float = 10.0
    health_check_timeout_s: float = 30.0
    graceful_shutdown_timeout_s: float = 20.0
    graceful_shutdown_wait_loop_s: float = 2.0
    user_config: Any = None
    logging_config: Any = None
    placement_group_bundles: Any = None
    max_replicas_per_node: int | None = None
    #: per-request deadline enforced by the router (bioengine extension; None -> env
    #: ``BIOENGINE_REQUEST_TIMEOUT_S`` or no deadline).  See ``runtime/faults.py``.
    request_timeout_s: float | None = None

    def num_cpus(self) -> float:
        return float(self.ray_actor_options.get("num_cpus", 1) or 0)

    def num_gpus(self) -> float:
        return float(self.ray_actor_options.get("num_gpus", 0) or 0)

    def memory(self) -> float:
        return float(self.ray_actor_options.get("memory", 0) or 0)

    def min_max_replicas(self) -> tuple[int, int, int]:
        ac = self.autoscaling_config
        if ac:
            lo = int(ac.get("min_replicas", 1))
            hi = int(ac.get("max_replicas", max(lo, 1)))
            init = int(ac.get("initial_replicas", lo) or lo)
            return lo, hi, max(lo, min(init, hi))
        n = self.num_replicas if isinstance(self.num_replicas, int) else 1
        return n, n, n


_OPT_KEYS = {f for f in DeploymentConfig.__dataclass_fields__ if f != "name"}


class Deployment:
    """Result of ``@serve.deployment``; ``.bind()`` builds an application node."""

    def __init__(self, func_or_class, config: DeploymentConfig):
        self.func_or_class = func_or_class
        self._config = config

    @property
    def name(self) -> str:
        return self._config.name

    @property
    def ray_actor_options(self) -> dict:
        return self._config.ray_actor_options

    @property
    def max_ongoing_requests(self) -> int:
        return self._config.max_ongoing_requests

    @property
    def config(self) -> DeploymentConfig:
        return self._config

    def options(self, **kwargs) -> "Deployment":
        cfg = copy.deepcopy(self._config)
        for k, v in kwargs.items():
            if k == "name":
                cfg.name = v
            elif k in _OPT_KEYS:
                setattr(cfg, k, copy.deepcopy(v))
            elif k == "max_concurrent_queries":
                cfg.max_ongoing_requests = v
            elif k == "version":
                pass
            else:
                raise TypeError(f"unknown deployment option '{k}'")
        return Deployment(self.func_or_class, cfg)

    def bind(self, *args, **kwargs) -> "Application":
        return Application(self, args, kwargs)

    def __call__(self, *a, **k):
        raise RuntimeError("Deployments cannot be constructed directly; use .bind() and serve.run()")


@dataclass
class Application:
    """A bound deployment (node of the application graph). Bound children appear in args."""

    deployment: Deployment
    args: tuple
    kwargs: dict

    def children(self) -> list["Application"]:
        out = []
        for v in list(self.args) + list(self.kwargs.values()):
            if isinstance(v, Application):
                out.append(v)
        return out


# Ray exposes the bound node type under several names.
BoundDeployment = Application


def deployment(_func_or_class=None, *, name: str | None = None, **kwargs):
    def wrap(obj):
        cfg = DeploymentConfig(name=name or getattr(obj, "__name__", "Deployment"))
        d = Deployment(obj, cfg)
        return d.options(**kwargs) if kwargs else d

    if _func_or_class is not None and (inspect.isclass(_func_or_class) or callable(_func_or_class)):
        return wrap(_func_or_class)
    return wrap


# ---------------------------------------------------------------------------------- multiplexing


def multiplexed(func=None, *, max_num_models_per_replica: int = 3):
    """Per-replica LRU of loaded models keyed by model id (``@serve.multiplexed``).

    The wrapped loader is called at most once per id while the id stays cached; concurrent loads
    of the same id share one in-flight load; evicted models get ``__del__``/``close`` semantics
    by dropping the reference (``.unload()`` is called if the model defines it)."""

    def deco(fn):
        if not inspect.iscoroutinefunction(fn):
            raise TypeError("@serve.multiplexed requires an async function")
        attr = f"__be_mux_{fn.__name__}"

        @functools.wraps(fn)
        async def wrapper(self, model_id: str | None = None):
            if model_id is None:
                model_id = get_multiplexed_model_id()
            state = self.__dict__.get(attr)
            if state is None:
                state = {"lru": collections.OrderedDict(), "inflight": {}}
                self.__dict__[attr] = state
            lru, inflight = state["lru"], state["inflight"]
            if model_id in lru:
                lru.move_to_end(model_id)
                return lru[model_id]
            if model_id in inflight:
                return await asyncio.shield(inflight[model_id])
            fut = asyncio.get_running_loop().create_future()
            inflight[model_id] = fut
            try:
                model = await fn(self, model_id)
            except BaseException as e:
                inflight.pop(model_id, None)
                if not fut.done():
                    fut.set_exception(e)
                    fut.exception()  # mark retrieved
                raise
            inflight.pop(model_id, None)
            lru[model_id] = model
            while len(lru) > max_num_models_per_replica:
                _, old = lru.popitem(last=False)
                unload = getattr(old, "unload", None)
                if callable(unload):
                    try:
                        r = unload()
                        if inspect.isawaitable(r):
                            await r
                    except Exception:
                        pass
            if not fut.done():
                fut.set_result(model)
            return model

        wrapper.__be_multiplexed__ = max_num_models_per_replica
        return wrapper

    if func is not None:
        return deco(func)
    return deco


# ---------------------------------------------------------------------------------- app control


def _controller():
    from .controller import get_controller

    return get_controller()


def run(target: Application, name: str = "default", route_prefix: str | None = None, blocking: bool = False,
        _local_testing_mode: bool = False, **kwargs):
    """Deploy an application.  Must be awaited (``await serve.run(...)``) inside a running event loop;
    when called without a loop it runs the deploy to completion and returns the ingress handle."""
    ctrl = _controller()
    coro = ctrl.deploy_application(target, name=name, route_prefix=route_prefix)
    try:
        asyncio.get_running_loop()
        return coro
    except RuntimeError:
        return asyncio.run(coro)


def run_async(target: Application, name: str = "default", route_prefix: str | None = None):
    return _controller().deploy_application(target, name=name, route_prefix=route_prefix)


def delete(name: str, _blocking: bool = True):
    coro = _controller().delete_application(name)
    try:
        asyncio.get_running_loop()
        return coro
    except RuntimeError:
        return asyncio.run(coro)


def status():
    return _controller().serve_status()


def get_app_handle(name: str):
    return _controller().get_app_handle(name)


def get_deployment_handle(deployment_name: str, app_name: str = "default"):
    from .handle import DeploymentHandle

    return DeploymentHandle(app_name, deployment_name)


def start(**_kwargs):
    _controller()


def shutdown():
    from .controller import shutdown_controller

    coro = shutdown_controller()
    try:
        asyncio.get_running_loop()
        return coro
    except RuntimeError:
        return asyncio.run(coro)


class ingress:  # noqa: N801 - FastAPI ingress is not supported (no HTTP proxy); kept for imports
    def __init__(self, app):
        self.app = app

    def __call__(self, cls):
        return cls
