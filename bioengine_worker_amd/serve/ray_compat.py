"""Build a ``ray`` module namespace backed by the native runtime (for unmodified app code).

Installed into ``sys.modules`` by :func:`bioengine_worker_amd.compat.install` only when the real Ray
is not importable, so ``from ray import serve``, ``from ray.serve.handle import DeploymentHandle``,
``from ray.exceptions import RayTaskError`` and ``ray.remote(...)`` keep working in app code.
"""
from __future__ import annotations

import types

from . import api, handle, tasks
from .controller import BackPressureError, DeploymentUnavailableError

__version__ = "2.55.1+bioengine.native"


def _module(name: str, **attrs) -> types.ModuleType:
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    return m


def build_modules() -> dict[str, types.ModuleType]:
    exceptions = _module("ray.exceptions", RayTaskError=tasks.RayTaskError, GetTimeoutError=tasks.GetTimeoutError,
                         RayActorError=RuntimeError, TaskCancelledError=RuntimeError, RayError=Exception,
                         ObjectLostError=RuntimeError)
    serve_handle = _module("ray.serve.handle", DeploymentHandle=handle.DeploymentHandle,
                           DeploymentResponse=handle.DeploymentResponse)
    serve_exc = _module("ray.serve.exceptions", BackPressureError=BackPressureError,
                        RayServeException=RuntimeError, DeploymentUnavailableError=DeploymentUnavailableError)
    serve = _module("ray.serve",
                    deployment=api.deployment, multiplexed=api.multiplexed, batch=api.batch,
                    get_multiplexed_model_id=api.get_multiplexed_model_id,
                    get_replica_context=api.get_replica_context, run=api.run, delete=api.delete,
                    status=api.status, start=api.start, shutdown=api.shutdown, get_app_handle=api.get_app_handle,
                    get_deployment_handle=api.get_deployment_handle, Application=api.Application,
                    Deployment=api.Deployment, ingress=api.ingress, handle=serve_handle, exceptions=serve_exc)
    serve.__path__ = []  # make it a package for submodule imports
    runtime_ctx = _module("ray.runtime_context", get_runtime_context=lambda: _RuntimeCtx())

    def is_initialized():
        return True

    def init(*a, **k):
        return None

    def _res():
        from .controller import get_controller

        return get_controller().resources

    ray = _module("ray", __version__=__version__, remote=tasks.remote, get=tasks.get, put=tasks.put, wait=tasks.wait,
                  ObjectRef=tasks.ObjectRef, init=init, is_initialized=is_initialized, shutdown=lambda: None,
                  available_resources=lambda: {"CPU": _res().total_cpu - _res().used_cpu,
                                               "GPU": _res().total_gpu - _res().used_gpu},
                  cluster_resources=lambda: {"CPU": _res().total_cpu, "GPU": _res().total_gpu},
                  nodes=lambda: [{"NodeID": "head", "Alive": True, "Resources": {"CPU": _res().total_cpu,
                                                                              "GPU": _res().total_gpu}}],
                  get_runtime_context=lambda: _RuntimeCtx(), exceptions=exceptions, serve=serve,
                  runtime_context=runtime_ctx)
    ray.__path__ = []
    return {"ray": ray, "ray.serve": serve, "ray.serve.handle": serve_handle, "ray.serve.exceptions": serve_exc,
            "ray.exceptions": exceptions, "ray.runtime_context": runtime_ctx}


class _RuntimeCtx:
    def get_node_id(self):
        return "head"

    def get_job_id(self):
        return "bioengine"

    def get_accelerator_ids(self):
        import os

        v = os.environ.get("HIP_VISIBLE_DEVICES", "")
        return {"GPU": [x for x in v.split(",") if x]}
