"""BioEngineWorker: the ``bioengine-worker`` service.

Service surface identical to the reference (``bioengine/worker/worker.py:614-664``):
``get_status, stop_worker, check_access, get_logs, list_datasets, run_code, upload_app,
list_app_directories, clear_app_directory, list_apps, get_app_manifest, delete_app, deploy_app,
stop_app, stop_all_apps, get_app_status`` registered as ``{workspace}/{client_id}:bioengine-worker``
with ``type: bioengine-worker``, ``visibility: public``, ``require_context: True``.

Lifecycle (``:925-1001``): start the node cluster, connect to the hub/Hypha, verify the token can
mint admin tokens, resolve admin users, initialise the apps manager and code executor, discover the
datasets server, recover/launch apps, register the service, then run the monitoring loop (1 s tick,
work every ``monitoring_interval_seconds``: hub echo + reconnect/re-register, token renewal when
< 1 h remains, cluster monitoring / SLURM scaling, datasets server rediscovery, app health +
auto-redeploy; 5 consecutive failures => not ready => cleanup; ``:780-883``).  Graceful shutdown
with a timeout (``:885-923``).
"""
from __future__ import annotations

import asyncio
import logging
import os
import platform
import time
import uuid
from pathlib import Path
from typing import Any

from pydantic import Field

from .. import __version__
from ..apps.manager import AppsManager
from ..cluster.node import NodeCluster
from ..serve.controller import ServeController, set_controller
from ..serve.ray_compat import __version__ as RUNTIME_VERSION
from ..transport.client import connect_to_server
from ..transport.schema import schema_method
from ..utils.logger import create_logger
from ..utils.permissions import check_permissions, create_context, is_authorized
from .code_executor import CodeExecutor

SERVICE_METHODS = ("get_status", "stop_worker", "check_access", "get_logs", "list_datasets", "run_code", "upload_app",
                   "list_app_directories", "clear_app_directory", "list_apps", "get_app_manifest", "delete_app",
                   "deploy_app", "stop_app", "stop_all_apps", "get_app_status")


class BioEngineWorker:
    def __init__(self, mode: str = "single-machine", admin_users: list[str] | None = None,
                 workspace_dir: str | Path = "~/.bioengine", server_url: str = "local://default",
                 workspace: str | None = None, token: str | None = None, client_id: str | None = None,
                 service_id: str = "bioengine-worker", worker_name: str | None = None,
                 startup_applications: list[dict] | None = None, monitoring_interval_seconds: float = 10.0,
                 graceful_shutdown_timeout: float = 60.0, data_server_url: str | None = "auto",
                 log_file: str | None = None, debug: bool = False, head_num_cpus: float | None = None,
                 head_num_gpus: int | None = None, head_memory_in_gb: float | None = None,
                 slurm_workers=None, slurm_config: dict | None = None, **_ignored):
        self.mode = mode
        self.workspace_dir = Path(workspace_dir).expanduser().resolve()
        self.workspace_dir.mkdir(parents=True, exist_ok=True)
        if log_file is None:
            log_file = str(self.workspace_dir / "logs" / f"bioengine_worker_{time.strftime('%Y%m%d_%H%M%S')}.log")
        self.log_file = None if str(log_file).lower() == "off" else log_file
        self.log = create_logger("BioEngineWorker", logging.DEBUG if debug else logging.INFO, self.log_file)
        self.server_url = server_url
        self.workspace = workspace
        self._token = token or os.environ.get("HYPHA_TOKEN") or os.environ.get("BIOENGINE_TOKEN")
        self.client_id = client_id or f"bioengine-worker-{uuid.uuid4().hex[:8]}"
        self.service_id = service_id
        self.worker_name = worker_name or f"BioEngine Worker ({platform.node()})"
        self.admin_users_param = admin_users
        self.admin_users: list[str] = []
        self.startup_applications = startup_applications or []
        self.monitoring_interval = monitoring_interval_seconds
        self.graceful_shutdown_timeout = graceful_shutdown_timeout
        self.data_server_url_param = data_server_url
        self.data_server_url: str | None = None
        if slurm_workers is None and mode == "slurm":
            from ..cluster.slurm import SlurmWorkers

            slurm_workers = SlurmWorkers(server_url, self._token, self.workspace_dir, logger=self.log,
                                         **(slurm_config or {}))
        self.cluster = NodeCluster(mode, head_num_cpus, head_num_gpus, head_memory_in_gb, slurm_workers=slurm_workers,
                                   logger=self.log)
        self.controller = ServeController(resources=self.cluster.resources,
                                          log_dir=str(self.workspace_dir / "logs" / "replicas"))
        set_controller(self.controller)
        self.apps_manager = AppsManager(self.controller, self.cluster, self.workspace_dir / "apps",
                                        logger=self.log, state_file=self.workspace_dir / "apps_state.json")
        self.code_executor = CodeExecutor(self.cluster, logger=self.log)
        self.server = None
        self.start_time: float | None = None
        self.is_ready = asyncio.Event()
        self._stop_event = asyncio.Event()
        self._monitor_task = None
        self._token_expires_at = float("inf")
        self.geo_location: dict | None = None
        self._admin_context = None
        self.full_service_id: str | None = None

    # ------------------------------------------------------------------ connection
    async def _connect(self):
        cfg = {"server_url": self.server_url, "token": self._token, "client_id": self.client_id}
        if self.workspace:
            cfg["workspace"] = self.workspace
        self.server = await connect_to_server(cfg)
        self.workspace = self.server.config.workspace
        user = self.server.config.user or {}
        uid, email = user.get("id"), user.get("email")
        if self._token:
            try:  # the worker must be able to mint admin tokens for deployments (reference :522-612)
                probe = await self.server.generate_token({"workspace": self.workspace, "permission": "admin",
                                                          "expires_in": 3600 * 3})
                info = await self.server.parse_token(probe)
                self._token_expires_at = float(info.get("expires_at") or float("inf"))
            except Exception as e:  # noqa: BLE001
                raise PermissionError(f"The provided token cannot generate admin tokens: {e}") from e
        admins = list(self.admin_users_param or [])
        for v in (uid, email):
            if v and v not in admins:
                admins.append(v)
        self.admin_users = admins
        self._admin_context = create_context(uid, email)
        self.full_service_id = f"{self.workspace}/{self.client_id}:{self.service_id}"

    async def route_call(self, payload: bytes, context: dict | None = None) -> bytes:
        """Node agents route DeploymentHandle calls of their replicas through the head (admin only)."""
        import cloudpickle

        from ..utils.permissions import check_permissions

        check_permissions(context, self.admin_users, "route deployment calls")
        app, dep, method, args, kwargs, model_id = cloudpickle.loads(payload)
        try:
            val = await self.controller.call(app, dep, method, args, kwargs, model_id)
            return cloudpickle.dumps((True, val))
        except BaseException as e:  # noqa: BLE001
            return cloudpickle.dumps((False, e))

    async def _register_service(self):
        desc = {"slurm": "Manages BioEngine Apps and Datasets on a HPC system with SLURM autoscaling.",
                "single-machine": "Manages BioEngine Apps and Datasets on a single machine (native MI355X runtime).",
                "external-cluster": "Manages BioEngine Apps and Datasets on an existing cluster."}[self.mode]
        methods = {
            "get_status": self.get_status, "stop_worker": self.stop, "check_access": self.check_access,
            "get_logs": self.get_logs, "list_datasets": self.list_datasets, "run_code": self.code_executor.run_code,
            "upload_app": self.apps_manager.upload_app, "list_app_directories": self.apps_manager.list_app_directories,
            "clear_app_directory": self.apps_manager.clear_app_directory, "list_apps": self.apps_manager.list_apps,
            "get_app_manifest": self.apps_manager.get_app_manifest, "delete_app": self.apps_manager.delete_app,
            "deploy_app": self.apps_manager.deploy_app, "stop_app": self.apps_manager.stop_app,
            "stop_all_apps": self.apps_manager.stop_all_apps, "get_app_status": self.apps_manager.get_app_status,
            "route_call": self.route_call,
        }
        info = await self.server.register_service({
            "id": self.service_id, "name": self.worker_name, "type": "bioengine-worker", "description": desc,
            "config": {"visibility": "public", "require_context": True}, **methods})
        if info["id"] != self.full_service_id:
            raise ValueError(f"Service ID mismatch: {self.full_service_id} vs {info['id']}")

    async def _discover_data_server(self):
        from ..datasets.client import BioEngineDatasets

        url = BioEngineDatasets.discover() if self.data_server_url_param == "auto" else self.data_server_url_param
        self.data_server_url = url
        self.apps_manager.data_server_url = url
        if self.apps_manager.builder is not None:
            self.apps_manager.builder.data_server_url = url

    # ------------------------------------------------------------------ start/stop
    async def start(self, blocking: bool = True):
        self.start_time = time.time()
        await self.cluster.start()
        await self._connect()
        self.cluster.attach(self.server, self.controller)
        await self._discover_data_server()
        await self.apps_manager.complete_initialization(self.server, self.admin_users, self.full_service_id,
                                                        self.server_url, self._token)
        self.apps_manager.data_server_url = self.data_server_url
        self.apps_manager.builder.data_server_url = self.data_server_url
        await self.code_executor.initialize(self.admin_users)
        try:
            recovered = await self.apps_manager.recover_deployed_applications(self._admin_context)
            if recovered:
                self.log.info(f"Recovered applications: {recovered}")
        except Exception as e:  # noqa: BLE001
            self.log.error(f"app recovery failed: {e}")
        await self.apps_manager.deploy_startup_applications(self.startup_applications, self._admin_context)
        await self._register_service()
        self.is_ready.set()
        from ..runtime.gcpolicy import serving_gc

        serving_gc()  # router / bridge / hub share this loop: keep gen-2 GC pauses out of request latency
        self._monitor_task = asyncio.ensure_future(self._monitor())
        self.log.info(f"BioEngine worker ready: service '{self.full_service_id}' on {self.server_url}")
        if blocking:
            await self._stop_event.wait()
        return self.full_service_id

    async def _monitor(self):
        errors = 0
        last = 0.0
        try:
            while not self._stop_event.is_set():
                await asyncio.sleep(1.0)
                if time.time() - last < self.monitoring_interval:
                    continue
                last = time.time()
                try:
                    await self._check_hub()
                    if self._token_expires_at - time.time() < 3600:
                        self._token = await self.server.generate_token({"workspace": self.workspace, "permission": "admin",
                                                                        "expires_in": 3600 * 3})
                        self._token_expires_at = float((await self.server.parse_token(self._token)).get("expires_at")
                                                       or float("inf"))
                    await self.cluster.monitor_cluster()
                    if self.data_server_url is None and self.data_server_url_param == "auto":
                        await self._discover_data_server()
                    await self.apps_manager.monitor_applications(self._admin_context)
                    errors = 0
                    self.is_ready.set()
                except Exception as e:  # noqa: BLE001
                    errors += 1
                    self.log.error(f"monitoring error ({errors}/5): {e}")
                    if errors >= 5:
                        self.is_ready.clear()
                        await self._cleanup()
                        return
        except asyncio.CancelledError:
            pass

    async def _check_hub(self):
        try:
            await asyncio.wait_for(self.server.echo("ping"), timeout=10)
        except Exception:
            self.log.warning("hub connection lost; reconnecting")
            await self._connect()
            await self._register_service()

    async def _cleanup(self):
        try:
            await asyncio.wait_for(self.apps_manager.stop_all_apps(context=self._admin_context),
                                   timeout=self.graceful_shutdown_timeout)
        except Exception as e:  # noqa: BLE001
            self.log.error(f"stopping apps during cleanup failed: {e}")
        await self.cluster.stop()  # SLURM nodes are shut down through the hub: before disconnecting
        await self.controller.shutdown()
        if self.server is not None:
            try:
                await self.server.unregister_service(self.service_id)
            except Exception:  # noqa: BLE001
                pass
            server = self.server

            async def _disconnect():
                # deferred so that a stop_worker(blocking=True) RPC can still deliver its reply
                await asyncio.sleep(0.25)
                try:
                    await server.disconnect()
                except Exception:  # noqa: BLE001
                    pass

            self._disconnect_task = asyncio.ensure_future(_disconnect())
        self.is_ready.clear()

    async def _stop(self, blocking: bool = False):
        if self._monitor_task is not None:
            self._monitor_task.cancel()
        self.apps_manager.state_file = None  # an explicit stop does not redeploy on the next start

        async def go():
            try:
                await asyncio.wait_for(self._cleanup(), timeout=self.graceful_shutdown_timeout)
            finally:
                self._stop_event.set()

        if blocking:
            await go()
        else:
            asyncio.ensure_future(go())

    # ------------------------------------------------------------------ service methods
    @schema_method
    async def get_status(self, context: dict = Field(..., description="Injected context.")) -> dict:
        """Worker status: uptime, versions, mode, cluster resources (per node and GPU), admins, readiness."""
        now = time.time()
        return {"service_start_time": self.start_time, "service_uptime": now - self.start_time if self.start_time else 0,
                "bioengine_version": __version__, "ray_version": RUNTIME_VERSION, "worker_mode": self.mode,
                "workspace": self.workspace, "client_id": self.client_id, "ray_cluster": self.cluster.status,
                "admin_users": self.admin_users, "geo_location": self.geo_location, "is_ready": self.is_ready.is_set(),
                "serving": {n: {"status": a.status, "deployments": {d: ds.status_dict() for d, ds in a.deployments.items()}}
                            for n, a in self.controller.apps.items()}}

    @schema_method
    async def stop(self, blocking: bool = Field(False, description="Wait for the shutdown to finish."),
                   context: dict = Field(..., description="Injected context.")) -> None:
        """Gracefully shut down the worker (admin only)."""
        check_permissions(context, self.admin_users, "shutdown the BioEngine worker")
        await self._stop(blocking)

    @schema_method
    async def check_access(self, context: dict = Field(..., description="Injected context.")) -> bool:
        """True when the caller is a worker admin."""
        return is_authorized(context, self.admin_users)

    @schema_method
    async def get_logs(self, tail: int = Field(200, description="Number of trailing lines (-1 = all)."),
                       context: dict = Field(..., description="Injected context.")) -> list:
        """Worker log lines (admin only)."""
        check_permissions(context, self.admin_users, "read the worker logs")
        if not self.log_file:
            return []
        try:
            lines = Path(self.log_file).read_text(errors="replace").splitlines()
        except OSError as e:
            raise RuntimeError(f"Failed to read log file {self.log_file}: {e}") from e
        return lines if tail is None or tail < 0 else lines[-tail:]

    @schema_method
    async def list_datasets(self, context: dict = Field(..., description="Injected context.")) -> dict:
        """Datasets published by the discovered datasets server."""
        from ..datasets.client import BioEngineDatasets

        if not self.data_server_url:
            await self._discover_data_server()
        if not self.data_server_url:
            return {}
        c = BioEngineDatasets(self.data_server_url)
        try:
            return await c.list_datasets()
        finally:
            await c.close()
