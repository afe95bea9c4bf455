"""AppsManager: application lifecycle behind the worker service.

API parity with ``bioengine/apps/manager.py`` (method names, parameters, defaults and return
shapes): ``deploy_app`` (``:1469-1814``), ``stop_app`` (``:1816-1887``),
``stop_all_apps`` (``:1889-1984``), ``get_app_status`` (``:1986-2097``), ``upload_app``
(``:1073-1182``), ``list_apps`` (``:1306-1354``), ``get_app_manifest`` (``:1356-1405``),
``delete_app`` (``:1407-1467``), ``list_app_directories`` / ``clear_app_directory``
(``:1184-1304``), startup apps (``:937-1001``), auto-redeploy monitor (``:1003-1071``).

Differences by design:

* apps are served by the native :class:`~bioengine_worker_amd.serve.controller.ServeController`
  and exposed by an in-worker :class:`~.bridge.AppServiceBridge` (no Ray / ProxyDeployment);
* deployed-app records are persisted (``<workspace>/apps_state.json``) so a restarted worker
  redeploys the apps it was running (the reference recovers from a Ray cluster that outlived the
  worker, ``:841-935``; without Ray the worker owns its replicas, so it replays its own records).
"""
from __future__ import annotations

import asyncio
import json
import logging
import random
import shutil
import time
from pathlib import Path
from typing import Any

from pydantic import Field

from ..serve.controller import ServeController
from ..transport.schema import schema_method
from ..utils.artifact_utils import create_application_from_files, get_static_site_url, load_manifest_from_files
from ..utils.permissions import check_permissions, user_identity
from .bridge import AppServiceBridge
from .builder import AppBuilder

_ADJ = ("amber", "brave", "calm", "dapper", "eager", "fancy", "gentle", "happy", "icy", "jolly", "keen", "lively",
        "mellow", "nimble", "odd", "proud", "quiet", "rapid", "shiny", "tidy", "upbeat", "vivid", "witty", "zesty",
        "bold", "crisp", "dusty", "fuzzy", "glossy", "hidden", "lucky", "misty", "noble", "plucky", "royal", "silent")
_NOUN = ("otter", "falcon", "badger", "lynx", "heron", "walrus", "gecko", "koala", "marten", "newt", "ocelot",
         "panda", "quail", "raven", "salmon", "tapir", "urchin", "viper", "wombat", "yak", "zebra", "bison", "crane",
         "dingo", "egret", "ferret", "gibbon", "hare", "ibis", "jackal", "kiwi", "lemur", "moose", "narwhal")

APP_STATES = ("NOT_STARTED", "DEPLOYING", "DEPLOY_FAILED", "RUNNING", "UNHEALTHY", "DELETING")
CTX = Field(..., description="Authentication context, automatically provided by the hub/Hypha during service calls.")


class AppsManager:
    def __init__(self, controller: ServeController, cluster, apps_workdir: str | Path, admin_users: list[str] | None = None,
                 data_server_url: str | None = None, logger: logging.Logger | None = None,
                 state_file: str | Path | None = None, monitor_interval: float = 10.0):
        self.controller = controller
        self.cluster = cluster
        self.apps_workdir = Path(apps_workdir)
        self.apps_workdir.mkdir(parents=True, exist_ok=True)
        self.admin_users = list(admin_users or [])
        self.data_server_url = data_server_url
        self.log = logger or logging.getLogger("bioengine.apps")
        self.state_file = Path(state_file) if state_file else None
        self.server = None
        self.server_url = None
        self.token = None
        self.artifact_manager = None
        self.worker_service_id = None
        self.builder: AppBuilder | None = None
        self.apps: dict[str, dict] = {}
        self._lock = asyncio.Lock()
        self.monitor_interval = monitor_interval

    # ------------------------------------------------------------------ init
    async def complete_initialization(self, server, admin_users: list[str], worker_service_id: str, server_url: str,
                                      token: str | None):
        self.server = server
        self.server_url = server_url
        self.token = token
        self.admin_users = list(admin_users)
        self.worker_service_id = worker_service_id
        try:
            self.artifact_manager = await server.get_service("public/artifact-manager")
        except Exception as e:  # noqa: BLE001
            self.log.warning(f"artifact manager unavailable: {e}")
            self.artifact_manager = None
        if self.artifact_manager is not None:
            from ..utils.artifact_utils import ensure_applications_collection

            try:
                await ensure_applications_collection(self.artifact_manager, server.config.workspace, self.log)
            except Exception as e:  # noqa: BLE001
                self.log.warning(f"could not ensure applications collection: {e}")
        self.builder = AppBuilder(self.apps_workdir, server, self.artifact_manager, self.data_server_url,
                                  worker_service_id, self.log)

    def _check_admin(self, context, what: str):
        check_permissions(context, self.admin_users, what)

    def _full_artifact_id(self, artifact_id: str) -> str:
        if "/" in artifact_id or Path(artifact_id).is_dir():
            return artifact_id
        return f"{self.server.config.workspace}/{artifact_id}"

    def _new_app_id(self) -> str:
        for _ in range(1000):
            aid = f"{random.choice(_ADJ)}-{random.choice(_NOUN)}"
            if aid not in self.apps:
                return aid
        return f"app-{int(time.time() * 1000) % 10 ** 8}"

    # ------------------------------------------------------------------ persistence
    def _save_state(self):
        if self.state_file is None:
            return
        recs = {}
        for aid, a in self.apps.items():
            if a.get("status") in ("DELETING",):
                continue
            recs[aid] = {k: a[k] for k in ("artifact_id", "version", "application_kwargs", "application_env_vars_raw",
                                            "disable_gpu", "max_ongoing_requests", "auto_redeploy", "debug",
                                            "authorized_users_param", "started_at", "last_updated_by") if k in a}
        tmp = self.state_file.with_suffix(".tmp")
        tmp.write_text(json.dumps(recs, default=str))
        tmp.replace(self.state_file)

    async def recover_deployed_applications(self, context) -> list[str]:
        if self.state_file is None or not self.state_file.exists():
            return []
        try:
            recs = json.loads(self.state_file.read_text())
        except Exception:
            return []
        out = []
        for aid, r in recs.items():
            try:
                await self.deploy_app(artifact_id=r["artifact_id"], version=r.get("version"), application_id=aid,
                                      application_kwargs=r.get("application_kwargs"),
                                      application_env_vars=r.get("application_env_vars_raw"),
                                      disable_gpu=r.get("disable_gpu", False),
                                      max_ongoing_requests=r.get("max_ongoing_requests", 10),
                                      auto_redeploy=r.get("auto_redeploy", False), debug=r.get("debug", False),
                                      authorized_users=r.get("authorized_users_param"), context=context)
                self.apps[aid]["recovered_app"] = True
                out.append(aid)
            except Exception as e:  # noqa: BLE001
                self.log.error(f"recovery of '{aid}' failed: {e}")
        return out

    # ------------------------------------------------------------------ deployment core
    def _check_resources(self, required: dict):
        res = self.controller.resources
        need_cpu, need_gpu = float(required.get("num_cpus", 0)), float(required.get("num_gpus", 0))
        free_cpu = res.total_cpu - res.used_cpu
        free_gpu = sum(1 for g in res.gpu_ids if res.gpu_used[g] == 0.0)
        if need_cpu <= free_cpu + 1e-9 and need_gpu <= free_gpu + 1e-9:
            return
        if getattr(self.cluster, "mode", "") == "slurm":
            self.log.info("insufficient local resources; SLURM autoscaling may provide them")
            return
        if getattr(self.cluster, "mode", "") == "external-cluster":
            self.log.warning("insufficient resources on the external cluster; deployment may stay pending")
            return
        raise RuntimeError(f"Insufficient resources: application needs num_cpus={need_cpu:g}, num_gpus={need_gpu:g}; "
                           f"available num_cpus={free_cpu:g}, num_gpus={free_gpu:g}")

    async def _run_deployment(self, aid: str):
        rec = self.apps[aid]
        built = rec["built"]
        try:
            reqs = built.metadata.get("pip_requirements") or []
            if reqs:
                from . import requirements

                rec["message"] = f"Resolving pip requirements {reqs}"
                rec["pip"] = await asyncio.to_thread(requirements.ensure, reqs,
                                                     self.builder.apps_workdir / aid / "site-packages")
                rec["message"] = ""
            handle = await self.controller.deploy_application(built.root, name=aid, route_prefix=f"/{aid}")
            bridge = AppServiceBridge(aid, built, handle, self.server_url, self.token,
                                      self.server.config.workspace, self.server.config.client_id, self.log)
            await bridge.start()
            rec["bridge"] = bridge
            rec["status"] = "RUNNING"
            rec["message"] = ""
            rec["is_deployed"] = True
            self.log.info(f"Application '{aid}' is RUNNING ({bridge.service_id})")
        except asyncio.CancelledError:
            rec["status"] = "DEPLOY_FAILED"
            rec["message"] = "deployment cancelled"
            raise
        except BaseException as e:  # noqa: BLE001
            rec["status"] = "DEPLOY_FAILED"
            rec["message"] = f"{type(e).__name__}: {e}"
            self.log.error(f"Deployment of '{aid}' failed: {e}")

    async def _undeploy(self, aid: str):
        rec = self.apps.get(aid)
        if rec is None:
            return
        rec["status"] = "DELETING"
        t = rec.get("task")
        if t is not None and not t.done():
            t.cancel()
            try:
                await t
            except BaseException:
                pass
        b = rec.get("bridge")
        if b is not None:
            await b.stop()
        await self.controller.delete_application(aid)
        self.apps.pop(aid, None)
        self._save_state()

    # ------------------------------------------------------------------ service methods
    @schema_method
    async def deploy_app(
        self,
        artifact_id: str = Field(..., description="Application artifact id ('workspace/alias' or alias), or a local app directory."),
        version: str | None = Field(None, description="Artifact version (latest if omitted; kept on update)."),
        application_id: str | None = Field(None, description="Application instance id; random if omitted; an existing id updates that app."),
        application_kwargs: dict | None = Field(None, description="{DeploymentClass: {init_kwarg: value}}"),
        application_env_vars: dict | None = Field(None, description="{DeploymentClass: {ENV: value}}; keys starting with '_' are secret."),
        hypha_token: str | None = Field(None, description="Token injected into replicas as HYPHA_TOKEN (secret)."),
        disable_gpu: bool = Field(False, description="Force all deployments to num_gpus=0."),
        max_ongoing_requests: int = Field(10, description="Concurrent requests admitted by the app service."),
        auto_redeploy: bool = Field(False, description="Redeploy automatically on DEPLOY_FAILED / UNHEALTHY."),
        debug: bool = Field(False, description="DEBUG logging in all replicas."),
        ice_servers: list | None = Field(None, description="WebRTC ICE servers."),
        authorized_users: Any = Field(None, description="{method: [users]} or [users] (= {'*': [users]})."),
        context: dict = CTX,
    ) -> str:
        """Deploy (or update) an application from an artifact. Returns the application id; the
        deployment continues in the background — poll get_app_status."""
        self._check_admin(context, "deploy applications")
        async with self._lock:
            if not self.controller.resources:
                raise RuntimeError("cluster not ready")
            aid = application_id or self._new_app_id()
            prev = self.apps.get(aid)
            if prev is not None:  # update: inherit unspecified params
                version = version if version is not None else prev.get("version")
                application_kwargs = application_kwargs if application_kwargs is not None else prev.get("application_kwargs")
                application_env_vars = application_env_vars if application_env_vars is not None else prev.get("application_env_vars_raw")
                authorized_users = authorized_users if authorized_users is not None else prev.get("authorized_users_param")
                ice_servers = ice_servers if ice_servers is not None else prev.get("ice_servers")
                started_at = prev.get("started_at")
                await self._undeploy(aid)
            else:
                started_at = None
            full_id = self._full_artifact_id(artifact_id)
            uid, email = user_identity(context)
            built = await self.builder.build(
                application_id=aid, artifact_id=full_id, version=version, application_kwargs=application_kwargs,
                application_env_vars=application_env_vars, hypha_token=hypha_token, disable_gpu=disable_gpu,
                max_ongoing_requests=max_ongoing_requests, debug=debug, started_at=started_at,
                last_updated_by=uid, auto_redeploy=auto_redeploy, ice_servers=ice_servers,
                authorized_users=authorized_users, deploying_user=(uid, email), admin_users=self.admin_users)
            self._check_resources(built.metadata["application_resources"])
            static_url = None
            if built.manifest.get("frontend_entry") and "/" in full_id and not Path(full_id).is_dir():
                static_url = get_static_site_url(full_id, self.server.config.public_base_url or self.server_url)
            rec = dict(built.metadata)
            rec.update({"built": built, "status": "DEPLOYING", "message": "", "recovered_app": False,
                        "is_deployed": False, "application_env_vars_raw": application_env_vars or {},
                        "authorized_users_param": authorized_users, "static_site_url": static_url,
                        "version": built.metadata.get("version")})
            self.apps[aid] = rec
            rec["task"] = asyncio.ensure_future(self._run_deployment(aid))
            self._save_state()
        return aid

    @schema_method
    async def stop_app(self, application_id: str = Field(..., description="Application id to stop."),
                       context: dict = CTX) -> None:
        """Stop a running application and remove its service."""
        self._check_admin(context, f"stop application '{application_id}'")
        if application_id not in self.apps:
            raise ValueError(f"Application '{application_id}' is not deployed")
        await self._undeploy(application_id)

    @schema_method
    async def stop_all_apps(self, context: dict = CTX) -> dict:
        """Stop every application. Returns {application_id: success}."""
        self._check_admin(context, "stop all applications")
        out = {}
        for aid in list(self.apps):
            try:
                await self._undeploy(aid)
                out[aid] = True
            except Exception as e:  # noqa: BLE001
                self.log.error(f"stopping '{aid}' failed: {e}")
                out[aid] = False
        return out

    async def _deployments_status(self, aid: str, logs_tail: int, n_previous: int) -> dict:
        app = self.controller.apps.get(aid)
        if app is None:
            return {}
        out = {}
        for name, ds in app.deployments.items():
            logs = {}
            for r in ds.replicas:
                logs[r.tag] = r.logs(logs_tail if logs_tail >= 0 else 0)
            prev = ds.history if n_previous < 0 else ds.history[-n_previous:] if n_previous > 0 else []
            for h in prev:
                logs[h["replica_id"]] = h["logs"][-logs_tail:] if logs_tail > 0 else h["logs"]
            st = ds.status_dict()
            out[name] = {"status": st["status"], "message": st["message"], "replica_states": st["replica_states"],
                         "logs": logs, "ongoing_requests": st["ongoing_requests"], "latency_ms": st["latency_ms"],
                         "requests_total": st["requests_total"]}
        return out

    async def _app_status(self, aid: str, logs_tail: int, n_previous: int) -> dict:
        rec = self.apps.get(aid)
        if rec is None:
            return {"status": "NOT_RUNNING",
                    "message": f"Application '{aid}' is not currently deployed. To deploy it, call "
                               f"deploy_app(application_id='{aid}', ...)."}
        status, message = rec["status"], rec.get("message", "")
        capp = self.controller.apps.get(aid)
        if status == "RUNNING" and capp is not None and capp.status == "UNHEALTHY":
            status, message = "UNHEALTHY", capp.message
        bridge = rec.get("bridge")
        sids = bridge.service_ids() if bridge else []
        static = None
        if rec.get("static_site_url") and sids:
            static = (f"{rec['static_site_url']}?server={self.server.config.public_base_url}"
                      f"&ws_service_id={sids[0]['websocket_service_id']}&webrtc_service_id={sids[0]['webrtc_service_id'] or ''}")
        return {
            "display_name": rec["display_name"], "description": rec["description"], "artifact_id": rec["artifact_id"],
            "version": rec.get("version") or "latest", "recovered_app": rec.get("recovered_app", False),
            "status": status, "message": message,
            "deployments": await self._deployments_status(aid, logs_tail, n_previous),
            "application_kwargs": rec.get("application_kwargs"), "application_env_vars": rec.get("application_env_vars"),
            "gpu_enabled": not rec.get("disable_gpu", False), "application_resources": rec.get("application_resources"),
            "authorized_users": rec.get("authorized_users"), "available_methods": rec.get("available_methods"),
            "max_ongoing_requests": rec.get("max_ongoing_requests"), "static_site_url": static, "service_ids": sids,
            "start_time": rec.get("started_at"), "last_updated_at": rec.get("last_updated_at"),
            "last_updated_by": rec.get("last_updated_by"), "auto_redeploy": rec.get("auto_redeploy", False),
            "metrics": bridge.metrics() if bridge else None,
        }

    @schema_method
    async def get_app_status(
        self,
        application_ids: list | None = Field(None, description="Application ids (all if omitted; a single id returns its status directly)."),
        logs_tail: int = Field(30, description="Log lines per replica (-1 = all)."),
        n_previous_replica: int = Field(0, description="Also include logs of this many previous replicas (-1 = all)."),
        context: dict = CTX,
    ) -> dict:
        """Status of deployed applications (public: no admin needed)."""
        ids = application_ids if application_ids is not None else list(self.apps)
        if isinstance(ids, str):
            ids = [ids]
        res = {aid: await self._app_status(aid, logs_tail, n_previous_replica) for aid in ids}
        if application_ids is not None and len(ids) == 1:
            return res[ids[0]]
        return res

    @schema_method
    async def upload_app(
        self,
        files: list = Field(..., description="[{name, content, type: 'text'|'base64'}], must include manifest.yaml."),
        workspace: str | None = Field(None, description="Target workspace (with hypha_token: no admin needed)."),
        hypha_token: str | None = Field(None, description="Token for the target workspace."),
        context: dict = CTX,
    ) -> str:
        """Create or update an application artifact from files. Returns the artifact id."""
        manifest = load_manifest_from_files(files)
        if workspace and hypha_token:
            from ..transport.client import connect_to_server

            client = await connect_to_server({"server_url": self.server_url, "token": hypha_token, "workspace": workspace})
            try:
                am = await client.get_service("public/artifact-manager")
                return await create_application_from_files(am, files, workspace, self.log)
            finally:
                await client.disconnect()
        self._check_admin(context, "upload applications")
        uid, _ = user_identity(context)
        if self.artifact_manager is None:
            raise RuntimeError("artifact manager unavailable")
        aid = await create_application_from_files(self.artifact_manager, files, self.server.config.workspace, self.log)
        self.log.info(f"User '{uid}' uploaded '{aid}' ({manifest.get('version')})")
        return aid

    @schema_method
    async def list_apps(self, context: dict = CTX) -> dict:
        """All application artifacts in the worker's workspace: {artifact_id: {manifest, files}}."""
        self._check_admin(context, "list applications")
        coll = f"{self.server.config.workspace}/applications"
        out = {}
        for art in await self.artifact_manager.list(coll):
            try:
                files = await self.artifact_manager.list_files(art["id"])
                out[art["id"]] = {"manifest": art.get("manifest"), "files": [f["name"] for f in files],
                                  "versions": [v["version"] for v in art.get("versions") or []]}
            except Exception as e:  # noqa: BLE001
                out[art["id"]] = {"error": str(e)}
        return out

    @schema_method
    async def get_app_manifest(self, artifact_id: str = Field(..., description="Artifact id."),
                               version: str | None = Field(None, description="Version (latest if omitted)."),
                               context: dict = CTX) -> dict:
        """Manifest of an application artifact."""
        self._check_admin(context, "read application manifests")
        art = await self.artifact_manager.read(self._full_artifact_id(artifact_id), version=version)
        return art.get("manifest")

    @schema_method
    async def delete_app(self, artifact_id: str = Field(..., description="Artifact id to delete."), context: dict = CTX) -> None:
        """Delete an application artifact (stop running instances first)."""
        self._check_admin(context, "delete applications")
        full = self._full_artifact_id(artifact_id)
        running = [aid for aid, r in self.apps.items() if r.get("artifact_id") == full]
        if running:
            raise ValueError(f"Artifact '{full}' is used by running applications {running}; stop them first")
        await self.artifact_manager.delete(full)

    @schema_method
    async def list_app_directories(self, context: dict = CTX) -> list:
        """Application working directories under the apps workspace."""
        self._check_admin(context, "list application directories")
        out = []
        for d in sorted(self.apps_workdir.iterdir()) if self.apps_workdir.exists() else []:
            if not d.is_dir():
                continue
            size = sum(p.stat().st_size for p in d.rglob("*") if p.is_file())
            out.append({"name": d.name, "path": str(d), "size_bytes": size, "is_running": d.name in self.apps})
        return out

    @schema_method
    async def clear_app_directory(self, application_id: str = Field(..., description="Directory (application id) to delete."),
                                  context: dict = CTX) -> None:
        """Delete an application's working directory (not allowed while it runs)."""
        self._check_admin(context, "clear application directories")
        if "/" in application_id or application_id in (".", "..", ""):
            raise ValueError("invalid application id")
        if application_id in self.apps:
            raise ValueError(f"Application '{application_id}' is running; stop it first")
        d = self.apps_workdir / application_id
        if not d.is_dir():
            raise ValueError(f"No working directory for '{application_id}'")
        shutil.rmtree(d)

    # ------------------------------------------------------------------ startup + monitoring
    async def deploy_startup_applications(self, startup: list[dict], context) -> list[str]:
        out = []
        for cfg in startup or []:
            cfg = dict(cfg)
            aid = await self.deploy_app(context=context, **{k: v for k, v in cfg.items() if k != "context"})
            out.append(aid)
        return out

    async def wait_for(self, application_id: str, timeout: float = 120.0, states=("RUNNING", "DEPLOY_FAILED")) -> str:
        t0 = time.time()
        while time.time() - t0 < timeout:
            rec = self.apps.get(application_id)
            if rec is not None and rec["status"] in states:
                return rec["status"]
            await asyncio.sleep(0.05)
        raise TimeoutError(f"application '{application_id}' did not reach {states} in {timeout}s")

    async def monitor_applications(self, context):
        for aid, rec in list(self.apps.items()):
            capp = self.controller.apps.get(aid)
            status = rec["status"]
            if status == "RUNNING" and capp is not None and capp.status == "UNHEALTHY":
                status = "UNHEALTHY"
            b = rec.get("bridge")
            if b is not None:
                if status == "UNHEALTHY" and b.registered:
                    await b.deregister()
                elif status == "RUNNING" and not b.registered:
                    await b.reregister()
            if rec.get("auto_redeploy") and status in ("DEPLOY_FAILED", "UNHEALTHY"):
                self.log.warning(f"auto-redeploying '{aid}' ({status})")
                try:
                    await self.deploy_app(artifact_id=rec["artifact_id"], application_id=aid, context=context)
                except Exception as e:  # noqa: BLE001
                    self.log.error(f"auto-redeploy of '{aid}' failed: {e}")
