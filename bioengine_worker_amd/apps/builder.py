"""AppBuilder: app artifact (manifest + Python files) -> deployable application graph.

Behavioural parity with the reference builder (``bioengine/apps/builder.py``):

* manifest from a local directory (``BIOENGINE_LOCAL_ARTIFACT_PATH`` or a directory path) or from
  the artifact manager (``:219-298``), validated (``artifact_utils.validate_manifest``);
* each ``file:Class`` is downloaded and ``exec``'d with the app's env vars as globals
  (``:1148-1215``); ``from ray import serve`` resolves to the native runtime;
* actor options rewritten: ``num_gpus=0`` when GPU is disabled, runtime env vars ``HOME``,
  ``TMPDIR``, ``HYPHA_SERVER_URL``, ``HYPHA_WORKSPACE``, ``HYPHA_ARTIFACT_ID``,
  ``BIOENGINE_WORKER_SERVICE_ID`` (``:385-398``), secrets (keys starting with ``_``) masked as
  ``*****`` until the replica's ``__init__`` (``:381-383,652-654``); ``runtime_env.pip`` pinned
  (``:345-372``) and satisfied before deployment by :mod:`.requirements` (installed offline from
  ``BIOENGINE_WHEELHOUSE`` into the app's ``site-packages``, else ``DEPLOY_FAILED`` naming them);
* lifecycle wrapping (``:532-890``): ``__init__`` (workdir, state flags, ``self.bioengine_datasets``),
  ``async_init`` (once), ``test_deployment`` (background, failure => unhealthy) and
  ``check_health`` (lazy init + test + datasets ping + user check);
* init kwargs validated against the class signature (``:892-1087``);
* composition: extra deployments bind to the entry ``__init__`` parameter named after their file
  stem (``:1474-1508``);
* summed resources (``:1248-1294``), entry ``@schema_method`` schemas (``:1453-1465``),
  ``authorized_users`` resolution with deploying-user/admin injection (``:1522-1569``).

Instead of binding a Ray ``ProxyDeployment`` in front of the entry, the resulting
:class:`BuiltApp` is served by an :class:`~.bridge.AppServiceBridge` inside the worker (one less
process hop per request).
"""
from __future__ import annotations

import asyncio
import copy
import inspect
import logging
import os
import sys
import time
from dataclasses import dataclass, field
from functools import wraps
from pathlib import Path
from typing import Any

import httpx
import yaml

from ..serve.api import Application, Deployment, deployment as serve_deployment
from ..utils.artifact_utils import validate_manifest
from .requirements import update_requirements

SECRET_MASK = "*****"


@dataclass
class BuiltApp:
    application_id: str
    root: Application
    manifest: dict
    metadata: dict
    method_schemas: list[dict] = field(default_factory=list)


def _merge_env(base: dict, extra: dict) -> dict:
    out = dict(base)
    out.update(extra)
    return out


class AppBuilder:
    def __init__(self, apps_workdir: str | Path, server=None, artifact_manager=None, data_server_url: str | None = None,
                 worker_service_id: str | None = None, logger: logging.Logger | None = None,
                 local_artifact_path: str | Path | None = None):
        self.apps_workdir = Path(apps_workdir)
        self.server = server
        self.artifact_manager = artifact_manager
        self.data_server_url = data_server_url
        self.worker_service_id = worker_service_id
        self.log = logger or logging.getLogger("bioengine.builder")
        lap = local_artifact_path or os.environ.get("BIOENGINE_LOCAL_ARTIFACT_PATH")
        self.local_artifact_path = Path(lap) if lap else None

    # ------------------------------------------------------------------ sources
    def _local_dir(self, artifact_id: str) -> Path | None:
        p = Path(artifact_id)
        if p.is_dir() and (p / "manifest.yaml").exists():
            return p
        if self.local_artifact_path is not None:
            alias = artifact_id.split("/")[-1]
            for cand in (self.local_artifact_path / alias, self.local_artifact_path / alias.replace("-", "_")):
                if (cand / "manifest.yaml").exists():
                    return cand
            for cand in sorted(self.local_artifact_path.glob("*/manifest.yaml")):  # match by manifest id
                try:
                    if (yaml.safe_load(cand.read_text()) or {}).get("id") == alias:
                        return cand.parent
                except Exception:
                    continue
        return None

    async def load_manifest(self, artifact_id: str, version: str | None = None) -> tuple[dict, str | None]:
        d = self._local_dir(artifact_id)
        if d is not None:
            m = yaml.safe_load((d / "manifest.yaml").read_text())
            validate_manifest(m)
            return m, version or m.get("version")
        if self.artifact_manager is None:
            raise FileNotFoundError(f"artifact '{artifact_id}' not found locally and no artifact manager configured")
        art = await self.artifact_manager.read(artifact_id, version=version)
        m = art.get("manifest")
        if m is None:
            raise ValueError(f"Manifest not found in artifact {artifact_id}.")
        validate_manifest(m)
        if version is None:
            vs = art.get("versions") or []
            version = vs[-1]["version"] if vs else None
        return m, version

    async def load_file(self, artifact_id: str, version: str | None, file_path: str) -> str:
        d = self._local_dir(artifact_id)
        if d is not None:
            return (d / file_path).read_text()
        url = await self.artifact_manager.get_file(artifact_id=artifact_id, version=version, file_path=file_path)
        async with httpx.AsyncClient(timeout=30) as c:
            r = await c.get(url)
            r.raise_for_status()
            return r.text

    # ------------------------------------------------------------------ code loading
    async def load_deployment(self, application_id: str, artifact_id: str, version: str | None, import_path: str,
                              env_vars: dict) -> Deployment:
        file_name, class_name = import_path.split(":")
        py = file_name if file_name.endswith(".py") else f"{file_name}.py"
        code = await self.load_file(artifact_id, version, py)
        from ..compat import install

        install()
        site = self.apps_workdir / application_id / "site-packages"
        if site.is_dir() and str(site) not in sys.path:  # requirements installed by an earlier deploy
            from .requirements import _APP_PATHS

            _APP_PATHS.add(str(site))
            sys.path.append(str(site))  # appended: an app's wheels never shadow the worker's own modules
        mod_name = f"bioengine_app_{application_id.replace('-', '_')}_{Path(py).stem}"
        ns: dict[str, Any] = {"__name__": mod_name, "__file__": f"<{artifact_id}/{py}>", "__builtins__": __builtins__}
        ns.update({k: v for k, v in env_vars.items()})
        try:
            exec(compile(code, f"<{artifact_id}/{py}>", "exec"), ns)  # noqa: S102 - app code is the artifact's content
        except ModuleNotFoundError as e:
            raise ModuleNotFoundError(
                f"'{py}' of artifact '{artifact_id}' imports '{e.name}' at module level, which is not installed on "
                f"this worker. Import it inside the deployment's methods and list it in "
                f"ray_actor_options.runtime_env.pip (installed from BIOENGINE_WHEELHOUSE at deploy time).",
                name=e.name) from e
        obj = ns.get(class_name)
        if obj is None:
            raise ValueError(f"Class '{class_name}' not found in '{py}' of artifact '{artifact_id}'")
        if not isinstance(obj, Deployment):
            obj = serve_deployment(obj)
        return obj

    # ------------------------------------------------------------------ options & wrapping
    def _split_env(self, env: dict) -> tuple[dict, dict]:
        public, secret = {}, {}
        for k, v in (env or {}).items():
            if k.startswith("_"):
                secret[k[1:]] = str(v)
            else:
                public[k] = str(v)
        return public, secret

    def _actor_options(self, application_id: str, artifact_id: str, dep: Deployment, env_public: dict,
                       env_secret: dict, disable_gpu: bool, hypha_token: str | None) -> dict:
        opts = copy.deepcopy(dep.ray_actor_options or {})
        if disable_gpu:
            opts["num_gpus"] = 0
        opts.setdefault("num_cpus", 1)
        rt = dict(opts.get("runtime_env") or {})
        workdir = self.apps_workdir / application_id
        envv = dict(rt.get("env_vars") or {})
        # the URL the worker itself connected with (a local:// hub has no WebSocket endpoint behind
        # its public HTTP base); for a real Hypha server both are the same
        server_url = getattr(self.server, "server_url", None) or \
            getattr(getattr(self.server, "config", None), "public_base_url", None) or ""
        workspace = getattr(getattr(self.server, "config", None), "workspace", None) or ""
        envv.update({
            "HOME": str(workdir), "TMPDIR": str(workdir / "tmp"), "TEMP": str(workdir / "tmp"), "TMP": str(workdir / "tmp"),
            "HYPHA_SERVER_URL": str(server_url), "HYPHA_WORKSPACE": str(workspace), "HYPHA_ARTIFACT_ID": artifact_id,
            "BIOENGINE_WORKER_SERVICE_ID": str(self.worker_service_id or ""),
        })
        envv.update(env_public)
        for k in env_secret:
            envv[k] = SECRET_MASK
        if hypha_token:
            envv["HYPHA_TOKEN"] = SECRET_MASK
        pip = [str(r) for r in (rt.get("pip") or [])]
        if pip:
            # pinned like the reference (worker's httpx/pydantic added, >=/~= -> ==); resolved and, if
            # needed, installed from the wheelhouse into the app's site-packages before deployment
            rt["pip"] = update_requirements(pip)
            site = str(workdir / "site-packages")
            envv["PYTHONPATH"] = site + (os.pathsep + envv["PYTHONPATH"] if envv.get("PYTHONPATH") else "")
        rt["env_vars"] = envv
        opts["runtime_env"] = rt
        return opts

    def _wrap_class(self, user_cls, application_id: str, secret_env: dict, debug: bool):
        """Lifecycle wrapper (a subclass, so the user's class object stays untouched)."""
        data_server_url = self.data_server_url
        workdir = self.apps_workdir / application_id
        user_async_init = getattr(user_cls, "async_init", None)
        user_test = getattr(user_cls, "test_deployment", None)
        user_health = getattr(user_cls, "check_health", None)

        class Wrapped(user_cls):  # type: ignore[misc, valid-type]
            @wraps(user_cls.__init__)
            def __init__(self, *args, **kwargs):
                log = logging.getLogger("ray.serve")
                log.setLevel(logging.DEBUG if debug else logging.INFO)
                os.environ["HOME"] = str(workdir)
                workdir.mkdir(parents=True, exist_ok=True)
                (workdir / "tmp").mkdir(exist_ok=True)
                if os.environ.get("BE_REPLICA_SOCK"):  # own process: adopt the app working directory
                    os.chdir(workdir)
                for k, v in secret_env.items():
                    os.environ[k] = v
                self._bioengine_replica_initialized = False
                self._bioengine_replica_test_failed = False
                self._bioengine_test_error = None
                self._bioengine_test_task = None
                self._bioengine_health_lock = None
                from ..datasets.client import BioEngineDatasets

                self.bioengine_datasets = BioEngineDatasets(data_server_url=data_server_url or None,
                                                            hypha_token=os.environ.get("HYPHA_TOKEN"), logger=log)
                user_cls.__init__(self, *args, **kwargs)

            async def async_init(self):
                if self._bioengine_replica_initialized:
                    return
                t0 = time.time()
                if user_async_init is not None:
                    r = user_async_init(self)
                    if inspect.isawaitable(r):
                        await r
                self._bioengine_replica_initialized = True
                logging.getLogger("ray.serve").info(f"async_init completed in {time.time() - t0:.2f}s")

            async def test_deployment(self):
                try:
                    if user_test is not None:
                        r = user_test(self)
                        if inspect.isawaitable(r):
                            r = await r
                        if r is False:
                            raise RuntimeError("test_deployment returned False")
                    logging.getLogger("ray.serve").info("test_deployment passed")
                except BaseException as e:  # noqa: BLE001
                    self._bioengine_replica_test_failed = True
                    self._bioengine_test_error = f"{type(e).__name__}: {e}"
                    logging.getLogger("ray.serve").error(f"test_deployment failed: {e}")
                    raise

            async def check_health(self):
                if self._bioengine_health_lock is None:
                    self._bioengine_health_lock = asyncio.Lock()
                async with self._bioengine_health_lock:
                    if not self._bioengine_replica_initialized:
                        await self.async_init()
                    if self._bioengine_test_task is None:
                        self._bioengine_test_task = asyncio.ensure_future(self.test_deployment())
                        self._bioengine_test_task.add_done_callback(lambda t: t.exception())
                    if self._bioengine_replica_test_failed:
                        raise RuntimeError(f"Deployment test failed - deployment is unhealthy: {self._bioengine_test_error}")
                    if self.bioengine_datasets.data_server_url:
                        try:
                            await self.bioengine_datasets.ping_data_server()
                        except Exception as e:  # noqa: BLE001
                            logging.getLogger("ray.serve").warning(f"datasets server unreachable: {e}")
                    if user_health is not None:
                        r = user_health(self)
                        if inspect.isawaitable(r):
                            await r

        Wrapped.__name__ = user_cls.__name__
        Wrapped.__qualname__ = user_cls.__qualname__
        Wrapped.__module__ = user_cls.__module__
        Wrapped.__doc__ = user_cls.__doc__
        return Wrapped

    @staticmethod
    def init_params(cls) -> dict[str, dict]:
        sig = inspect.signature(cls.__init__)
        out = {}
        for name, p in list(sig.parameters.items())[1:]:
            if p.kind in (p.VAR_POSITIONAL, p.VAR_KEYWORD):
                continue
            out[name] = {"required": p.default is inspect.Parameter.empty,
                         "annotation": getattr(p.annotation, "__name__", str(p.annotation))}
        return out

    @staticmethod
    def validate_kwargs(cls, kwargs: dict, handle_params: set[str]):
        params = AppBuilder.init_params(cls)
        accepts_var = any(p.kind == p.VAR_KEYWORD for p in inspect.signature(cls.__init__).parameters.values())
        for k in kwargs:
            if k not in params and not accepts_var:
                raise ValueError(f"Unknown init parameter '{k}' for deployment '{cls.__name__}'. "
                                 f"Valid parameters: {sorted(params)}")
        missing = [k for k, v in params.items() if v["required"] and k not in kwargs and k not in handle_params]
        if missing:
            raise ValueError(f"Missing required init parameter(s) {missing} for deployment '{cls.__name__}'")

    @staticmethod
    def method_schemas(cls) -> list[dict]:
        out = []
        for name in dir(cls):
            if name.startswith("_"):
                continue
            fn = getattr(cls, name, None)
            sch = getattr(fn, "__schema__", None)
            if callable(fn) and sch:
                try:
                    takes_ctx = "context" in inspect.signature(fn).parameters
                except (TypeError, ValueError):
                    takes_ctx = False
                out.append(dict(sch, name=name, _accepts_context=takes_ctx))
        return out

    @staticmethod
    def resolve_authorized_users(authorized_users, manifest: dict, deploying_user: tuple | None,
                                 admin_users: list[str] | None) -> dict[str, list[str]]:
        src = authorized_users if authorized_users is not None else manifest.get("authorized_users", ["*"])
        rules = {k: list(v) for k, v in src.items()} if isinstance(src, dict) else {"*": list(src)}
        dep = [v for v in (deploying_user or ()) if v]
        extra = dep + list(admin_users or [])
        for key, rule in rules.items():
            if "*" not in rule:
                rule.extend(u for u in extra if u not in rule)
            rules[key] = list(dict.fromkeys(rule))
        if "*" not in rules:
            rules["*"] = list(dict.fromkeys(extra))
        return rules

    # ------------------------------------------------------------------ build
    async def build(self, application_id: str, artifact_id: str, version: str | None = None,
                    application_kwargs: dict | None = None, application_env_vars: dict | None = None,
                    hypha_token: str | None = None, disable_gpu: bool = False, max_ongoing_requests: int = 10,
                    debug: bool = False, started_at: float | None = None, last_updated_at: float | None = None,
                    last_updated_by: str | None = None, auto_redeploy: bool = False, ice_servers=None,
                    authorized_users=None, deploying_user: tuple | None = None,
                    admin_users: list[str] | None = None) -> BuiltApp:
        application_kwargs = dict(application_kwargs or {})
        application_env_vars = dict(application_env_vars or {})
        manifest, version = await self.load_manifest(artifact_id, version)
        paths = manifest["deployments"]
        deps: list[tuple[str, Deployment]] = []
        for ip in paths:
            cls_name = ip.split(":")[1]
            env = dict(application_env_vars.get(cls_name) or {})
            if hypha_token:
                env.setdefault("_HYPHA_TOKEN", hypha_token)
            pub, sec = self._split_env(env)
            dep = await self.load_deployment(application_id, artifact_id, version, ip, pub)
            opts = self._actor_options(application_id, artifact_id, dep, pub, sec, disable_gpu, hypha_token)
            wrapped = self._wrap_class(dep.func_or_class, application_id, sec, debug)
            d2 = Deployment(wrapped, copy.deepcopy(dep.config)).options(ray_actor_options=opts)
            deps.append((ip, d2))
        entry_ip, entry = deps[0]
        user_entry_cls = entry.func_or_class.__mro__[1]
        schemas = self.method_schemas(user_entry_cls)
        if not schemas:
            raise ValueError(f"Entry deployment '{user_entry_cls.__name__}' exposes no @schema_method methods")
        # composition: bind extra deployments to entry params named after their file stem
        handles = {}
        for ip, d in deps[1:]:
            stem = Path(ip.split(":")[0]).stem
            user_cls = d.func_or_class.__mro__[1]
            kw = dict(application_kwargs.get(user_cls.__name__) or {})
            self.validate_kwargs(user_cls, kw, set())
            handles[stem] = d.bind(**kw)
        entry_params = self.init_params(user_entry_cls)
        for stem in handles:
            if stem not in entry_params:
                raise ValueError(f"Entry deployment '{user_entry_cls.__name__}' has no __init__ parameter '{stem}' "
                                 f"for the composed deployment file '{stem}.py'")
        ekw = dict(application_kwargs.get(user_entry_cls.__name__) or {})
        self.validate_kwargs(user_entry_cls, ekw, set(handles))
        root = entry.bind(**ekw, **handles)
        pip_reqs: list[str] = []
        for _, d in deps:
            for r in ((d.ray_actor_options or {}).get("runtime_env") or {}).get("pip") or []:
                if r not in pip_reqs:
                    pip_reqs.append(r)
        resources = {"num_cpus": 0.0, "num_gpus": 0.0, "memory": 0.0}
        for _, d in deps:
            lo, _, init = d.config.min_max_replicas()
            n = max(1, init)
            resources["num_cpus"] += d.config.num_cpus() * n
            resources["num_gpus"] += d.config.num_gpus() * n
            resources["memory"] += d.config.memory() * n
        users = self.resolve_authorized_users(authorized_users, manifest, deploying_user, admin_users)
        now = time.time()
        masked_env = {cls: {(k[1:] if k.startswith("_") else k): (SECRET_MASK if k.startswith("_") else v)
                            for k, v in sorted(env.items())} for cls, env in application_env_vars.items()}
        meta = {
            "display_name": manifest["name"], "description": manifest["description"], "artifact_id": artifact_id,
            "version": version, "application_kwargs": application_kwargs, "application_env_vars": masked_env,
            "disable_gpu": disable_gpu, "gpu_enabled": (not disable_gpu) and resources["num_gpus"] > 0,
            "max_ongoing_requests": max_ongoing_requests, "application_resources": resources,
            "authorized_users": users, "available_methods": [s["name"] for s in schemas],
            "started_at": started_at or now, "last_updated_at": last_updated_at or now,
            "last_updated_by": last_updated_by, "auto_redeploy": auto_redeploy, "debug": debug,
            "frontend_entry": manifest.get("frontend_entry"), "ice_servers": ice_servers,
            "deployments": [ip for ip in paths], "hypha_token_set": bool(hypha_token),
            "pip_requirements": pip_reqs,
        }
        self.log.info(f"Built application '{application_id}' from '{artifact_id}' (version {version}); "
                      f"methods: {meta['available_methods']}")
        return BuiltApp(application_id, root, manifest, meta, schemas)
