"""Serve controller: application graph deployment, request routing, autoscaling, health checks.

Native replacement of the Ray Serve controller + router + proxy (reference uses
``serve.run/delete/status``: ``bioengine/apps/manager.py:355-455,502-558``; autoscaling and health
semantics from deployment options, e.g. ``bioengine/apps/proxy_deployment.py:35-47``,
``apps/model-runner/runtime_deployment.py:40-55``).

Routing: each deployment keeps its replicas and an admission queue.  A request goes to the RUNNING
replica with the fewest in-flight requests below ``max_ongoing_requests``; when all are saturated
it waits in FIFO order, and is rejected with :class:`BackPressureError` beyond
``max_queued_requests`` (-1 = unbounded).  Autoscaling follows Ray's policy: desired replicas =
ceil(total in-flight / target_ongoing_requests), clamped to [min, max], applied after
``upscale_delay_s`` / ``downscale_delay_s`` of persistence.  Health: every
``health_check_period_s`` the replica's ``check_health`` runs with ``health_check_timeout_s``; a
failing replica is replaced (restart with back-off), and the deployment reports UNHEALTHY meanwhile.

GPU replicas are :class:`~.replica.ProcessReplica` pinned to GPUs reserved from the node's
:class:`ResourcePool`; CPU-only deployments run as in-process :class:`~.replica.LocalReplica`.
"""
from __future__ import annotations

import asyncio
import collections
import math
import os
import time
from dataclasses import dataclass, field

from .api import Application, DeploymentConfig
from .handle import DeploymentHandle
from ..runtime import faults
from .replica import DEAD, RUNNING, STARTING, STOPPING, LocalReplica, ProcessReplica


class BackPressureError(RuntimeError):
    pass


class DeploymentUnavailableError(RuntimeError):
    pass


# ====================================================================== resources


class ResourcePool:
    """Logical CPU / GPU / memory accounting for one node (Ray's logical resources)."""

    def __init__(self, num_cpus: float | None = None, gpu_ids: list[int] | None = None, memory: float | None = None):
        self.total_cpu = float(num_cpus if num_cpus is not None else (os.cpu_count() or 1))
        self.gpu_ids = list(gpu_ids if gpu_ids is not None else [])
        self.total_memory = float(memory if memory is not None else _total_memory())
        self.used_cpu = 0.0
        self.used_memory = 0.0
        self.gpu_used: dict[int, float] = {g: 0.0 for g in self.gpu_ids}
        self.custom: dict[str, float] = {}

    @property
    def total_gpu(self) -> float:
        return float(len(self.gpu_ids))

    @property
    def used_gpu(self) -> float:
        return float(sum(self.gpu_used.values()))

    def can_fit(self, cpus: float, gpus: float, memory: float) -> bool:
        if cpus > self.total_cpu - self.used_cpu + 1e-9:
            return False
        if memory and memory > self.total_memory - self.used_memory + 1:
            return False
        return self._pick_gpus(gpus) is not None

    def _pick_gpus(self, gpus: float):
        if gpus <= 0:
            return []
        if gpus < 1:
            for g in self.gpu_ids:
                if self.gpu_used[g] + gpus <= 1.0 + 1e-9:
                    return [g]
            return None
        need = int(math.ceil(gpus))
        free = [g for g in self.gpu_ids if self.gpu_used[g] == 0.0]
        return free[:need] if len(free) >= need else None

    def reserve(self, cpus: float, gpus: float, memory: float) -> list[int]:
        ids = self._pick_gpus(gpus)
        if ids is None or cpus > self.total_cpu - self.used_cpu + 1e-9:
            raise ResourceWarning(f"insufficient resources for num_cpus={cpus}, num_gpus={gpus} "
                                  f"(free cpu={self.total_cpu - self.used_cpu:g}, free gpu="
                                  f"{sum(1 for g in self.gpu_ids if self.gpu_used[g] == 0)})")
        self.used_cpu += cpus
        self.used_memory += memory or 0.0
        share = gpus if gpus < 1 else 1.0
        for g in ids:
            self.gpu_used[g] += share
        return ids

    def release(self, cpus: float, gpus: float, memory: float, ids: list[int]):
        self.used_cpu = max(0.0, self.used_cpu - cpus)
        self.used_memory = max(0.0, self.used_memory - (memory or 0.0))
        share = gpus if gpus < 1 else 1.0
        for g in ids:
            self.gpu_used[g] = max(0.0, self.gpu_used[g] - share)


def _total_memory() -> float:
    try:
        import psutil

        return float(psutil.virtual_memory().total)
    except Exception:
        return 16 * 1024 ** 3


# ====================================================================== deployments


@dataclass
class _Waiter:
    fut: asyncio.Future
    t: float = field(default_factory=time.time)


class DeploymentState:
    def __init__(self, ctrl: "ServeController", app: str, cfg: DeploymentConfig, cls, args, kwargs):
        self.ctrl = ctrl
        self.app = app
        self.cfg = cfg
        self.name = cfg.name
        self.cls = cls
        self.args = args
        self.kwargs = kwargs
        self.replicas: list = []
        self.status = "UPDATING"
        self.message = ""
        self.waiters: collections.deque[_Waiter] = collections.deque()
        lo, hi, init = cfg.min_max_replicas()
        self.min_r, self.max_r, self.target = lo, hi, init
        self._scale_since: tuple[int, float] | None = None
        self.restarts = 0
        self.history: list[dict] = []  # dead replicas (for logs of previous replicas)
        self.requests_total = 0
        self.deadline_exceeded = 0
        self.latency = collections.deque(maxlen=2048)
        self._stopping = False

    # ---------------------------------------------------------------- replicas
    def _use_process(self) -> bool:
        mode = os.environ.get("BIOENGINE_REPLICA_MODE", "auto")
        if mode == "process":
            return True
        if mode == "local":
            return False
        if self.cfg.num_gpus() > 0:
            return True
        pip = (self.cfg.ray_actor_options.get("runtime_env") or {}).get("pip") or []
        if isinstance(pip, dict):
            pip = pip.get("packages") or []
        if pip:
            from ..apps.requirements import shadowed

            if shadowed([str(r) for r in pip]):  # pinned versions differ from the worker's: isolate
                return True
        return False

    async def add_replica(self):
        cpus, gpus, mem = self.cfg.num_cpus(), self.cfg.num_gpus(), self.cfg.memory()
        node, ids = await self.ctrl.place(cpus, gpus, mem, self)
        env = dict((self.cfg.ray_actor_options.get("runtime_env") or {}).get("env_vars") or {})
        cls = self.ctrl._replica_cls(self)
        if node is not None:
            from .remote import RemoteReplica

            r = RemoteReplica(node, self.app, self.name, cls, self.args, self.kwargs, ids, env)
        elif self._use_process():
            r = ProcessReplica(self.app, self.name, cls, self.args, self.kwargs, ids, env, log_dir=self.ctrl.log_dir)
        else:
            r = LocalReplica(self.app, self.name, cls, self.args, self.kwargs, ids, env)
        r._res = (cpus, gpus, mem, ids)
        r._pool = node.pool if node is not None else self.ctrl.resources
        self.replicas.append(r)
        try:
            await r.start()
            # initial readiness probe: runs the app's lazy async_init before traffic is admitted
            from .replica import STARTING as _ST

            r.state = _ST
            await asyncio.wait_for(r.check_health(), timeout=max(120.0, 10 * self.cfg.health_check_timeout_s))
            r.state = RUNNING
        except BaseException as e:
            r.error = r.error or f"{type(e).__name__}: {e}"
            try:
                await r.stop(1.0)
            except Exception:
                pass
            self._retire(r)
            raise
        self._wake()
        return r

    def _retire(self, r):
        if r in self.replicas:
            self.replicas.remove(r)
        cpus, gpus, mem, ids = r._res
        getattr(r, "_pool", self.ctrl.resources).release(cpus, gpus, mem, ids)
        self.history.append({"replica_id": r.tag, "logs": r.logs(200), "error": r.error, "stopped_at": time.time()})
        self.history = self.history[-10:]

    async def remove_replica(self, r):
        r.state = STOPPING
        try:
            await r.stop(self.cfg.graceful_shutdown_timeout_s)
        finally:
            self._retire(r)

    async def start(self):
        errs = []
        for _ in range(self.target):
            for attempt in range(3):
                try:
                    await self.add_replica()
                    break
                except ResourceWarning as e:
                    errs.append(str(e))
                    break
                except BaseException as e:  # noqa: BLE001
                    errs.append(f"{type(e).__name__}: {e}")
                    if attempt == 2:
                        break
        if not self.running():
            self.status = "DEPLOY_FAILED"
            self.message = "; ".join(errs[-3:]) or "no replica could be started"
            raise RuntimeError(f"Deployment '{self.name}' failed to start: {self.message}")
        self.status = "HEALTHY" if len(self.running()) >= self.target else "UPDATING"
        self.message = "; ".join(errs[-1:]) if errs else ""

    def running(self):
        return [r for r in self.replicas if r.state == RUNNING]

    async def stop(self):
        self._stopping = True
        for w in self.waiters:
            if not w.fut.done():
                w.fut.set_exception(DeploymentUnavailableError(f"deployment {self.name} is shutting down"))
        await asyncio.gather(*[self.remove_replica(r) for r in list(self.replicas)], return_exceptions=True)

    # ---------------------------------------------------------------- routing
    def _pick(self):
        best = None
        for r in self.replicas:
            if r.state != RUNNING or r.ongoing >= self.cfg.max_ongoing_requests:
                continue
            if best is None or r.ongoing < best.ongoing:
                best = r
        return best

    def _wake(self):
        while self.waiters:
            r = self._pick()
            if r is None:
                return
            w = self.waiters.popleft()
            if not w.fut.done():
                r.ongoing += 1  # reserve the slot for the woken request
                w.fut.set_result(r)

    async def acquire(self):
        if self._stopping:
            raise DeploymentUnavailableError(f"deployment {self.name} is shutting down")
        r = self._pick()
        if r is not None and not self.waiters:
            r.ongoing += 1
            return r
        if self.cfg.max_queued_requests >= 0 and len(self.waiters) >= self.cfg.max_queued_requests:
            raise BackPressureError(f"Request dropped: deployment '{self.name}' queue is full "
                                    f"({self.cfg.max_queued_requests} queued)")
        if not self.running() and not any(r.state == STARTING for r in self.replicas):
            raise DeploymentUnavailableError(f"deployment '{self.name}' has no running replicas")
        w = _Waiter(asyncio.get_running_loop().create_future())
        self.waiters.append(w)
        try:
            return await w.fut
        except asyncio.CancelledError:  # deadline / caller gave up while queued
            try:
                self.waiters.remove(w)
            except ValueError:
                pass
            if w.fut.done() and not w.fut.cancelled():  # a slot was reserved for us: hand it on
                w.fut.result().ongoing -= 1
                self._wake()
            raise

    def request_timeout(self) -> float | None:
        t = self.cfg.request_timeout_s
        if t is None and os.environ.get("BIOENGINE_REQUEST_TIMEOUT_S"):
            t = float(os.environ["BIOENGINE_REQUEST_TIMEOUT_S"])
        return t if t and t > 0 else None

    async def call(self, method, args, kwargs, model_id=""):
        """Route one request: admission (queue for a free replica slot), then the replica call,
        both bounded by the request deadline (the caller's, tightened by ``request_timeout_s``)."""
        with faults.deadline_scope(self.request_timeout()) as deadline:
            if deadline is None:
                return await self._call(method, args, kwargs, model_id)
            left = deadline - time.time()
            try:
                if left <= 0:
                    raise asyncio.TimeoutError
                return await asyncio.wait_for(self._call(method, args, kwargs, model_id), left)
            except asyncio.TimeoutError:
                self.deadline_exceeded += 1
                raise faults.DeadlineExceeded(
                    f"request {self.name}.{method} exceeded its deadline") from None

    async def _call(self, method, args, kwargs, model_id=""):
        from ..profiling import trace

        with trace.span("router.admission", cat="router", deployment=self.name):
            r = await self.acquire()
        t0 = time.perf_counter()
        try:
            r.ongoing -= 1  # replica.call() tracks its own in-flight count
            with trace.span(f"replica.{method}", cat="replica", deployment=self.name, replica=r.tag):
                return await r.call(method, args, kwargs, model_id)
        finally:
            self.requests_total += 1
            self.latency.append(time.perf_counter() - t0)
            self._wake()

    @property
    def ongoing(self) -> int:
        return sum(r.ongoing for r in self.replicas) + len(self.waiters)

    # ---------------------------------------------------------------- control loops
    async def health_tick(self):
        for r in list(self.running()):
            try:
                await asyncio.wait_for(r.check_health(), timeout=self.cfg.health_check_timeout_s)
                r.health_failures = 0
            except BaseException as e:  # noqa: BLE001
                r.health_failures += 1
                r.error = f"health check failed: {type(e).__name__}: {e}"
                self.status = "UNHEALTHY"
                self.message = r.error
                if r.health_failures >= 1:
                    await self._replace(r)
        if self.status == "UNHEALTHY" and all(rr.health_failures == 0 for rr in self.running()) and self.running():
            self.status = "HEALTHY"
            self.message = ""

    async def _replace(self, r):
        self.restarts += 1
        try:
            await self.remove_replica(r)
        except Exception:
            pass
        await asyncio.sleep(min(30.0, 0.5 * 2 ** min(self.restarts, 6)))
        try:
            await self.add_replica()
        except BaseException as e:  # noqa: BLE001
            self.status = "UNHEALTHY"
            self.message = f"replica restart failed: {type(e).__name__}: {e}"

    async def autoscale_tick(self):
        ac = self.cfg.autoscaling_config
        if not ac:
            return
        target_per = float(ac.get("target_ongoing_requests", ac.get("target_num_ongoing_requests_per_replica", 2)) or 2)
        desired = math.ceil(self.ongoing / target_per) if self.ongoing > 0 else self.min_r
        desired = max(self.min_r, min(self.max_r, desired))
        cur = len([r for r in self.replicas if r.state in (RUNNING, STARTING)])
        if desired == cur:
            self._scale_since = None
            return
        now = time.time()
        if self._scale_since is None or self._scale_since[0] != desired:
            self._scale_since = (desired, now)
            return
        delay = float(ac.get("upscale_delay_s", 30.0) if desired > cur else ac.get("downscale_delay_s", 600.0))
        if now - self._scale_since[1] < delay:
            return
        self._scale_since = None
        if desired > cur:
            self.status = "UPSCALING"
            for _ in range(desired - cur):
                if not self.ctrl.can_place(self.cfg.num_cpus(), self.cfg.num_gpus(), self.cfg.memory()):
                    self.ctrl.pending_demands.append({"deployment": self.name, "app": self.app,
                                                      "num_cpus": self.cfg.num_cpus(), "num_gpus": self.cfg.num_gpus()})
                    break
                try:
                    await self.add_replica()
                except BaseException:
                    break
        else:
            self.status = "DOWNSCALING"
            idle = sorted(self.running(), key=lambda r: r.ongoing)
            for r in idle[: cur - desired]:
                await self.remove_replica(r)
        self.target = desired
        self.status = "HEALTHY"

    # ---------------------------------------------------------------- status
    def status_dict(self) -> dict:
        counts = collections.Counter(r.state for r in self.replicas)
        return {"status": self.status, "message": self.message, "replica_states": dict(counts),
                "replicas": [r.info() for r in self.replicas], "target_replicas": self.target,
                "ongoing_requests": self.ongoing, "requests_total": self.requests_total, "deadline_exceeded": self.deadline_exceeded,
                "latency_ms": _pcts(self.latency)}


def _pcts(d) -> dict:
    if not d:
        return {}
    s = sorted(d)
    return {p: round(1e3 * s[min(len(s) - 1, int(q * (len(s) - 1)))], 3) for p, q in (("p50", .5), ("p95", .95), ("p99", .99))}


@dataclass
class AppState:
    name: str
    route_prefix: str | None
    ingress: str
    deployments: dict[str, DeploymentState]
    status: str = "DEPLOYING"
    message: str = ""
    deployed_at: float = field(default_factory=time.time)


# ====================================================================== controller


class ServeController:
    def __init__(self, resources: ResourcePool | None = None, log_dir: str | None = None, tick_s: float = 1.0):
        try:
            self.loop = asyncio.get_running_loop()
        except RuntimeError:
            self.loop = None  # bound on first deploy
        self.resources = resources or ResourcePool(gpu_ids=_detect_gpus())
        self.apps: dict[str, AppState] = {}
        self.log_dir = log_dir
        self.tick_s = tick_s
        self.pending_demands: list = []
        self.remote_nodes: dict = {}          # node_id -> serve.remote.RemoteNode
        self.wait_for_nodes_s = 0.0           # > 0 (SLURM mode): wait this long for a node to join
        self._task = None
        self._health_last: dict = {}
        self.replica_class_wrappers = []  # callables (DeploymentState, cls) -> cls
        from .gang import GangManager

        self.gangs = GangManager(self.resources, log_dir)  # multi-rank jobs (serve/gang.py)

    def can_place(self, cpus: float, gpus: float, mem: float) -> bool:
        return self.resources.can_fit(cpus, gpus, mem) or any(n.pool.can_fit(cpus, gpus, mem)
                                                               for n in self.remote_nodes.values())

    async def place(self, cpus: float, gpus: float, mem: float, ds=None):
        """Reserve resources for one replica: the head first, then remote nodes (least loaded).
        Returns (RemoteNode | None, gpu_ids).  In SLURM mode an unplaceable replica is recorded as
        pending demand (the autoscaler submits a worker job) and waited for."""
        deadline = time.time() + self.wait_for_nodes_s
        demand = None
        while True:
            if self.resources.can_fit(cpus, gpus, mem):
                if demand in self.pending_demands:
                    self.pending_demands.remove(demand)
                return None, self.resources.reserve(cpus, gpus, mem)
            fits = [n for n in self.remote_nodes.values() if n.pool.can_fit(cpus, gpus, mem)]
            if fits:
                n = min(fits, key=lambda n: (n.pool.used_gpu, n.pool.used_cpu))
                if demand in self.pending_demands:
                    self.pending_demands.remove(demand)
                return n, n.pool.reserve(cpus, gpus, mem)
            if time.time() >= deadline:
                if demand in self.pending_demands:
                    self.pending_demands.remove(demand)
                return None, self.resources.reserve(cpus, gpus, mem)  # raises with the usual message
            if demand is None:
                demand = {"deployment": getattr(ds, "name", "?"), "app": getattr(ds, "app", "?"), "num_cpus": cpus,
                          "num_gpus": gpus, "since": time.time()}
                self.pending_demands.append(demand)
            await asyncio.sleep(0.5)

    def add_remote_node(self, node) -> None:
        self.remote_nodes[node.node_id] = node

    def remove_remote_node(self, node_id: str) -> None:
        self.remote_nodes.pop(node_id, None)

    def _replica_cls(self, ds: DeploymentState):
        cls = ds.cls
        for w in self.replica_class_wrappers:
            cls = w(ds, cls)
        return cls

    def _ensure_loop(self):
        self.loop = asyncio.get_running_loop()
        if self._task is None or self._task.done():
            self._task = asyncio.get_running_loop().create_task(self._control_loop())

    async def _control_loop(self):
        while True:
            await asyncio.sleep(self.tick_s)
            now = time.time()
            for app in list(self.apps.values()):
                for ds in list(app.deployments.values()):
                    try:
                        await ds.autoscale_tick()
                        key = (app.name, ds.name)
                        if now - self._health_last.get(key, 0) >= ds.cfg.health_check_period_s:
                            self._health_last[key] = now
                            asyncio.ensure_future(ds.health_tick())
                    except Exception:
                        pass
                self._refresh_app_status(app)

    def _refresh_app_status(self, app: AppState):
        if app.status in ("DELETING", "DEPLOY_FAILED", "DEPLOYING"):
            return
        sts = [d.status for d in app.deployments.values()]
        if any(s == "UNHEALTHY" for s in sts):
            app.status = "UNHEALTHY"
            app.message = "; ".join(d.message for d in app.deployments.values() if d.message)
        else:
            app.status = "RUNNING"
            app.message = ""

    async def deploy_application(self, root: Application, name: str = "default", route_prefix: str | None = None):
        self._ensure_loop()
        if name in self.apps:
            await self.delete_application(name)
        order: list[Application] = []
        seen = {}

        def visit(node: Application):
            if id(node) in seen:
                return
            for ch in node.children():
                visit(ch)
            seen[id(node)] = node.deployment.name
            order.append(node)

        visit(root)
        app = AppState(name, route_prefix, root.deployment.name, {})
        self.apps[name] = app

        def sub(v):
            if isinstance(v, Application):
                return DeploymentHandle(name, v.deployment.name)
            return v

        try:
            for node in order:
                cfg = node.deployment.config
                args = [sub(a) for a in node.args]
                kwargs = {k: sub(v) for k, v in node.kwargs.items()}
                ds = DeploymentState(self, name, cfg, node.deployment.func_or_class, args, kwargs)
                app.deployments[cfg.name] = ds
            await asyncio.gather(*[ds.start() for ds in app.deployments.values()])
        except BaseException as e:
            app.status = "DEPLOY_FAILED"
            app.message = str(e)
            for ds in app.deployments.values():
                if ds.status != "DEPLOY_FAILED":
                    await ds.stop()
            raise
        app.status = "RUNNING"
        return DeploymentHandle(name, app.ingress)

    async def delete_application(self, name: str):
        app = self.apps.get(name)
        if app is None:
            return
        app.status = "DELETING"
        await asyncio.gather(*[ds.stop() for ds in app.deployments.values()], return_exceptions=True)
        self.apps.pop(name, None)

    def get_app_handle(self, name: str) -> DeploymentHandle:
        app = self.apps[name]
        return DeploymentHandle(name, app.ingress)

    async def call(self, app: str, dep: str, method: str, args, kwargs, model_id: str = ""):
        if app == "__bioengine__":  # runtime services reachable from replicas over the handle channel
            if dep == "gang" and method == "run":
                return await self.gangs.run(*args, **kwargs)
            if dep == "gang" and method == "status":
                return self.gangs.status()
            raise DeploymentUnavailableError(f"unknown runtime service {dep}.{method}")
        a = self.apps.get(app)
        if a is None:
            raise DeploymentUnavailableError(f"application '{app}' is not running")
        ds = a.deployments.get(dep)
        if ds is None:
            raise DeploymentUnavailableError(f"deployment '{dep}' not found in application '{app}'")
        return await ds.call(method, args, kwargs, model_id)

    def serve_status(self):
        return ServeStatus({n: AppStatusOverview(a) for n, a in self.apps.items()})

    async def shutdown(self):
        for n in list(self.apps):
            await self.delete_application(n)
        if self._task is not None:
            self._task.cancel()


# ---------------------------------------------------------------------- status objects (Ray-like)


class DeploymentStatusOverview:
    def __init__(self, ds: DeploymentState):
        self.name = ds.name
        self.status = ds.status
        self.message = ds.message
        self.status_trigger = "CONFIG_UPDATE_STARTED" if ds.status == "UPDATING" else "CONFIG_UPDATE_COMPLETED"
        self.replica_states = dict(collections.Counter(r.state for r in ds.replicas))
        self.details = ds.status_dict()


class AppStatusOverview:
    def __init__(self, a: AppState):
        self.name = a.name
        self.status = a.status
        self.message = a.message
        self.last_deployed_time_s = a.deployed_at
        self.route_prefix = a.route_prefix
        self.deployments = {n: DeploymentStatusOverview(d) for n, d in a.deployments.items()}


class ServeStatus:
    def __init__(self, applications: dict):
        self.applications = applications


# ---------------------------------------------------------------------- singletons


_controller: ServeController | None = None
_child_router = None


def _detect_gpus() -> list[int]:
    env = os.environ.get("BIOENGINE_GPU_IDS")
    if env is not None:
        return [int(x) for x in env.split(",") if x.strip() != ""]
    try:
        import torch

        return list(range(torch.cuda.device_count()))
    except Exception:
        return []


def get_controller(**kw) -> ServeController:
    global _controller
    if _controller is None:
        _controller = ServeController(**kw)
    return _controller


def set_controller(c: ServeController | None):
    global _controller
    _controller = c


async def shutdown_controller():
    global _controller
    if _controller is not None:
        await _controller.shutdown()
        _controller = None


def _set_child_router(r):
    global _child_router
    _child_router = r


def get_router():
    """The object that routes handle calls: the controller, or (inside a replica process) the parent."""
    if _child_router is not None:
        return _child_router
    return get_controller()
