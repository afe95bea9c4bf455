"""AppServiceBridge: exposes a running application as a Hypha/hub service.

Replaces the reference's ``ProxyDeployment`` Ray Serve deployment
(``bioengine/apps/proxy_deployment.py``): per-method authorization (method-specific rule, then
``"*"``, else deny; ``:345-403``), a concurrency cap of ``max_ongoing_requests`` (``:249,507``),
service registration with every entry ``@schema_method`` plus ``get_load``, ``get_num_pcs`` and
``get_rtc_service_id`` (``:854-930``), and health-driven deregistration so clients stop seeing a
broken app (``:997-1088``).

Architecturally it is *not* a separate serving deployment: it lives in the worker process next to
the native router, so a client request goes hub -> worker -> (in-process or GPU) replica, one
process hop fewer than proxy-replica -> entry-replica -> runtime-replica.  The "mimic HTTP
request" the reference sends to make Ray's autoscaler see RPC load (``:405-442``) is unnecessary:
the router measures load directly.

Service ids keep the reference format ``{ws}/{worker_client_id}-{bridge_id}:{application_id}``
(and ``...:{application_id}-rtc`` when WebRTC is available).
"""
from __future__ import annotations

import asyncio
import logging
import os
import time
import uuid

from ..transport.client import connect_to_server


class AppServiceBridge:
    def __init__(self, application_id: str, built, handle, server_url: str, token: str | None,
                 workspace: str | None, worker_client_id: str, logger: logging.Logger | None = None):
        self.application_id = application_id
        self.built = built
        self.handle = handle
        self.server_url = server_url
        self.token = token
        self.workspace = workspace
        self.worker_client_id = worker_client_id
        self.bridge_id = uuid.uuid4().hex[:8]
        self.log = logger or logging.getLogger("bioengine.bridge")
        self.max_ongoing = int(built.metadata.get("max_ongoing_requests") or 10)
        self.sem = asyncio.Semaphore(self.max_ongoing)
        self.active = 0
        self.authorized_users = dict(built.metadata.get("authorized_users") or {"*": []})
        self.client = None
        self.service_id: str | None = None
        self.rtc_service_id: str | None = None
        # WebRTC: deploy-time ICE servers (else fetched, else hypha-rpc's defaults) and the live
        # peer connections get_num_pcs reports (reference proxy_deployment.py:599-732, 767-791)
        self.ice_servers = built.metadata.get("ice_servers")
        self.peer_connections: dict[str, dict] = {}
        self.registered = False
        self.calls = 0
        self.errors = 0
        self.latency: list[float] = []

    # ------------------------------------------------------------------ auth
    def check_permissions(self, context: dict | None, method: str = "*"):
        if not isinstance(context, dict) or not isinstance(context.get("user"), dict):
            raise PermissionError("Invalid context without user information")
        user = context["user"]
        uid, email = user.get("id", ""), user.get("email", "")
        if not uid and not email:
            raise PermissionError("Invalid user information in context")
        allowed = self.authorized_users.get(method) or self.authorized_users.get("*")
        if not allowed or not ("*" in allowed or uid in allowed or email in allowed):
            raise PermissionError(f"User '{uid}' ({email}) is not authorized to call '{method}' on application "
                                  f"'{self.application_id}'")

    def update_authorized_users(self, users: dict):
        self.authorized_users = dict(users)

    # ------------------------------------------------------------------ service functions
    def _make_method(self, schema: dict):
        name = schema["name"]
        pass_ctx = bool(schema.get("_accepts_context"))

        async def fn(*args, context=None, **kwargs):
            self.check_permissions(context, name)
            if pass_ctx:
                kwargs["context"] = context
            async with self.sem:
                self.active += 1
                t0 = time.perf_counter()
                try:
                    self.calls += 1
                    return await getattr(self.handle, name).remote(*args, **kwargs)
                except Exception:
                    self.errors += 1
                    raise
                finally:
                    self.active -= 1
                    self.latency.append(time.perf_counter() - t0)
                    if len(self.latency) > 4096:
                        del self.latency[:2048]

        fn.__name__ = name
        fn.__doc__ = schema.get("description")
        fn.__schema__ = schema
        return fn

    async def get_load(self, context=None) -> float:
        return self.active / max(1, self.max_ongoing)

    async def get_num_pcs(self, context=None) -> int:
        return len(self.peer_connections)

    # ------------------------------------------------------------------ WebRTC
    ICE_SERVERS_URL = "https://hypha.aicell.io/turn-server/services/coturn/get_rtc_ice_servers"

    async def fetch_ice_servers(self, url: str | None = None, timeout: float = 30.0) -> list | None:
        """ICE servers for the RTC service: the deploy-time list if one was given, else the TURN
        endpoint's list (``BIOENGINE_ICE_SERVERS_URL`` overrides the URL), else None so hypha-rpc uses
        its built-in defaults.  Fetch failures are logged, never raised."""
        if self.ice_servers is not None:
            return self.ice_servers
        url = url or os.environ.get("BIOENGINE_ICE_SERVERS_URL") or self.ICE_SERVERS_URL
        try:
            import httpx

            async with httpx.AsyncClient(timeout=timeout) as client:
                r = await client.get(url)
                r.raise_for_status()
                servers = r.json()
            if not isinstance(servers, list) or not all(isinstance(e, dict) and "urls" in e for e in servers):
                raise ValueError(f"unexpected ICE server payload: {str(servers)[:200]}")
            return servers
        except Exception as e:  # noqa: BLE001
            self.log.warning(f"ICE server fetch for '{self.application_id}' failed ({type(e).__name__}: {e}); "
                             "using the RTC library's defaults")
            return None

    async def on_webrtc_init(self, peer_connection) -> None:
        """hypha-rpc ``on_init`` hook: track the connection until it reports closed / failed."""
        cid = uuid.uuid4().hex
        self.peer_connections[cid] = {"created_at": time.time(), "state": "new"}

        def on_state_change():
            state = getattr(peer_connection, "connectionState", None)
            ent = self.peer_connections.get(cid)
            if ent is None:
                return
            ent["state"] = state
            if state in ("closed", "failed"):
                self.peer_connections.pop(cid, None)
            self.log.info(f"WebRTC connection {cid[:8]} of '{self.application_id}' -> {state} "
                          f"({len(self.peer_connections)} active)")

        try:
            peer_connection.on("connectionstatechange")(on_state_change)
        except Exception as e:  # noqa: BLE001  (not an event emitter: keep counting it)
            self.log.warning(f"WebRTC connection {cid[:8]}: no state events ({e})")

    async def get_rtc_service_id(self, context=None):
        return self.rtc_service_id

    def service_dict(self) -> dict:
        md = self.built.metadata
        svc = {
            "id": self.application_id,
            "name": md.get("display_name", self.application_id),
            "type": "bioengine-app",
            "description": md.get("description", ""),
            "config": {"visibility": "public", "require_context": True},
            "service_schema": {s["name"]: s for s in self.built.method_schemas},
            "get_load": self.get_load,
            "get_num_pcs": self.get_num_pcs,
            "get_rtc_service_id": self.get_rtc_service_id,
        }
        for s in self.built.method_schemas:
            svc[s["name"]] = self._make_method(s)
        return svc

    # ------------------------------------------------------------------ lifecycle
    async def start(self):
        cfg = {"server_url": self.server_url, "token": self.token, "client_id": f"{self.worker_client_id}-{self.bridge_id}"}
        if self.workspace:
            cfg["workspace"] = self.workspace
        self.client = await connect_to_server(cfg)
        info = await self.client.register_service(self.service_dict())
        self.service_id = info.id if hasattr(info, "id") else info["id"]
        self.registered = True
        try:
            import aiortc  # noqa: F401

            from hypha_rpc import register_rtc_service  # type: ignore

            rtc_id = f"{self.application_id}-rtc"
            rtc_cfg = {"visibility": "public", "on_init": self.on_webrtc_init}
            ice = await self.fetch_ice_servers()
            if ice:
                rtc_cfg["ice_servers"] = ice
            await register_rtc_service(self.client, rtc_id, rtc_cfg)
            self.rtc_service_id = f"{self.service_id.split(':')[0]}:{rtc_id}"
        except Exception:
            self.rtc_service_id = None
        self.log.info(f"Registered application service '{self.service_id}'")

    async def deregister(self):
        if self.client is not None and self.registered:
            try:
                await self.client.unregister_service(self.service_id)
            except Exception:
                pass
            self.registered = False

    async def reregister(self):
        if self.client is not None and not self.registered:
            info = await self.client.register_service(self.service_dict())
            self.service_id = info.id if hasattr(info, "id") else info["id"]
            self.registered = True

    async def stop(self):
        await self.deregister()
        if self.client is not None:
            try:
                await self.client.disconnect()
            except Exception:
                pass
            self.client = None

    def service_ids(self) -> list[dict]:
        if not self.service_id:
            return []
        return [{"websocket_service_id": self.service_id, "webrtc_service_id": self.rtc_service_id}]

    def metrics(self) -> dict:
        lat = sorted(self.latency)
        pct = (lambda q: round(1e3 * lat[int(q * (len(lat) - 1))], 3)) if lat else (lambda q: None)
        return {"calls": self.calls, "errors": self.errors, "active": self.active, "max_ongoing": self.max_ongoing,
                "latency_ms": {"p50": pct(0.5), "p95": pct(0.95), "p99": pct(0.99)}}
