"""Client side of the BioEngine hub (Hypha-compatible surface).

``await connect_to_server({"server_url": ..., "token": ..., "workspace": ..., "client_id": ...})``
returns a :class:`ServerClient` with the calls the reference makes on a hypha-rpc server object
(``register_service``, ``unregister_service``, ``get_service``, ``list_services``,
``generate_token``, ``parse_token``, ``echo``, ``disconnect``, ``config``).

* ``local://<name>`` (or ``local``) — the in-process :class:`~.hub.Hub` named ``<name>``.
* ``ws://host:port`` / ``http://host:port`` — a hub server in another process
  (:mod:`.ws_client`), same API.
* Any other ``http(s)://`` URL uses the real ``hypha_rpc`` package when it is installed.
"""
from __future__ import annotations

import asyncio
import inspect
import time
from typing import Any

from .hub import Hub, ObjDict, Session, get_local_hub


class ServiceProxy:
    """Remote service handle: attribute access returns awaitable remote methods."""

    def __init__(self, caller, info: ObjDict, method_names: list[str] | None = None):
        self._caller = caller  # async fn(method, args, kwargs)
        self._info = info
        self._methods = method_names

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        if name in self._info:
            return self._info[name]
        return _RemoteMethod(self._caller, name)

    def __getitem__(self, k):
        return getattr(self, k)

    def __repr__(self):
        return f"<ServiceProxy {self._info.get('id')}>"

    def keys(self):
        return list(self._info.keys()) + list(self._methods or [])


class _RemoteMethod:
    def __init__(self, caller, path):
        self._caller = caller
        self._path = path

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return _RemoteMethod(self._caller, f"{self._path}.{name}")

    def __call__(self, *args, **kwargs):
        kwargs.pop("_rkwargs", None)
        return self._caller(self._path, list(args), kwargs)


class ServerClient:
    """In-process client bound to one hub Session."""

    def __init__(self, hub: Hub, session: Session, server_url: str):
        self.hub = hub
        self.session = session
        self.server_url = server_url
        self.config = ObjDict(workspace=session.workspace, client_id=session.client_id,
                              public_base_url=hub.public_base_url or server_url, server_url=server_url,
                              user=session.user)

    # -- the hypha-rpc server surface
    async def register_service(self, service: dict, overwrite: bool = True, **_):
        return await self.hub.register_service(self.session, service, overwrite)

    async def unregister_service(self, service_id: str, **_):
        await self.hub.unregister_service(self.session, service_id)

    async def get_service(self, service_id, config=None, **_):
        if isinstance(service_id, dict):
            service_id = service_id.get("id")
        entry = self.hub._find(self.session, service_id)
        full = entry.full_id

        async def caller(method, args, kwargs):
            return await self.hub.call(self.session, full, method, args, kwargs)

        return ServiceProxy(caller, entry.info, list(entry.methods().keys()))

    async def list_services(self, query=None, **_):
        return self.hub.list_service_infos(self.session, query)

    async def generate_token(self, config: dict | None = None, **_):
        config = config or {}
        u = self.session.user
        return self.hub.tokens.mint({
            "id": u["id"], "email": u.get("email"), "workspace": config.get("workspace", self.session.workspace),
            "permission": config.get("permission", "read_write"),
            "expires_at": time.time() + float(config.get("expires_in", 3600)), "roles": u.get("roles", []),
        })

    async def parse_token(self, token: str, **_):
        p = self.hub.tokens.parse(token)
        return ObjDict(id=p["id"], email=p.get("email"), expires_at=p.get("expires_at"),
                       scope=ObjDict(workspaces={p["workspace"]: p.get("permission")}), roles=p.get("roles", []))

    async def echo(self, x, **_):
        return x

    async def disconnect(self):
        self.hub.close_session(self.session)

    # hypha helper used by ProxyDeployment for WebRTC ICE
    async def get_ice_servers(self):
        return []


async def connect_to_server(config: dict | None = None, **kw) -> Any:
    cfg = dict(config or {})
    cfg.update(kw)
    url = cfg.get("server_url") or "local://default"
    if url == "local" or url.startswith("local://"):
        name = url.split("://", 1)[1] if "://" in url else "default"
        hub = get_local_hub(name or "default")
        if hub.http_base is None:
            await hub.start_http()
        session = hub.open_session(cfg.get("token"), cfg.get("workspace"), cfg.get("client_id"))
        return ServerClient(hub, session, url)
    if url.startswith("ws://") or url.startswith("wss://") or cfg.get("bioengine_hub"):
        from .ws_client import connect_ws

        return await connect_ws(url, cfg)
    if url.startswith("http://127.0.0.1") or url.startswith("http://localhost"):
        from .ws_client import connect_ws

        return await connect_ws(url, cfg)
    try:  # a real Hypha deployment
        from hypha_rpc import connect_to_server as _hypha_connect  # type: ignore

        return await _hypha_connect(cfg)
    except ImportError as e:
        raise RuntimeError(f"hypha_rpc is not installed; cannot connect to {url}. Use local:// or a bioengine hub") from e


def call_maybe_async(fn, *args, **kwargs):
    res = fn(*args, **kwargs)
    if inspect.isawaitable(res):
        return res
    fut = asyncio.get_event_loop().create_future()
    fut.set_result(res)
    return fut
