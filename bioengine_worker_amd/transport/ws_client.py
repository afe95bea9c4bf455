"""WebSocket client for a BioEngine hub server (same API as the in-process ServerClient)."""
from __future__ import annotations

import asyncio
import inspect
import itertools

from .client import ServiceProxy
from .hub import ObjDict, _resolve_method
from .wire import error_payload, pack, raise_remote, unpack


def _method_names(svc: dict, prefix: str = "") -> list[str]:
    out = []
    for k, v in svc.items():
        if k in ("config",) or k.startswith("_"):
            continue
        if callable(v):
            out.append(prefix + k)
        elif isinstance(v, dict) and k not in ("service_schema",):
            out.extend(_method_names(v, prefix + k + "."))
    return out


class WSServerClient:
    def __init__(self, url: str):
        self.url = url
        self._http = None
        self.ws = None
        self.pending: dict[int, asyncio.Future] = {}
        self.ids = itertools.count(1)
        self.cbs: dict[str, object] = {}
        self.cb_ids = itertools.count(1)
        self.services: dict[str, dict] = {}
        self.config = ObjDict()
        self._reader = None
        self._send_lock = asyncio.Lock()

    # -- plumbing
    def _register_cb(self, fn) -> str:
        cid = f"c{next(self.cb_ids)}"
        self.cbs[cid] = fn
        return cid

    def _cb_proxy(self, cbid):
        async def proxy(*args, **kwargs):
            return await self._req("cb", cb=cbid, args=list(args), kwargs=kwargs)
        return proxy

    async def _send(self, msg):
        data = pack(msg, self._register_cb)
        async with self._send_lock:
            await self.ws.send_bytes(data)

    async def _req(self, op, **kwargs):
        mid = next(self.ids)
        fut = asyncio.get_running_loop().create_future()
        self.pending[mid] = fut
        await self._send({"t": "req", "id": mid, "op": op, "kwargs": kwargs})
        res = await fut
        if not res.get("ok"):
            raise_remote(res.get("error", {}))
        return _objify(res.get("result"))

    async def connect(self, cfg: dict):
        import aiohttp

        url = self.url.replace("http://", "ws://").replace("https://", "wss://").rstrip("/")
        if not url.endswith("/ws"):
            url += "/ws"
        self._http = aiohttp.ClientSession()
        self.ws = await self._http.ws_connect(url, max_msg_size=0, heartbeat=30)
        await self.ws.send_bytes(pack({"t": "hello", "token": cfg.get("token"), "workspace": cfg.get("workspace"),
                                       "client_id": cfg.get("client_id")}))
        msg = await self.ws.receive()
        w = unpack(msg.data)
        if not w.get("ok"):
            await self._http.close()
            raise_remote(w.get("error", {}))
        self.config = ObjDict(workspace=w["workspace"], client_id=w["client_id"], user=w.get("user"),
                              public_base_url=w.get("public_base_url"), server_url=self.url)
        self._reader = asyncio.create_task(self._read_loop())
        return self

    async def _read_loop(self):
        from aiohttp import WSMsgType

        try:
            async for msg in self.ws:
                if msg.type != WSMsgType.BINARY:
                    continue
                d = unpack(msg.data, self._cb_proxy)
                t = d.get("t")
                if t == "res":
                    fut = self.pending.pop(d.get("id"), None)
                    if fut is not None and not fut.done():
                        fut.set_result(d)
                elif t in ("call", "cb"):
                    asyncio.create_task(self._serve(d))
        finally:
            for fut in self.pending.values():
                if not fut.done():
                    fut.set_exception(ConnectionError("hub connection closed"))

    async def _serve(self, d):
        try:
            if d["t"] == "call":
                svc = self.services[d["service"].split(":")[-1]]
                fn = _resolve_method(svc, d["method"])
            else:
                fn = self.cbs[d["cb"]]
            res = fn(*(d.get("args") or []), **(d.get("kwargs") or {}))
            if inspect.isawaitable(res):
                res = await res
            await self._send({"t": "res", "id": d["id"], "ok": True, "result": res})
        except Exception as e:  # noqa: BLE001
            await self._send({"t": "res", "id": d["id"], "ok": False, "error": error_payload(e)})

    # -- hypha-rpc surface
    async def register_service(self, service: dict, overwrite: bool = True, **_):
        sid = service.get("id", "default")
        self.services[sid] = service
        meta = {k: v for k, v in service.items() if not callable(v) and not (isinstance(v, dict) and k not in ("config", "service_schema"))}
        meta["__methods__"] = _method_names(service)
        return await self._req("register_service", service=meta, overwrite=overwrite)

    async def unregister_service(self, service_id: str, **_):
        await self._req("unregister_service", service_id=service_id)
        self.services.pop(service_id.split(":")[-1], None)

    async def get_service(self, service_id, config=None, **_):
        if isinstance(service_id, dict):
            service_id = service_id.get("id")
        r = await self._req("get_service", service_id=service_id)
        info = ObjDict(r["info"])
        full = info["id"]

        async def caller(method, args, kwargs):
            return await self._req("call", service_id=full, method=method, args=args, kwargs=kwargs)

        return ServiceProxy(caller, info, r.get("methods"))

    async def list_services(self, query=None, **_):
        return await self._req("list_services", query=query)

    async def generate_token(self, config: dict | None = None, **_):
        return await self._req("generate_token", config=config or {})

    async def parse_token(self, token: str, **_):
        return await self._req("parse_token", token=token)

    async def echo(self, x, **_):
        return await self._req("echo", value=x)

    async def disconnect(self):
        try:
            if self.ws is not None:
                await self.ws.close()
        finally:
            if self._http is not None:
                await self._http.close()
            if self._reader is not None:
                self._reader.cancel()

    async def get_ice_servers(self):
        return []


def _objify(x):
    if isinstance(x, dict):
        return ObjDict({k: _objify(v) for k, v in x.items()})
    if isinstance(x, list):
        return [_objify(v) for v in x]
    return x


async def connect_ws(url: str, cfg: dict) -> WSServerClient:
    c = WSServerClient(url)
    return await c.connect(cfg)
