"""WebSocket front-end of the BioEngine hub: ``python -m bioengine_worker_amd.transport.hub_server``.

Clients connect to ``ws://host:port/ws`` and exchange msgpack frames (:mod:`.wire`):

client -> server  ``{"t": "hello", token, workspace, client_id}`` then
                  ``{"t": "req", id, op, kwargs}`` with op in register_service / unregister_service /
                  get_service / list_services / generate_token / parse_token / echo / call / cb
server -> client  ``{"t": "res", id, ok, result | error}``,
                  ``{"t": "call", id, service, method, args, kwargs}`` (invoke a service the client
                  registered; the server has already injected ``context``), ``{"t": "cb", ...}``.

Service calls between two WebSocket clients are relayed by the server, exactly the topology of a
Hypha deployment (worker, app replicas and users are all clients of one server).
"""
from __future__ import annotations

import argparse
import asyncio
import itertools
import logging

from .hub import Hub, ObjDict
from .wire import error_payload, pack, raise_remote, unpack

log = logging.getLogger("bioengine.hub")


def _stub(*_a, **_k):  # placeholder for methods living in a remote client
    raise RuntimeError("remote method stub called locally")


class _Conn:
    def __init__(self, ws):
        self.ws = ws
        self.pending: dict[int, asyncio.Future] = {}
        self.ids = itertools.count(1)
        self.cbs: dict[str, object] = {}  # server-side callables exposed to this client
        self.cb_ids = itertools.count(1)
        self.send_lock = asyncio.Lock()

    def register_cb(self, fn) -> str:
        cid = f"s{next(self.cb_ids)}"
        self.cbs[cid] = fn
        return cid

    async def send(self, msg):
        data = pack(msg, self.register_cb)
        async with self.send_lock:
            await self.ws.send_bytes(data)

    async def request(self, msg) -> object:
        mid = next(self.ids)
        fut = asyncio.get_running_loop().create_future()
        self.pending[mid] = fut
        msg["id"] = mid
        await self.send(msg)
        res = await fut
        if not res.get("ok"):
            raise_remote(res.get("error", {}))
        return res.get("result")

    def make_cb_proxy(self, cbid: str):
        async def proxy(*args, **kwargs):
            return await self.request({"t": "cb", "cb": cbid, "args": list(args), "kwargs": kwargs})
        return proxy


class HubServer(Hub):
    def _extra_routes(self, app):
        app.router.add_get("/ws", self._ws_handler)

    async def _ws_handler(self, request):
        from aiohttp import WSMsgType, web

        ws = web.WebSocketResponse(max_msg_size=0, heartbeat=30)
        await ws.prepare(request)
        conn = _Conn(ws)
        session = None
        try:
            first = await ws.receive()
            hello = unpack(first.data)
            async def remote_caller(local_id, method, args, kwargs):
                return await conn.request({"t": "call", "service": local_id, "method": method, "args": args,
                                           "kwargs": kwargs})
            try:
                session = self.open_session(hello.get("token"), hello.get("workspace"), hello.get("client_id"),
                                            remote_caller=remote_caller)
            except Exception as e:
                await conn.send({"t": "welcome", "ok": False, "error": error_payload(e)})
                return ws
            await conn.send({"t": "welcome", "ok": True, "workspace": session.workspace, "client_id": session.client_id,
                             "user": session.user, "public_base_url": self.public_base_url})
            async for msg in ws:
                if msg.type != WSMsgType.BINARY:
                    continue
                d = unpack(msg.data, conn.make_cb_proxy)
                t = d.get("t")
                if t == "res":
                    fut = conn.pending.pop(d.get("id"), None)
                    if fut is not None and not fut.done():
                        fut.set_result(d)
                elif t == "req":
                    asyncio.create_task(self._handle(conn, session, d))
        finally:
            for fut in conn.pending.values():
                if not fut.done():
                    fut.set_exception(ConnectionError("client disconnected"))
            if session is not None:
                self.close_session(session)
        return ws

    async def _handle(self, conn: _Conn, session, d):
        op, kw, rid = d.get("op"), d.get("kwargs") or {}, d.get("id")
        try:
            if op == "register_service":
                svc = dict(kw["service"])
                methods = svc.pop("__methods__", [])
                for m in methods:
                    svc.setdefault(m, _stub)
                result = await self.register_service(session, svc, kw.get("overwrite", True))
            elif op == "unregister_service":
                result = await self.unregister_service(session, kw["service_id"])
            elif op == "get_service":
                e = self._find(session, kw["service_id"])
                result = {"info": e.info, "methods": [k for k in e.methods() if k not in ("config",)]}
            elif op == "list_services":
                result = self.list_service_infos(session, kw.get("query"))
            elif op == "generate_token":
                import time

                cfg = kw.get("config") or {}
                u = session.user
                result = self.tokens.mint({"id": u["id"], "email": u.get("email"),
                                           "workspace": cfg.get("workspace", session.workspace),
                                           "permission": cfg.get("permission", "read_write"),
                                           "expires_at": time.time() + float(cfg.get("expires_in", 3600)),
                                           "roles": u.get("roles", [])})
            elif op == "parse_token":
                p = self.tokens.parse(kw["token"])
                result = ObjDict(id=p["id"], email=p.get("email"), expires_at=p.get("expires_at"),
                                 scope={"workspaces": {p["workspace"]: p.get("permission")}}, roles=p.get("roles", []))
            elif op == "echo":
                result = kw.get("value")
            elif op == "call":
                result = await self.call(session, kw["service_id"], kw["method"], kw.get("args") or [],
                                         kw.get("kwargs") or {})
            elif op == "cb":
                fn = conn.cbs.get(kw["cb"])
                if fn is None:
                    raise KeyError(f"callback {kw['cb']} expired")
                result = fn(*(kw.get("args") or []), **(kw.get("kwargs") or {}))
                if asyncio.iscoroutine(result):
                    result = await result
            else:
                raise ValueError(f"unknown op {op}")
            await conn.send({"t": "res", "id": rid, "ok": True, "result": result})
        except Exception as e:  # noqa: BLE001
            try:
                await conn.send({"t": "res", "id": rid, "ok": False, "error": error_payload(e)})
            except Exception:
                pass


async def serve(host: str, port: int, data_dir: str | None, admin_user: str, token_file: str | None):
    hub = HubServer(data_dir=data_dir, name="server")
    base = await hub.start_http(host, port)
    hub.ws_server_url = base.replace("http://", "ws://")
    tok = hub.issue_token(admin_user, workspace=f"ws-user-{admin_user}", roles=["admin"], expires_in=3600 * 24 * 30)
    print(f"BioEngine hub listening on {base} (ws: {hub.ws_server_url}/ws)", flush=True)
    print(f"admin token for '{admin_user}': {tok}", flush=True)
    if token_file:
        with open(token_file, "w") as f:
            f.write(tok)
    await asyncio.Event().wait()


def main(argv=None):
    ap = argparse.ArgumentParser(description="BioEngine hub (Hypha-compatible RPC/artifact server)")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=9527)
    ap.add_argument("--data-dir", default=None)
    ap.add_argument("--admin-user", default="admin")
    ap.add_argument("--token-file", default=None)
    a = ap.parse_args(argv)
    asyncio.run(serve(a.host, a.port, a.data_dir, a.admin_user, a.token_file))


if __name__ == "__main__":
    main()
