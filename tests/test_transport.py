"""Hub transport: in-process and over WebSocket (two clients relayed by the server)."""
import asyncio

import numpy as np
import pytest

from bioengine_worker_amd.transport import connect_to_server
from bioengine_worker_amd.transport.hub import Hub, get_local_hub, reset_local_hubs
from bioengine_worker_amd.transport.hub_server import HubServer


def run(coro):
    return asyncio.run(coro)


def _service(received):
    async def whoami(context=None):
        return context["user"]["id"]

    async def add(a, b, context=None):
        return a + b

    async def stream(n, cb, context=None):
        for i in range(n):
            await cb(f"line {i}")
        return n

    def matsum(x, context=None):
        received.append(x)
        return float(np.asarray(x).sum()), np.asarray(x) * 2

    return {"id": "calc", "name": "Calc", "type": "calc", "config": {"visibility": "public", "require_context": True},
            "whoami": whoami, "add": add, "stream": stream, "matsum": matsum, "nested": {"mul": lambda a, b, context=None: a * b}}


async def _exercise(url, hub):
    tok_a = hub.issue_token("alice", workspace="ws-a")
    tok_b = hub.issue_token("bob", workspace="ws-b")
    a = await connect_to_server({"server_url": url, "token": tok_a, "client_id": "worker"})
    b = await connect_to_server({"server_url": url, "token": tok_b, "client_id": "user"})
    received = []
    info = await a.register_service(_service(received))
    assert info.id == "ws-a/worker:calc"
    svc = await b.get_service("ws-a/worker:calc")
    assert await svc.whoami() == "bob"  # context is the CALLER's
    assert await svc.add(2, 3) == 5
    assert await svc.nested.mul(3, 4) == 12
    lines = []
    assert await svc.stream(3, lambda s: lines.append(s)) == 3
    assert lines == ["line 0", "line 1", "line 2"]
    arr = np.arange(12, dtype=np.float32).reshape(3, 4)
    s, doubled = await svc.matsum(arr)
    assert s == 66.0 and np.array_equal(doubled, arr * 2)
    with pytest.raises(Exception):
        await svc.add(1)
    tok = await a.generate_token({"expires_in": 60})
    info = await b.parse_token(tok)
    assert info.id == "alice"
    svcs = await b.list_services({"workspace": "ws-a"})
    assert any(x.id == "ws-a/worker:calc" for x in svcs)
    await a.disconnect()
    with pytest.raises(Exception):
        await (await b.get_service("ws-a/worker:calc")).add(1, 2)
    await b.disconnect()


@pytest.mark.unit
def test_inprocess_hub():
    reset_local_hubs()

    async def main():
        hub = get_local_hub("t1")
        await hub.start_http()
        await _exercise("local://t1", hub)
        await hub.stop_http()

    run(main())


@pytest.mark.integration
def test_websocket_hub():
    async def main():
        hub = HubServer(name="ws")
        base = await hub.start_http()
        await _exercise(base.replace("http://", "ws://"), hub)
        await hub.stop_http()

    run(main())


@pytest.mark.unit
def test_artifact_versioning_semantics():
    """Port of tests/test_artifact_version.py (reference): new tag -> new snapshot; re-saving latest
    updates in place; re-saving an older tag is rejected by the app uploader."""
    import httpx

    async def main():
        hub = Hub(name="art")
        await hub.start_http()
        am = hub.artifacts
        ctx = {"user": {"id": "u"}, "ws": "ws1"}
        await am.create(type="collection", alias="applications", config={"permissions": {"*": "r"}}, context=ctx)
        await am.create(type="application", alias="app1", parent_id="ws1/applications",
                        manifest={"version": "1.0"}, stage=True, context=ctx)
        async with httpx.AsyncClient() as c:
            url = await am.put_file("ws1/app1", "main.py", context=ctx)
            await c.put(url, content=b"v1")
            await am.commit("ws1/app1", version="1.0", context=ctx)
            await am.edit("ws1/app1", manifest={"version": "1.1"}, stage=True, version="new", context=ctx)
            url = await am.put_file("ws1/app1", "main.py", context=ctx)
            await c.put(url, content=b"v2")
            await am.commit("ws1/app1", version="1.1", context=ctx)
            a = await am.read("ws1/app1", context=ctx)
            assert [v["version"] for v in a.versions] == ["1.0", "1.1"]
            r1 = await c.get(await am.get_file("ws1/app1", "main.py", version="1.0", context=ctx))
            r2 = await c.get(await am.get_file("ws1/app1", "main.py", context=ctx))
            assert r1.content == b"v1" and r2.content == b"v2"
            # update latest in place
            await am.edit("ws1/app1", manifest={"version": "1.1", "x": 1}, stage=True, version=None, context=ctx)
            url = await am.put_file("ws1/app1", "main.py", context=ctx)
            await c.put(url, content=b"v2b")
            await am.commit("ws1/app1", context=ctx)
            a = await am.read("ws1/app1", context=ctx)
            assert [v["version"] for v in a.versions] == ["1.0", "1.1"] and a.manifest["x"] == 1
            r = await c.get(await am.get_file("ws1/app1", "main.py", context=ctx))
            assert r.content == b"v2b"
            # other workspace can read (public collection) but not write
            other = {"user": {"id": "eve"}, "ws": "ws2"}
            await am.read("ws1/app1", context=other)
            with pytest.raises(PermissionError):
                await am.edit("ws1/app1", manifest={}, stage=True, context=other)
        await hub.stop_http()

    run(main())


@pytest.mark.unit
def test_anonymous_cannot_join_or_hijack_workspace():
    """an anonymous client must not join a named workspace (and so call its
    protected services), and nobody but the same user may replace a live client id."""

    async def main():
        hub = Hub(name="sec")
        tok = hub.issue_token("admin", workspace="ws-user-admin")
        admin = hub.open_session(tok, client_id="worker")
        await hub.register_service(admin, {"id": "secret", "config": {"visibility": "protected"},
                                           "peek": lambda: "classified"})
        with pytest.raises(PermissionError):
            hub.open_session(None, workspace="ws-user-admin", client_id="spy")
        with pytest.raises(PermissionError):  # hijack the worker's client id as another user
            hub.open_session(hub.issue_token("eve", workspace="ws-user-admin"), client_id="worker")
        anon = hub.open_session(None)
        assert anon.workspace.startswith("ws-anonymouz-")
        with pytest.raises(PermissionError):
            await hub.call(anon, "ws-user-admin/worker:secret", "peek", [], {})
        assert await hub.call(admin, "ws-user-admin/worker:secret", "peek", [], {}) == "classified"
        # the same user reconnecting replaces its own stale session; closing the OLD one later
        # must not drop the new session or its services
        again = hub.open_session(tok, client_id="worker")
        await hub.register_service(again, {"id": "secret", "config": {"visibility": "protected"},
                                           "peek": lambda: "v2"})
        hub.close_session(admin)
        assert hub.sessions["ws-user-admin/worker"] is again
        assert await hub.call(again, "ws-user-admin/worker:secret", "peek", [], {}) == "v2"

    run(main())
