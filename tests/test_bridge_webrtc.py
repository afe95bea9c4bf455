"""WebRTC plumbing of the app bridge (reference bioengine/apps/proxy_deployment.py:599-732): ICE
server resolution order (deploy-time list > TURN endpoint > library defaults) and peer-connection
tracking behind get_num_pcs.  aiortc / hypha_rpc are not importable here, so the endpoint is a local
aiohttp server and the peer connection a minimal event emitter."""
import asyncio
import types

from aiohttp import web

from bioengine_worker_amd.apps.bridge import AppServiceBridge


def _bridge(ice=None):
    built = types.SimpleNamespace(metadata={"ice_servers": ice}, method_schemas=[])
    return AppServiceBridge("app-x", built, None, "local://", None, None, "wk")


async def _serve(payload, status=200):
    async def h(_req):
        return web.json_response(payload, status=status)

    app = web.Application()
    app.router.add_get("/ice", h)
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    port = site._server.sockets[0].getsockname()[1]
    return runner, f"http://127.0.0.1:{port}/ice"


def test_ice_servers_resolution_order():
    servers = [{"urls": "stun:stun.example.org:19302"},
               {"urls": "turn:turn.example.org:3478", "username": "u", "credential": "p"}]

    async def run():
        custom = [{"urls": "stun:custom:1"}]
        assert await _bridge(custom).fetch_ice_servers(url="http://127.0.0.1:9/never") == custom
        runner, url = await _serve(servers)
        try:
            assert await _bridge().fetch_ice_servers(url=url) == servers
        finally:
            await runner.cleanup()
        runner, url = await _serve({"error": "nope"}, status=500)
        try:
            assert await _bridge().fetch_ice_servers(url=url) is None  # HTTP error -> defaults
        finally:
            await runner.cleanup()
        runner, url = await _serve({"not": "a list"})
        try:
            assert await _bridge().fetch_ice_servers(url=url) is None  # malformed payload -> defaults
        finally:
            await runner.cleanup()
        assert await _bridge().fetch_ice_servers(url="http://127.0.0.1:9/closed", timeout=2) is None

    asyncio.run(run())


class _FakePC:
    def __init__(self):
        self.connectionState = "new"
        self._h = {}

    def on(self, ev):
        def deco(fn):
            self._h[ev] = fn
            return fn
        return deco

    def set(self, state):
        self.connectionState = state
        self._h["connectionstatechange"]()


def test_peer_connections_tracked_until_closed():
    async def run():
        b = _bridge()
        a, c = _FakePC(), _FakePC()
        await b.on_webrtc_init(a)
        await b.on_webrtc_init(c)
        assert await b.get_num_pcs() == 2
        a.set("connected")
        assert await b.get_num_pcs() == 2
        a.set("closed")
        assert await b.get_num_pcs() == 1
        c.set("failed")
        assert await b.get_num_pcs() == 0
        await b.on_webrtc_init(object())  # no event API: still counted, no crash
        assert await b.get_num_pcs() == 1

    asyncio.run(run())
