"""Datasets server + client (reference's datasets e2e tests are skip placeholders; these are real)."""
import asyncio
import threading
import time

import numpy as np
import pytest
import yaml


@pytest.fixture()
def data_server(tmp_path):
    import uvicorn

    from bioengine_worker_amd.datasets.server import build_app
    from bioengine_worker_amd.transport.hub_server import HubServer
    from bioengine_worker_amd.utils.network import acquire_free_port
    from bioengine_worker_amd.datasets.store import write_zarr_array

    d = tmp_path / "data"
    (d / "blobs").mkdir(parents=True)
    (d / "blobs" / "manifest.yaml").write_text(yaml.safe_dump({"id": "blobs", "authorized_users": ["*"]}))
    (d / "blobs" / "a.txt").write_text("hello")
    arr = np.arange(40 * 30, dtype=np.uint16).reshape(40, 30)
    write_zarr_array(str(d / "blobs" / "img.zarr"), arr, (16, 16), compress=True)
    (d / "secret").mkdir()
    (d / "secret" / "manifest.yaml").write_text(yaml.safe_dump({"id": "secret", "authorized_users": ["alice"]}))
    (d / "secret" / "x.bin").write_bytes(b"\x00\x01")

    hub = HubServer(name="ds")
    loop = asyncio.new_event_loop()
    base = loop.run_until_complete(hub.start_http())
    th_hub = threading.Thread(target=loop.run_forever, daemon=True)
    th_hub.start()
    port = acquire_free_port(0)
    app = build_app(d, auth_url=base.replace("http", "ws"))
    cfg = uvicorn.Config(app, host="127.0.0.1", port=port, log_level="warning")
    server = uvicorn.Server(cfg)
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    for _ in range(100):
        if server.started:
            break
        time.sleep(0.05)
    yield f"http://127.0.0.1:{port}", hub, arr
    server.should_exit = True
    th.join(5)
    loop.call_soon_threadsafe(loop.stop)


@pytest.mark.integration
def test_datasets_roundtrip(data_server):
    from bioengine_worker_amd.datasets import BioEngineDatasets, read_zarr_array

    url, hub, arr = data_server
    tok = hub.issue_token("alice", workspace="ws-a")

    async def main():
        anon = BioEngineDatasets(url)
        assert await anon.ping_data_server()
        ds = await anon.list_datasets()
        assert set(ds) == {"blobs", "secret"}
        assert "a.txt" in await anon.list_files("blobs")
        assert await anon.get_file("blobs", "a.txt") == b"hello"
        with pytest.raises(PermissionError):
            await anon.list_files("secret")
        store = await anon.get_file("blobs", "img.zarr")
        full = await read_zarr_array(store)
        np.testing.assert_array_equal(full, arr)
        part = await read_zarr_array(store, region=(slice(5, 33), slice(10, 29)))
        np.testing.assert_array_equal(part, arr[5:33, 10:29])
        alice = BioEngineDatasets(url, hypha_token=tok)
        assert await alice.get_file("secret", "x.bin") == b"\x00\x01"
        r = await alice.save_file("notes.txt", "private", public=False)
        assert r["dataset_id"].startswith("saved-")
        await alice.save_file("pub.txt", b"pub", public=True)
        with pytest.raises(RuntimeError):
            await alice.save_file("pub.txt", b"again", public=True)  # public files are immutable
        saved = await alice.list_saved_files()
        assert "notes.txt" in saved["private"] and "pub.txt" in saved["public"]
        assert await alice.get_saved_file("notes.txt") == b"private"
        await anon.close()
        await alice.close()

    asyncio.run(main())
