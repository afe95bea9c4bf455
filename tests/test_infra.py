"""Deployment assets: upload script against a live WebSocket hub, docker / compose / HPC launcher
sanity (no docker or apptainer in CI: structure and shell syntax are checked, not image builds)."""
import asyncio
import json
import subprocess
import sys
import threading
from pathlib import Path

import pytest
import yaml

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def live_hub(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("hub")
    loop = asyncio.new_event_loop()
    ready = threading.Event()
    box = {}

    async def boot():
        from bioengine_worker_amd.transport.hub_server import HubServer

        hub = HubServer(data_dir=str(tmp / "hub"), name="server")
        base = await hub.start_http("127.0.0.1", 0)
        box.update(url=base.replace("http://", "ws://"), hub=hub,
                   tok=hub.issue_token("dev-user", workspace="ws-dev", roles=["admin"]))
        ready.set()

    t = threading.Thread(target=lambda: (loop.run_until_complete(boot()), loop.run_forever()), daemon=True)
    t.start()
    assert ready.wait(60)
    box["loop"] = loop
    yield box
    loop.call_soon_threadsafe(loop.stop)


def test_upload_app_script_roundtrip(live_hub, tmp_path):
    app = tmp_path / "my-app"
    app.mkdir()
    (app / "manifest.yaml").write_text(yaml.safe_dump({
        "id": "my-app", "name": "My app", "id_emoji": "x", "version": "1.0.0", "type": "ray-serve", "description": "x",
        "deployments": ["main:Main"], "authorized_users": ["*"]}))
    (app / "main.py").write_text("class Main:\n    def ping(self):\n        return 'pong'\n")
    (app / "data.bin").write_bytes(bytes(range(256)))
    sys.path.insert(0, str(ROOT / "scripts"))
    import upload_app

    args = upload_app.parse_args([str(app), "--server-url", live_hub["url"], "--token", live_hub["tok"]])
    aid = asyncio.run(upload_app.upload(args))
    assert aid.endswith("/my-app")

    async def files():
        from bioengine_worker_amd.transport import connect_to_server

        s = await connect_to_server({"server_url": live_hub["url"], "token": live_hub["tok"]})
        am = await s.get_service("public/artifact-manager")
        out = await am.list_files(aid)
        await s.disconnect()
        return sorted(f["name"] for f in out)

    assert asyncio.run(files()) == ["data.bin", "main.py", "manifest.yaml"]
    # dry run prints the plan without a server
    r = subprocess.run([sys.executable, str(ROOT / "scripts/upload_app.py"), str(app), "--dry-run"],
                       capture_output=True, text=True, check=True)
    assert json.loads(r.stdout)["id"] == "my-app"


def test_compose_and_dockerfiles():
    c = yaml.safe_load((ROOT / "docker-compose.yaml").read_text())
    w = c["services"]["worker"]
    assert "/dev/kfd" in w["devices"] and "/dev/dri" in w["devices"]  # ROCm, not the nvidia runtime
    assert "HSA_ENABLE_IPC_MODE_LEGACY=0" in w["environment"]
    assert "bioengine_worker_amd.worker" in w["command"]
    assert "bioengine_worker_amd.datasets" in c["services"]["data-server"]["command"]
    wd = (ROOT / "docker/worker.Dockerfile").read_text()
    assert "gfx950" in wd and "tools/build_native.py" in wd
    assert "nvidia" not in wd.lower() and "cuda" not in wd.lower()
    assert (ROOT / "docker/datasets.Dockerfile").exists()


def test_hpc_launcher_shell_syntax_and_rocm():
    sh = ROOT / "scripts/start_hpc_worker.sh"
    subprocess.run(["bash", "-n", str(sh)], check=True)
    text = sh.read_text()
    assert "exec --rocm" in text and "exec --nv" not in text
    assert "bioengine-worker" in text  # cancels the SLURM jobs named by cluster/slurm.py
    from bioengine_worker_amd.cluster.slurm import JOB_NAME

    assert JOB_NAME == "bioengine-worker"


def test_pyproject_entry_points_resolve():
    import importlib

    try:
        import tomllib
    except ModuleNotFoundError:  # py3.10
        import tomli as tomllib
    meta = tomllib.loads((ROOT / "pyproject.toml").read_text())
    for target in meta["project"]["scripts"].values():
        mod, fn = target.split(":")
        assert callable(getattr(importlib.import_module(mod), fn))
    from bioengine_worker_amd import __version__

    assert meta["project"]["version"] == __version__


def test_every_app_frontend_entry_exists():
    """Each app that declares a frontend (manifest ``frontend_entry``) ships it; the reference has one
    per app (apps/*/frontend/index.html)."""
    import yaml
    from pathlib import Path

    apps = Path(__file__).resolve().parent.parent / "apps"
    with_fe = 0
    for m in apps.glob("*/manifest.yaml"):
        man = yaml.safe_load(m.read_text())
        fe = man.get("frontend_entry")
        if fe:
            with_fe += 1
            page = (m.parent / fe).read_text()
            assert "ws_service_id" in page and "connectToServer" in page, m.parent.name
    assert with_fe >= 5
