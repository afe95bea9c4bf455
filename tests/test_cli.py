"""``bioengine`` CLI and ``python -m bioengine.worker`` argument handling against a live worker on a
WebSocket hub (hub + worker run on a background event loop; commands run through click's runner)."""
import asyncio
import json
import threading
from pathlib import Path

import pytest
from click.testing import CliRunner

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def live_worker(tmp_path_factory):
    import os

    tmp = tmp_path_factory.mktemp("cli")
    os.environ["BIOENGINE_LOCAL_ARTIFACT_PATH"] = str(ROOT / "apps")
    os.environ["BIOENGINE_REPLICA_MODE"] = "local"
    loop = asyncio.new_event_loop()
    ready = threading.Event()
    box = {}

    async def boot():
        from bioengine_worker_amd.transport.hub_server import HubServer
        from bioengine_worker_amd.worker.worker import BioEngineWorker

        hub = HubServer(data_dir=str(tmp / "hub"), name="server")
        base = await hub.start_http("127.0.0.1", 0)
        url = base.replace("http://", "ws://")
        tok = hub.issue_token("admin-user", workspace="ws-admin", roles=["admin"])
        w = BioEngineWorker(mode="single-machine", workspace_dir=tmp / "be", server_url=url, token=tok, client_id="w1",
                            log_file="off", head_num_cpus=4, head_num_gpus=0, monitoring_interval_seconds=1,
                            data_server_url=None)
        await w.start(blocking=False)
        box.update(url=url, tok=tok, wid=w.full_service_id, w=w)
        ready.set()

    t = threading.Thread(target=lambda: (loop.run_until_complete(boot()), loop.run_forever()), daemon=True)
    t.start()
    assert ready.wait(120)
    yield box
    loop.call_soon_threadsafe(loop.stop)
    os.environ.pop("BIOENGINE_REPLICA_MODE", None)


def _run(args, box):
    from bioengine_worker_amd.cli import main

    env = {"BIOENGINE_SERVER_URL": box["url"], "HYPHA_TOKEN": box["tok"], "BIOENGINE_WORKER_SERVICE_ID": box["wid"]}
    r = CliRunner().invoke(main, args, env=env, catch_exceptions=False)
    assert r.exit_code == 0, r.output
    return r.output


def test_cli_call_and_apps_and_cluster(live_worker):
    out = json.loads(_run(["call", live_worker["wid"], "get_status", "--json"], live_worker))
    assert out["worker_mode"] == "single-machine"
    methods = json.loads(_run(["call", live_worker["wid"], "--list-methods", "--json"], live_worker))["methods"]
    assert "deploy_app" in methods and "get_app_status" in methods
    aid = _run(["apps", "deploy", str(ROOT / "apps" / "demo-app"), "--id", "clidemo", "--no-gpu"], live_worker)
    assert "application: clidemo" in aid
    for _ in range(100):
        st = json.loads(_run(["apps", "status", "clidemo", "--json"], live_worker))
        if st["status"] == "RUNNING":
            break
        import time

        time.sleep(0.2)
    assert st["status"] == "RUNNING"
    sid = st["service_ids"][0]["websocket_service_id"]
    res = json.loads(_run(["call", sid, "reverse_text", "--arg", "text=abc", "--json"], live_worker))
    assert res["reversed"] == "cba"
    assert "demo-app" in _run(["apps", "list"], live_worker)
    assert "cpu" in _run(["cluster", "status"], live_worker)
    _run(["apps", "logs", "clidemo", "--tail", "5"], live_worker)
    assert "stopped clidemo" in _run(["apps", "stop", "clidemo", "--yes"], live_worker)


def test_worker_cli_parser():
    from bioengine_worker_amd.worker.__main__ import create_parser, worker_kwargs

    a = create_parser().parse_args(["--mode", "slurm", "--startup-applications", '{"artifact_id": "demo-app"}',
                                    "--startup-applications", '[{"artifact_id": "x", "disable_gpu": true}]',
                                    "--further-slurm-args", "--partition=gpu --account='a b'", "--max-workers", "3"])
    kw = worker_kwargs(a)
    assert [s["artifact_id"] for s in kw["startup_applications"]] == ["demo-app", "x"]
    assert kw["slurm_config"]["further_slurm_args"] == ["--partition=gpu", "--account=a b"]
    assert kw["slurm_config"]["max_workers"] == 3
    with pytest.raises(SystemExit):
        worker_kwargs(create_parser().parse_args(["--startup-applications", '{"no_id": 1}']))
