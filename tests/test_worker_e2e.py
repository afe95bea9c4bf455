"""End-to-end: worker + apps over the hub (offline port of tests/end_to_end/test_worker.py and
test_applications.py from the reference, which require live Hypha + Ray)."""
import asyncio
import os
from pathlib import Path

import pytest

from bioengine_worker_amd.transport import connect_to_server
from bioengine_worker_amd.transport.hub import get_local_hub, reset_local_hubs
from bioengine_worker_amd.utils import create_file_list_from_directory
from bioengine_worker_amd.worker.worker import BioEngineWorker

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture()
def env(tmp_path, monkeypatch):
    monkeypatch.setenv("BIOENGINE_LOCAL_ARTIFACT_PATH", str(ROOT / "apps"))
    monkeypatch.setenv("BIOENGINE_REPLICA_MODE", "local")
    reset_local_hubs()
    yield tmp_path
    reset_local_hubs()


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 120))


async def _start(tmp_path, hubname, **kw):
    hub = get_local_hub(hubname)
    await hub.start_http()
    admin_tok = hub.issue_token("admin-user", email="admin@example.com", workspace="ws-admin")
    w = BioEngineWorker(mode="single-machine", workspace_dir=tmp_path / "be", server_url=f"local://{hubname}",
                        token=admin_tok, client_id="worker1", log_file="off", head_num_cpus=6, head_num_gpus=0,
                        monitoring_interval_seconds=0.2, data_server_url=None, **kw)
    await w.start(blocking=False)
    return hub, admin_tok, w


@pytest.mark.end_to_end
def test_worker_status_and_apps(env):
    async def main():
        hub, admin_tok, w = await _start(env, "e2e1", startup_applications=[
            {"artifact_id": "demo-app", "application_id": "demo", "disable_gpu": True}])
        admin = await connect_to_server({"server_url": "local://e2e1", "token": admin_tok, "client_id": "cli"})
        user_tok = hub.issue_token("bob", workspace="ws-bob")
        user = await connect_to_server({"server_url": "local://e2e1", "token": user_tok})
        svc = await admin.get_service(w.full_service_id)
        st = await svc.get_status()
        for k in ("service_start_time", "service_uptime", "bioengine_version", "ray_version", "worker_mode",
                  "workspace", "client_id", "ray_cluster", "admin_users", "geo_location", "is_ready"):
            assert k in st
        assert st["worker_mode"] == "single-machine" and st["is_ready"]
        rc = st["ray_cluster"]
        assert rc["mode"] == "single-machine" and rc["cluster"]["total_cpu"] == 6 and rc["cluster"]["total_gpu"] == 0
        node = next(iter(rc["nodes"].values()))
        for k in ("node_ip", "head", "total_cpu", "used_cpu", "total_gpu", "used_gpu", "accelerator_type"):
            assert k in node
        assert "admin-user" in st["admin_users"]
        assert await svc.check_access() is True
        usvc = await user.get_service(w.full_service_id)
        assert await usvc.check_access() is False
        with pytest.raises(PermissionError):
            await usvc.deploy_app(artifact_id="demo-app")

        assert await w.apps_manager.wait_for("demo") == "RUNNING"
        s = await svc.get_app_status(application_ids=["demo"])
        assert s["status"] == "RUNNING" and s["deployments"]["DemoDeployment"]["status"] == "HEALTHY"
        assert set(s["available_methods"]) >= {"ping", "reverse_text", "ascii_art", "set_fail_health_check"}
        assert s["gpu_enabled"] is False and s["authorized_users"]["*"] == ["*"]
        sid = s["service_ids"][0]["websocket_service_id"]
        assert sid.startswith("ws-admin/worker1-") and sid.endswith(":demo")
        app = await user.get_service(sid)
        assert (await app.reverse_text(text="abc"))["reversed"] == "cba"
        assert (await app.ping())["status"] == "ok"
        assert (await app.get_model(model_id="m1"))["model"]["model_id"] == "m1"
        assert await app.get_load() >= 0.0

        # composition app with secret env + kwargs
        aid = await svc.deploy_app(artifact_id="bioengine-composition-demo", application_id="comp",
                                   application_env_vars={"RuntimeA": {"_SECRET": "x", "PLAIN": "1"}})
        assert await w.apps_manager.wait_for(aid) == "RUNNING", (await svc.get_app_status(application_ids=[aid]))["message"]
        comp = await admin.get_service((await svc.get_app_status(application_ids=[aid]))["service_ids"][0]["websocket_service_id"])
        out = await comp.process(text="hello world", numbers=[1, 2, 3], delay=0.0)
        assert out["text"]["upper"] == "HELLO WORLD" and out["stats"]["mean"] == 2.0
        # reference composition API (apps/composition-demo/entry_deployment.py:53-131)
        allr = await comp.run_all(text="a b c", values=[2, 4], count=2)
        assert allr["text_result"]["word_count"] == 3 and allr["data_result"]["sum"] == 6.0
        assert len(allr["time_result"]["timestamps"]) == 2
        assert (await comp.analyze_numbers(values=[1, 3]))["mean"] == 2.0
        assert (await comp.process_text(text="ab"))["reversed"] == "ba"
        assert (await comp.time_operations(count=1))["count"] == 1
        assert set((await comp.status())) == {"entry_uptime", "runtime_a", "runtime_b", "runtime_c"}
        cs = await svc.get_app_status(application_ids=[aid])
        assert set(cs["deployments"]) == {"EntryDeployment", "RuntimeA", "RuntimeB", "RuntimeC"}
        assert cs["application_env_vars"]["RuntimeA"] == {"PLAIN": "1", "SECRET": "*****"}
        allst = await svc.get_app_status()
        assert set(allst) == {"demo", "comp"}
        assert (await svc.get_app_status(application_ids=["nope"]))["status"] == "NOT_RUNNING"

        # health-check fault injection -> UNHEALTHY, service deregistered
        await app.set_fail_health_check()
        ds = w.controller.apps["demo"].deployments["DemoDeployment"]
        ds.cfg.health_check_period_s = 0.1
        for _ in range(100):
            await asyncio.sleep(0.05)
            if ds.restarts > 0:
                break
        assert ds.restarts > 0  # unhealthy replica replaced

        await svc.stop_app(application_id="comp")
        assert "comp" not in await svc.get_app_status()
        dirs = await svc.list_app_directories()
        assert any(d["name"] == "demo" and d["is_running"] for d in dirs)
        logs = await svc.get_logs(tail=5)
        assert isinstance(logs, list)
        res = await svc.stop_all_apps()
        assert res == {"demo": True}
        await svc.stop_worker(blocking=True)
        await admin.disconnect()
        await user.disconnect()

    run(main())


@pytest.mark.end_to_end
def test_upload_deploy_from_artifact_and_run_code(env):
    async def main():
        hub, admin_tok, w = await _start(env, "e2e2")
        admin = await connect_to_server({"server_url": "local://e2e2", "token": admin_tok})
        svc = await admin.get_service(w.full_service_id)
        files = create_file_list_from_directory(ROOT / "apps" / "demo-app", _artifact_id_suffix="t1")
        aid = await svc.upload_app(files=files)
        assert aid == "ws-admin/demo-app-t1"
        apps = await svc.list_apps()
        assert aid in apps and "demo_deployment.py" in apps[aid]["files"]
        assert (await svc.get_app_manifest(artifact_id=aid))["id"] == "demo-app-t1"
        os.environ.pop("BIOENGINE_LOCAL_ARTIFACT_PATH", None)
        w.apps_manager.builder.local_artifact_path = None
        app_id = await svc.deploy_app(artifact_id=aid, disable_gpu=True, authorized_users=["carol"])
        assert await w.apps_manager.wait_for(app_id) == "RUNNING"
        st = await svc.get_app_status(application_ids=[app_id])
        assert st["authorized_users"]["*"][0] == "carol" and "admin-user" in st["authorized_users"]["*"]
        assert st["static_site_url"] and "ws_service_id=" in st["static_site_url"]
        # a user not in authorized_users is rejected by the bridge
        tok = hub.issue_token("mallory", workspace="ws-m")
        m = await connect_to_server({"server_url": "local://e2e2", "token": tok})
        s = await m.get_service(st["service_ids"][0]["websocket_service_id"])
        with pytest.raises(PermissionError):
            await s.ping()
        with pytest.raises(ValueError):
            await svc.delete_app(artifact_id=aid)  # still running
        await svc.stop_app(application_id=app_id)
        await svc.delete_app(artifact_id=aid)
        assert aid not in await svc.list_apps()

        lines = []
        r = await svc.run_code(code="def analyze(x, y=1):\n    print('hi', x)\n    return x * y\n", args=[21],
                               kwargs={"y": 2}, write_stdout=lambda s: lines.append(s))
        assert r["result"] == 42 and "hi 21" in r["stdout"] and lines == ["hi 21"]
        r = await svc.run_code(code="def analyze():\n    raise ValueError('bad')\n")
        assert "bad" in r["error"]
        r = await svc.run_code(code="def analyze():\n    import time; time.sleep(10)\n", timeout=0.5)
        assert "timed out" in r["error"]
        import cloudpickle

        def f(a):
            return a + 1

        r = await svc.run_code(func_bytes=cloudpickle.dumps(f), mode="pickle", args=[1])
        assert r["result"] == 2
        await svc.stop_worker(blocking=True)

    run(main())
