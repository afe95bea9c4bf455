"""App dependency handling (reference ``bioengine/utils/requirements.py``, ``apps/builder.py:300-517``):
pinning, resolution against the installed environment, offline install from a local wheelhouse
into the app's ``site-packages``, and ``DEPLOY_FAILED`` naming what cannot be satisfied.

The wheel is built here from a two-line package with ``pip wheel --no-index`` (no network)."""
import asyncio
import sys
from pathlib import Path

import pytest

from bioengine_worker_amd.apps import requirements as rq
from bioengine_worker_amd.transport import connect_to_server
from bioengine_worker_amd.transport.hub import get_local_hub, reset_local_hubs
from bioengine_worker_amd.worker.worker import BioEngineWorker

MANIFEST = """name: {name}
id: {id}
id_emoji: "x"
description: dependency handling test app
type: ray-serve
format_version: 0.5.0
version: 1.0.0
authors: [{{name: test}}]
license: MIT
deployments:
  - dep:DepApp
"""

DEPLOYMENT = '''
from hypha_rpc.utils.schema import schema_method
from ray import serve


@serve.deployment(ray_actor_options={{"num_cpus": 1, "runtime_env": {{"pip": {pip!r}}}}})
class DepApp:
    @schema_method
    async def value(self) -> str:
        """Value exported by the wheel-installed package."""
        import bioengine_testdep

        return bioengine_testdep.VALUE
'''


@pytest.mark.unit
def test_pinning_and_resolution():
    assert rq.normalize_requirement("numpy>=1.21.0") == "numpy==1.21.0"
    assert rq.normalize_requirement("pydantic~=2.12.0") == "pydantic==2.12.0"
    pinned = rq.update_requirements(["numpy>=1.0", "httpx==0.0.1"])
    names = [rq._name(r) for r in pinned]
    assert names.count("httpx") == 1 and "pydantic" in names  # existing entries win, worker pins added
    assert not any(n == "hypha-rpc" for n in names)  # provided by the framework's shim
    ok, missing = rq.resolve(["numpy", "numpy<0.1", "definitely-not-a-package==1.0", "ray[serve]==2.0",
                              "some-win-only==1; sys_platform == 'win32'"])
    assert ok == ["numpy", "ray[serve]==2.0", "some-win-only==1; sys_platform == 'win32'"]
    assert [m[0] for m in missing] == ["numpy<0.1", "definitely-not-a-package==1.0"]
    assert "does not satisfy" in missing[0][1] and missing[1][1] == "not installed"


@pytest.mark.unit
def test_ensure_installs_from_wheelhouse_or_fails(tmp_path, wheelhouse):
    target = tmp_path / "site-packages"
    with pytest.raises(rq.MissingRequirementsError, match="bioengine-testdep.*no wheelhouse configured"):
        rq.ensure(["bioengine-testdep==0.1.0"], target, wheel_dirs=[])
    info = rq.ensure(["bioengine-testdep==0.1.0"], target, wheel_dirs=[str(wheelhouse)])
    assert info["installed"] == ["bioengine-testdep==0.1.0"] and (target / "bioengine_testdep.py").exists()
    # already satisfied from the target: nothing installed the second time
    assert rq.ensure(["bioengine-testdep==0.1.0"], target, wheel_dirs=[str(wheelhouse)])["installed"] == []
    with pytest.raises(rq.MissingRequirementsError, match="bioengine-testdep==9.9"):
        rq.ensure(["bioengine-testdep==9.9"], tmp_path / "other", wheel_dirs=[str(wheelhouse)])


def _write_app(root: Path, app_id: str, pip: list[str]):
    d = root / app_id
    d.mkdir(parents=True)
    (d / "manifest.yaml").write_text(MANIFEST.format(name=app_id, id=app_id))
    (d / "dep.py").write_text(DEPLOYMENT.format(pip=pip))


@pytest.mark.end_to_end
@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["local", "process"])
def test_deploy_installs_requirements_or_reports_deploy_failed(tmp_path, monkeypatch, wheelhouse, mode):
    apps = tmp_path / "apps"
    _write_app(apps, "needs-wheel", ["bioengine-testdep==0.1.0"])
    _write_app(apps, "needs-missing", ["bioengine-testdep==0.1.0", "definitely-not-a-package>=1.0"])
    monkeypatch.setenv("BIOENGINE_LOCAL_ARTIFACT_PATH", str(apps))
    monkeypatch.setenv("BIOENGINE_WHEELHOUSE", str(wheelhouse))
    monkeypatch.setenv("BIOENGINE_REPLICA_MODE", mode)
    monkeypatch.setenv("HOME", str(tmp_path / "home"))
    reset_local_hubs()

    async def main():
        hub = get_local_hub("reqs")
        tok = hub.issue_token("admin-user", workspace="ws-admin")
        w = BioEngineWorker(mode="single-machine", workspace_dir=tmp_path / "be", server_url="local://reqs", token=tok,
                            client_id="worker1", log_file="off", head_num_cpus=4, head_num_gpus=0,
                            monitoring_interval_seconds=0.5, data_server_url=None)
        await w.start(blocking=False)
        admin = await connect_to_server({"server_url": "local://reqs", "token": tok})
        svc = await admin.get_service(w.full_service_id)
        ok_id = await svc.deploy_app(artifact_id="needs-wheel", application_id="needs-wheel", disable_gpu=True)
        bad_id = await svc.deploy_app(artifact_id="needs-missing", application_id="needs-missing", disable_gpu=True)
        assert await w.apps_manager.wait_for(ok_id, timeout=240) == "RUNNING", \
            (await svc.get_app_status(application_ids=[ok_id]))["message"]
        s = await svc.get_app_status(application_ids=[ok_id])
        app = await admin.get_service(s["service_ids"][0]["websocket_service_id"])
        assert await app.value() == "wheel-ok"
        pip = w.apps_manager.apps[ok_id]["pip"]  # installed into the app's own site-packages
        assert pip["installed"] == ["bioengine-testdep==0.1.0"] and pip["target"].endswith("needs-wheel/site-packages")
        assert (Path(pip["target"]) / "bioengine_testdep.py").exists()
        assert await w.apps_manager.wait_for(bad_id, timeout=240) == "DEPLOY_FAILED"
        msg = (await svc.get_app_status(application_ids=[bad_id]))["message"]
        assert "definitely-not-a-package" in msg and "Missing pip requirements" in msg
        await svc.stop_worker(blocking=True)
        await admin.disconnect()

    asyncio.run(asyncio.wait_for(main(), 280))
    reset_local_hubs()


def test_code_executor_runtime_env_pip(tmp_path, monkeypatch, wheelhouse):
    """run_code honours remote_options.runtime_env.pip: installed from the wheelhouse into a shared
    per-set directory on the child's PYTHONPATH, or a clear error naming what is missing."""
    from bioengine_worker_amd.worker.code_executor import CodeExecutor

    monkeypatch.setenv("BIOENGINE_ENV_CACHE", str(tmp_path / "envs"))
    ex = CodeExecutor(admin_users=["admin"])
    ctx = {"user": {"id": "admin", "email": "admin"}}
    code = "def analyze():\n    import bioengine_testdep\n    return bioengine_testdep.VALUE\n"

    async def run(pip):
        return await ex.run_code(code=code, function_name="analyze", mode="source", args=None, kwargs=None,
                                 remote_options={"runtime_env": {"pip": pip}}, write_stdout=None, write_stderr=None,
                                 timeout=120, context=ctx)

    monkeypatch.setenv("BIOENGINE_WHEELHOUSE", str(wheelhouse))
    out = asyncio.run(run(["bioengine-testdep==0.1.0"]))
    assert out.get("result") == "wheel-ok", out
    assert list((tmp_path / "envs").iterdir())  # the shared install directory
    bad = asyncio.run(run(["bioengine-testdep-missing"]))
    assert "bioengine-testdep-missing" in bad["error"]


def test_isolated_task_runtime_env_pip(tmp_path, monkeypatch, wheelhouse):
    from bioengine_worker_amd.serve import tasks

    monkeypatch.setenv("BIOENGINE_ENV_CACHE", str(tmp_path / "envs"))
    monkeypatch.setenv("BIOENGINE_WHEELHOUSE", str(wheelhouse))

    def value():
        import bioengine_testdep

        return bioengine_testdep.VALUE

    ref = tasks.remote(runtime_env={"pip": ["bioengine-testdep==0.1.0"]})(value).remote()
    assert tasks.get(ref, timeout=120) == "wheel-ok"
    ref = tasks.remote(runtime_env={"pip": ["bioengine-testdep-missing"]})(value).remote()
    with pytest.raises(Exception, match="bioengine-testdep-missing"):
        tasks.get(ref, timeout=120)
