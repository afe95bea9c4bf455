"""model-runner runtime behaviour beyond the reference's one-request replica
(reference apps/model-runner/runtime_deployment.py:40,101-156,234-312), on CPU through the worker:

* the replica's event loop keeps answering (runtime health check + cached test report) while a
  long prediction runs -- ``predict`` runs its GPU work on a worker thread;
* concurrent same-model requests are served by ``@serve.batch`` with shared forwards
  (``PredictionPipeline.predict_many``), and every request still gets its own exact result;
* ``test(additional_requirements=[...])`` installs the extra wheel from the local wheelhouse and runs
  the package test in an isolated task; without the wheelhouse the call fails naming the
  requirement; without the requirement the package's own import fails the test.
"""
import asyncio
import threading
import time
from pathlib import Path

import numpy as np
import pytest
import yaml

from bioengine_worker_amd.bioimageio.package import write_unet2d_package
from bioengine_worker_amd.bioimageio.spec import sha256_file

ROOT = Path(__file__).resolve().parents[1]


def _needs_dep_package(root: Path) -> Path:
    """A U-Net package whose architecture module imports ``bioengine_testdep``."""
    d = root / "needs-dep"
    write_unet2d_package(d, "needs-dep", features=(8, 16), test_shape=(1, 1, 64, 64), torchscript=False)
    src = d / "model.py"
    src.write_text("import bioengine_testdep  # noqa: F401  (extra requirement of this package)\n" + src.read_text())
    rdf = yaml.safe_load((d / "rdf.yaml").read_text())
    rdf["weights"]["pytorch_state_dict"]["architecture"]["sha256"] = sha256_file(src)
    (d / "rdf.yaml").write_text(yaml.safe_dump(rdf, sort_keys=False))
    return d


@pytest.mark.end_to_end
def test_model_runner_runtime_batching_health_and_requirements(tmp_path, monkeypatch, wheelhouse):
    from bioengine_worker_amd.bioimageio.runner import PredictionPipeline
    from bioengine_worker_amd.transport import connect_to_server
    from bioengine_worker_amd.transport.hub import get_local_hub, reset_local_hubs
    from bioengine_worker_amd.worker.worker import BioEngineWorker

    zoo = tmp_path / "zoo"
    write_unet2d_package(zoo / "tiny-unet", "tiny-unet", features=(8, 16, 32), test_shape=(1, 1, 96, 96),
                         torchscript=False)
    _needs_dep_package(zoo)
    monkeypatch.setenv("BIOENGINE_MODEL_ZOO", str(zoo))
    monkeypatch.setenv("BIOENGINE_LOCAL_ARTIFACT_PATH", str(ROOT / "apps"))
    monkeypatch.setenv("BIOENGINE_REPLICA_MODE", "local")  # in-process replicas: the patch below applies
    monkeypatch.setenv("HOME", str(tmp_path / "home"))
    monkeypatch.setenv("BIOENGINE_ENV_CACHE", str(tmp_path / "envs"))
    monkeypatch.setenv("BIOENGINE_WHEELHOUSE", "")
    reset_local_hubs()

    slow = {"on": False, "batches": []}
    fwd = PredictionPipeline._forward

    def slow_forward(self, xs):
        if slow["on"]:
            assert threading.current_thread() is not threading.main_thread()  # never on the event loop
            slow["batches"].append(int(xs[0].shape[0]))
            time.sleep(0.6)
        return fwd(self, xs)

    monkeypatch.setattr(PredictionPipeline, "_forward", slow_forward)

    async def main():
        hub = get_local_hub("mrt")
        await hub.start_http()
        tok = hub.issue_token("admin-user", workspace="ws-admin")
        w = BioEngineWorker(mode="single-machine", workspace_dir=tmp_path / "be", server_url="local://mrt", token=tok,
                            client_id="worker1", log_file="off", head_num_cpus=4, head_num_gpus=0,
                            monitoring_interval_seconds=0.5, data_server_url=None)
        await w.start(blocking=False)
        admin = await connect_to_server({"server_url": "local://mrt", "token": tok})
        svc = await admin.get_service(w.full_service_id)
        aid = await svc.deploy_app(artifact_id="model-runner", application_id="mrt", disable_gpu=True)
        assert await w.apps_manager.wait_for(aid, timeout=240) == "RUNNING", \
            (await svc.get_app_status(application_ids=[aid]))["message"]
        st = await svc.get_app_status(application_ids=[aid])
        app = await admin.get_service(st["service_ids"][0]["websocket_service_id"])

        x = np.load(zoo / "tiny-unet" / "test_input.npy")
        ref = np.load(zoo / "tiny-unet" / "test_output.npy")
        assert (await app.test(model_id="tiny-unet"))["status"] == "passed"  # report cached from here on
        await app.infer(model_id="tiny-unet", inputs=x)  # pipeline loaded

        # ---- concurrent same-model requests while the device is busy: batched, loop stays live
        slow["on"] = True
        scales = [1.0, 0.5, 2.0, 1.5]
        t0 = time.perf_counter()
        reqs = [asyncio.ensure_future(app.infer(model_id="tiny-unet", inputs=(x * s).astype(x.dtype)))
                for s in scales]
        await asyncio.sleep(0.15)
        t = time.perf_counter()
        rep = await app.test(model_id="tiny-unet")  # runtime check_health + cached report
        health_s = time.perf_counter() - t
        outs = await asyncio.gather(*reqs)
        total_s = time.perf_counter() - t0
        slow["on"] = False
        assert rep["status"] == "passed"
        assert health_s < 0.4 < total_s, (health_s, total_s)
        assert sum(slow["batches"]) == 4 and max(slow["batches"]) >= 2 and len(slow["batches"]) < 4, slow["batches"]
        np.testing.assert_allclose(outs[0]["probabilities"], ref, atol=1e-4)
        for s, o in zip(scales, outs):  # batched forwards return each request's own result
            solo = await app.infer(model_id="tiny-unet", inputs=(x * s).astype(x.dtype))
            np.testing.assert_allclose(o["probabilities"], solo["probabilities"], atol=1e-5)

        # ---- additional_requirements: isolated test task with a wheelhouse-installed extra package
        plain = await app.test(model_id="needs-dep")  # the package's own import fails without it
        assert plain["status"] == "failed"
        # no wheelhouse: unsatisfiable.  As upstream (entry_deployment.py:1651-1701) a test run that
        # raises yields a failed fallback report carrying the traceback, not an exception
        bad = await app.test(model_id="needs-dep", additional_requirements=["bioengine-testdep==0.1.0"], skip_cache=True)
        assert bad["status"] == "failed" and "bioengine-testdep" in str(bad["details"]), bad
        assert "tested_at" in bad and any(r[0] == "bioengine" for r in bad["env"])
        monkeypatch.setenv("BIOENGINE_WHEELHOUSE", str(wheelhouse))
        rep = await app.test(model_id="needs-dep", additional_requirements=["bioengine-testdep==0.1.0"],
                             skip_cache=True)
        assert rep["status"] == "passed", rep
        assert rep["additional_requirements"] == ["bioengine-testdep==0.1.0"]
        assert any((tmp_path / "envs").glob("*/bioengine_testdep.py"))
        await svc.stop_worker(blocking=True)
        await admin.disconnect()

    asyncio.run(asyncio.wait_for(main(), 600))
    reset_local_hubs()
