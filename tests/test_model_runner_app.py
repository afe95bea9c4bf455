"""model-runner app end-to-end through the worker on CPU (offline counterpart of the reference's
tests/apps/model-runner, which need the public bioimage.io zoo): local zoo package, search, RDF,
documentation, validate, test (cached report), infer whole and tiled."""
import asyncio
from pathlib import Path

import numpy as np
import pytest

from bioengine_worker_amd.bioimageio.package import write_unet2d_package

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.end_to_end
def test_model_runner_e2e(tmp_path, monkeypatch):
    from bioengine_worker_amd.transport import connect_to_server
    from bioengine_worker_amd.transport.hub import get_local_hub, reset_local_hubs
    from bioengine_worker_amd.worker.worker import BioEngineWorker

    zoo = tmp_path / "zoo"
    write_unet2d_package(zoo / "tiny-unet", "tiny-unet", features=(8, 16, 32), test_shape=(1, 1, 96, 96),
                         torchscript=False)
    write_unet2d_package(zoo / "tiny-onnx", "tiny-onnx", features=(8, 16, 32), test_shape=(1, 1, 96, 96),
                         torchscript=False, state_dict=False, onnx=True)  # ONNX-only weights
    monkeypatch.setenv("BIOENGINE_MODEL_ZOO", str(zoo))
    monkeypatch.setenv("BIOENGINE_LOCAL_ARTIFACT_PATH", str(ROOT / "apps"))
    monkeypatch.setenv("BIOENGINE_REPLICA_MODE", "local")
    monkeypatch.setenv("HOME", str(tmp_path / "home"))
    reset_local_hubs()

    async def main():
        hub = get_local_hub("mr")
        await hub.start_http()
        tok = hub.issue_token("admin-user", workspace="ws-admin")
        w = BioEngineWorker(mode="single-machine", workspace_dir=tmp_path / "be", server_url="local://mr", token=tok,
                            client_id="worker1", log_file="off", head_num_cpus=4, head_num_gpus=0,
                            monitoring_interval_seconds=0.5, data_server_url=None)
        await w.start(blocking=False)
        admin = await connect_to_server({"server_url": "local://mr", "token": tok})
        svc = await admin.get_service(w.full_service_id)
        aid = await svc.deploy_app(artifact_id="model-runner", application_id="mr", disable_gpu=True)
        assert await w.apps_manager.wait_for(aid, timeout=240) == "RUNNING", \
            (await svc.get_app_status(application_ids=[aid]))["message"]
        st = await svc.get_app_status(application_ids=[aid])
        assert set(st["deployments"]) == {"EntryDeployment", "RuntimeDeployment"}
        app = await admin.get_service(st["service_ids"][0]["websocket_service_id"])
        found = await app.search_models(keywords=["unet"])
        assert sorted(m["model_id"] for m in found) == ["tiny-onnx", "tiny-unet"]
        rdf = await app.get_model_rdf(model_id="tiny-unet")
        assert rdf["inputs"][0]["id"] == "raw"
        doc = await app.get_model_documentation(model_id="tiny-unet")
        assert doc.startswith("# tiny-unet")
        v = await app.validate(rdf_dict=rdf)
        assert v["success"], v
        bad = dict(rdf)
        bad.pop("inputs")
        assert not (await app.validate(rdf_dict=bad))["success"]
        rep = await app.test(model_id="tiny-unet")
        assert rep["status"] == "passed", rep
        rep2 = await app.test(model_id="tiny-unet")  # served from the cached report
        assert rep2 == rep
        x = np.load(zoo / "tiny-unet" / "test_input.npy")
        out = await app.infer(model_id="tiny-unet", inputs=x)
        ref = np.load(zoo / "tiny-unet" / "test_output.npy")
        assert np.abs(out["probabilities"] - ref).max() < 1e-4
        out2 = await app.infer(model_id="tiny-unet", inputs=x[0, 0, :80, :72], default_blocksize_parameter=0)
        assert out2["probabilities"].shape == (1, 2, 80, 72)
        with pytest.raises(Exception):
            await app.infer(model_id="no-such-model", inputs=x)
        # ONNX-only package: own graph executor (no onnxruntime), test + infer through the app
        assert (await app.test(model_id="tiny-onnx"))["status"] == "passed"
        xo = np.load(zoo / "tiny-onnx" / "test_input.npy")
        outo = await app.infer(model_id="tiny-onnx", inputs=xo, weights_format="onnx")
        assert np.abs(outo["probabilities"] - np.load(zoo / "tiny-onnx" / "test_output.npy")).max() < 1e-4
        await svc.stop_worker(blocking=True)
        await admin.disconnect()

    asyncio.run(asyncio.wait_for(main(), 600))
    reset_local_hubs()
