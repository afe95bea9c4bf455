"""Cellpose fine-tuning app end-to-end through the worker (offline counterpart of the reference's
apps/cellpose-finetuning tests, which need a live Hypha server + Ray + pretrained weights).

Runs on CPU: the app's inference path falls back to the PyTorch reference ops and the trainer's
CPU paths; the GPU variant (HIP kernels) is exercised by ``test_cellpose_gpu.py``.
"""
import asyncio
from pathlib import Path

import numpy as np
import pytest

from bioengine_worker_amd.cellpose.pipeline import synthetic_cells
from bioengine_worker_amd.train.cellpose_train import synthetic_instances
from bioengine_worker_amd.transport import connect_to_server
from bioengine_worker_amd.transport.hub import get_local_hub, reset_local_hubs
from bioengine_worker_amd.worker.worker import BioEngineWorker

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture()
def env(tmp_path, monkeypatch):
    monkeypatch.setenv("BIOENGINE_LOCAL_ARTIFACT_PATH", str(ROOT / "apps"))
    monkeypatch.setenv("BIOENGINE_REPLICA_MODE", "local")
    monkeypatch.setenv("HOME", str(tmp_path / "home"))
    reset_local_hubs()
    yield tmp_path
    reset_local_hubs()


async def _wait_status(app, sid, done=("completed", "failed", "stopped"), timeout=240):
    for _ in range(int(timeout / 0.25)):
        st = await app.get_training_status(session_id=sid)
        if st["status_type"] in done:
            return st
        await asyncio.sleep(0.25)
    raise TimeoutError(st)


@pytest.mark.end_to_end
def test_cellpose_app_infer_train_restart_export(env):
    async def main():
        hub = get_local_hub("cpapp")
        await hub.start_http()
        tok = hub.issue_token("admin-user", workspace="ws-admin")
        w = BioEngineWorker(mode="single-machine", workspace_dir=env / "be", server_url="local://cpapp", token=tok,
                            client_id="worker1", log_file="off", head_num_cpus=4, head_num_gpus=0,
                            monitoring_interval_seconds=0.5, data_server_url=None)
        await w.start(blocking=False)
        admin = await connect_to_server({"server_url": "local://cpapp", "token": tok})
        svc = await admin.get_service(w.full_service_id)
        aid = await svc.deploy_app(artifact_id="cellpose-finetuning", application_id="cp", disable_gpu=True)
        st = await w.apps_manager.wait_for(aid, timeout=240)
        assert st == "RUNNING", (await svc.get_app_status(application_ids=[aid]))["message"]
        s = await svc.get_app_status(application_ids=[aid])
        assert {"infer", "start_training", "get_training_status", "export_model"} <= set(s["available_methods"])
        app = await admin.get_service(s["service_ids"][0]["websocket_service_id"])

        # inference: two concurrent requests share one continuous batch
        imgs = synthetic_cells(2, 96, 96, ncells=6)
        outs = await asyncio.gather(app.infer(input_arrays=[imgs[0]]),
                                    app.infer(input_arrays=[imgs[1]], return_flows=True))
        assert outs[0][0]["output"].shape == (96, 96) and outs[0][0]["output"].dtype == np.int32
        assert outs[1][0]["flows"].shape[-2:] == (96, 96)
        js = await app.infer(input_arrays=[imgs[0][0]], json_safe=True)
        assert isinstance(js[0]["output"], str)

        # fine-tuning on arrays (2 epochs), validation metrics, checkpoint
        ims, labs = synthetic_instances(3, 128, 128, seed=1)
        r = await app.start_training(train_arrays=[i for i in ims], label_arrays=[l for l in labs], n_epochs=2,
                                     batch_size=2, min_train_masks=1, learning_rate=1e-4, validation_interval=1,
                                     label="unit", test_arrays=[ims[0]], test_label_arrays=[labs[0]])
        sid = r["session_id"]
        st = await _wait_status(app, sid)
        assert st["status_type"] == "completed", st
        assert len(st["train_losses"]) == 2 and all(np.isfinite(st["train_losses"]))
        im = st["instance_metrics"]  # reference InstanceMetrics: AP@0.5/0.75/0.9 + label counts
        assert set(im) == {"ap_0_5", "ap_0_75", "ap_0_9", "n_true", "n_pred"} and im["n_true"] == int(labs[0].max())
        sessions = await app.list_training_sessions(labels=["unit"])
        assert sid in sessions

        # the trained session is usable as an inference model
        out = await app.infer(input_arrays=[imgs[0]], model=sid)
        assert out[0]["output"].shape == (96, 96)

        # continue the session for one more epoch from its exact optimizer state
        r2 = await app.restart_training(session_id=sid, n_epochs=3)
        st2 = await _wait_status(app, r2["session_id"])
        assert st2["status_type"] == "completed", st2
        assert st2["continued_from"] == sid and len(st2["train_losses"]) >= 3

        ex = await app.export_model(session_id=sid, model_name="unit-model")
        assert {"rdf.yaml", "weights.pt"} <= set(ex["files"])
        assert (await app.delete_training_session(session_id=r2["session_id"]))["deleted"] == r2["session_id"]
        with pytest.raises(Exception):
            await app.get_training_status(session_id=r2["session_id"])
        await svc.stop_worker(blocking=True)
        await admin.disconnect()

    asyncio.run(asyncio.wait_for(main(), 600))
