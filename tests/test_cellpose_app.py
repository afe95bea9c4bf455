"""Cellpose fine-tuning app end-to-end through the worker, offline (the reference's app tests need a
live Hypha server, Ray and pretrained weights).

* The reference's own offline fixtures (``tests/apps/cellpose/test_metadata_and_glob.py``) run
  unmodified against this app's ``main.py`` when the reference tree is present.
* A dataset artifact with a nested glob layout is created on the in-process hub; ``start_training``
  (reference signature, default model ``cpsam``) pairs, downloads and trains; the session is used
  for inference, restarted from disk, and exported as a committed BioImage.IO model artifact.
* A 2-rank data-parallel session runs as a gang of gloo processes with identical final weights.

Runs on CPU with a tiny Cellpose-SAM encoder; the HIP paths are covered by the GPU tests.
"""
import asyncio
import importlib.util
import inspect
import io
import sys
from pathlib import Path

import numpy as np
import pytest

from bioengine_worker_amd.train.cellpose_train import synthetic_instances
from bioengine_worker_amd.transport import connect_to_server
from bioengine_worker_amd.transport.hub import get_local_hub, reset_local_hubs
from bioengine_worker_amd.worker.worker import BioEngineWorker

ROOT = Path(__file__).resolve().parents[1]
APP_MAIN = ROOT / "apps" / "cellpose-finetuning" / "main.py"
REF_TEST = Path("/root/reference/tests/apps/cellpose/test_metadata_and_glob.py")


def _load_app_module():
    from bioengine_worker_amd.compat import install

    install()
    spec = importlib.util.spec_from_file_location("cellpose_finetuning_main_test", APP_MAIN)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.unit
@pytest.mark.skipif(not REF_TEST.exists(), reason="reference tree not present")
def test_reference_pairing_fixtures_pass(tmp_path):
    """Execute the reference's test module with its ``_main_path`` pointed at this app."""
    from bioengine_worker_amd.compat import install

    install()
    src = REF_TEST.read_text()
    src = src.replace('Path(__file__).parents[3] / "apps" / "cellpose-finetuning" / "main.py"', repr(str(APP_MAIN)))
    ns = {"__name__": "ref_cellpose_pairing", "__file__": str(REF_TEST)}
    exec(compile(src, str(REF_TEST), "exec"), ns)  # noqa: S102 - test fixture code, no I/O beyond tmp_path
    tests = [(k, v) for k, v in ns.items() if k.startswith("test_") and callable(v)]
    assert len(tests) >= 5
    for i, (name, fn) in enumerate(tests):
        kw = {"tmp_path": tmp_path / str(i)} if "tmp_path" in inspect.signature(fn).parameters else {}
        if kw:
            kw["tmp_path"].mkdir()
        fn(**kw)


@pytest.mark.unit
def test_pairing_semantics(tmp_path):
    m = _load_app_module()
    pairs = m.match_image_annotation_pairs(["img/a/x1.tif", "img/b/x2.tif", "img/c/z.tif"],
                                           ["ann/a/x1_mask.tif", "ann/b/x2_mask.tif"], "img/*/*.tif",
                                           "ann/*/*_mask.tif")
    assert pairs == [("img/a/x1.tif", "ann/a/x1_mask.tif"), ("img/b/x2.tif", "ann/b/x2_mask.tif")]
    # mixed conventions fall back to base-name keys
    assert m.match_image_annotation_pairs(["i/q.tif"], ["a/q-label.png"], "i/*.tif", "a/*_mask.ome.tif") == \
        [("i/q.tif", "a/q-label.png")]
    # colab RGB annotation: 16-bit ids over R (high) and G (low) with B == 0
    from bioengine_worker_amd.cellpose.datasets import decode_labels

    rgb = np.zeros((2, 2, 3), np.uint8)
    rgb[0, 0] = (1, 2, 0)
    assert decode_labels(rgb)[0, 0] == 258
    rgb[1, 1, 2] = 5
    assert decode_labels(rgb)[0, 0] == 1  # B != 0 -> R channel


def _tif(arr) -> bytes:
    from PIL import Image

    buf = io.BytesIO()
    Image.fromarray(arr).save(buf, format="TIFF")
    return buf.getvalue()


@pytest.fixture()
def env(tmp_path, monkeypatch):
    monkeypatch.setenv("BIOENGINE_LOCAL_ARTIFACT_PATH", str(ROOT / "apps"))
    monkeypatch.setenv("BIOENGINE_REPLICA_MODE", "local")
    monkeypatch.setenv("HOME", str(tmp_path / "home"))
    reset_local_hubs()
    yield tmp_path
    reset_local_hubs()


async def _wait_status(app, sid, done=("completed", "failed", "stopped"), timeout=300):
    st = None
    for _ in range(int(timeout / 0.25)):
        st = await app.get_training_status(session_id=sid)
        if st["status_type"] in done:
            return st
        await asyncio.sleep(0.25)
    raise TimeoutError(st)


async def _dataset(hub, ctx):
    """Artifact with images/<plate>/<name>.tif + annotations/<plate>/<name>_mask.tif (+ test split)."""
    import httpx

    am = hub.artifacts
    await am.create(type="dataset", alias="cells", stage=True, context=ctx)
    ims, labs = synthetic_instances(5, 96, 112, ncells=12, seed=3)
    files = {}
    for i in range(4):
        files[f"images/p{i % 2}/t{i:03d}.tif"] = _tif((ims[i, 0] * 1000 + 200).astype(np.uint16))
        files[f"annotations/p{i % 2}/t{i:03d}_mask.tif"] = _tif(labs[i].astype(np.uint16))
    files["test/images/t100.tif"] = _tif((ims[4, 0] * 1000 + 200).astype(np.uint16))
    files["test/masks/t100_mask.tif"] = _tif(labs[4].astype(np.uint16))
    async with httpx.AsyncClient() as c:
        for path, data in files.items():
            r = await c.put(await am.put_file("ws-admin/cells", path, context=ctx), content=data)
            r.raise_for_status()
    await am.commit("ws-admin/cells", context=ctx)
    await am.create(type="collection", alias="models", config={"permissions": {"*": "r"}}, context=ctx)
    return labs


@pytest.mark.end_to_end
@pytest.mark.timeout(900)
def test_cellpose_app_cpsam_train_restart_export(env):
    async def main():
        hub = get_local_hub("cpapp")
        await hub.start_http()
        tok = hub.issue_token("admin-user", workspace="ws-admin")
        ctx = {"user": {"id": "admin-user"}, "ws": "ws-admin"}
        labs = await _dataset(hub, ctx)
        w = BioEngineWorker(mode="single-machine", workspace_dir=env / "be", server_url="local://cpapp", token=tok,
                            client_id="worker1", log_file="off", head_num_cpus=8, head_num_gpus=0,
                            monitoring_interval_seconds=0.5, data_server_url=None)
        await w.start(blocking=False)
        admin = await connect_to_server({"server_url": "local://cpapp", "token": tok})
        svc = await admin.get_service(w.full_service_id)
        aid = await svc.deploy_app(artifact_id="cellpose-finetuning", application_id="cp", disable_gpu=True, hypha_token=tok,
                                   application_kwargs={"CellposeFinetune": {"cpsam_arch": "tiny"}})
        st = await w.apps_manager.wait_for(aid, timeout=300)
        assert st == "RUNNING", (await svc.get_app_status(application_ids=[aid]))["message"]
        s = await svc.get_app_status(application_ids=[aid])
        assert {"infer", "start_training", "restart_training", "export_model"} <= set(s["available_methods"])
        app = await admin.get_service(s["service_ids"][0]["websocket_service_id"])

        # default model is cpsam; random weights are reported
        img = np.random.default_rng(0).integers(0, 4000, (80, 90), dtype=np.uint16)
        out = await app.infer(input_arrays=[img])
        assert out[0]["output"].shape == (80, 90) and out[0].get("weights") == "random"
        js = await app.infer(input_arrays=[img], json_safe=True, return_flows=True)
        assert js[0]["output"]["encoding"] == "mask_png_base64" and len(js[0]["flows"]) == 3

        # reference contract: glob strings over the artifact, test split, cpsam default
        r = await app.start_training(artifact="ws-admin/cells", train_images="images/*/*.tif",
                                     train_annotations="annotations/*/*_mask.tif", test_images="test/images/",
                                     test_annotations="test/masks/*_mask.tif", n_epochs=2, min_train_masks=1,
                                     learning_rate=1e-4, validation_interval=1, label="unit")
        sid = r["session_id"]
        st = await _wait_status(app, sid)
        assert st["status_type"] == "completed", st
        assert st["n_train"] == 4 and st["n_test"] == 1 and st["model"] == "cpsam"
        assert len(st["train_losses"]) == 2 and all(np.isfinite(st["train_losses"]))
        im = st["instance_metrics"]
        assert set(im) == {"ap_0_5", "ap_0_75", "ap_0_9", "n_true", "n_pred"} and im["n_true"] == int(labs[4].max())
        assert sid in await app.list_training_sessions(labels=["unit"])
        out = await app.infer(input_arrays=[img], model=sid)
        assert out[0]["output"].shape == (80, 90) and "weights" not in out[0]

        # restart reads everything back from disk (no in-memory cache) and inherits the loss history
        r2 = await app.restart_training(session_id=sid, n_epochs=1)
        st2 = await _wait_status(app, r2["session_id"])
        assert st2["status_type"] == "completed", st2
        assert st2["continued_from"] == sid and r2["restarted_from"] == sid and len(st2["train_losses"]) == 3

        # export: created, uploaded and committed into the collection
        ex = await app.export_model(session_id=sid, model_name="unit-cpsam", collection="ws-admin/models",
                                    authors=[{"name": "Tester"}])
        assert ex["status"] == "exported" and ex["artifact_id"] == "ws-admin/unit-cpsam"
        art = await hub.artifacts.read("ws-admin/unit-cpsam", context=ctx)
        assert art["manifest"]["type"] == "model" and art["parent_id"] == "ws-admin/models"
        names = {f["name"] for f in await hub.artifacts.list_files("ws-admin/unit-cpsam", context=ctx)}
        assert {"rdf.yaml", "model_weights.pth", "model.py", "input_sample.npy", "cover.png"} <= names
        found = await app.list_models_by_dataset(dataset_id="ws-admin/cells", collection="ws-admin/models")
        assert [f["id"] for f in found] == ["ws-admin/unit-cpsam"]
        # the exported artifact is itself a valid model reference
        out = await app.infer(input_arrays=[img], model="ws-admin/unit-cpsam")
        assert out[0]["output"].shape == (80, 90)

        # data-parallel: 2 gloo ranks (gang of processes), weights identical on both ranks
        r3 = await app.start_training(artifact="ws-admin/cells", train_images="images/*/*.tif",
                                      train_annotations="annotations/*/*_mask.tif", n_epochs=1, min_train_masks=1,
                                      learning_rate=1e-4, n_gpus=2)
        st3 = await _wait_status(app, r3["session_id"])
        assert st3["status_type"] == "completed", st3
        for _ in range(200):  # the launcher records the per-rank digests once the gang has exited
            if "rank_weight_digests" in st3:
                break
            await asyncio.sleep(0.1)
            st3 = await app.get_training_status(session_id=r3["session_id"])
        d = st3["rank_weight_digests"]
        assert len(d) == 2 and d[0] == d[1] == st3["weights_sha256"]
        assert st3["world_size"] == 2

        assert (await app.delete_training_session(session_id=r2["session_id"]))["deleted"] == r2["session_id"]
        with pytest.raises(Exception):
            await app.get_training_status(session_id=r2["session_id"])
        await svc.stop_worker(blocking=True)
        await admin.disconnect()
        await hub.stop_http()

    asyncio.run(asyncio.wait_for(main(), 840))
