"""EM mitochondria app through the worker (CPU, small U-Net): analyze + analyze_volume."""
import asyncio
import base64
import io
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.end_to_end
def test_em_app_e2e(tmp_path, monkeypatch):
    from bioengine_worker_amd.transport import connect_to_server
    from bioengine_worker_amd.transport.hub import get_local_hub, reset_local_hubs
    from bioengine_worker_amd.worker.worker import BioEngineWorker

    monkeypatch.setenv("BIOENGINE_LOCAL_ARTIFACT_PATH", str(ROOT / "apps"))
    monkeypatch.setenv("BIOENGINE_REPLICA_MODE", "local")
    monkeypatch.setenv("HOME", str(tmp_path / "home"))
    monkeypatch.delenv("BIOENGINE_MODEL_ZOO", raising=False)
    monkeypatch.setenv("BIOENGINE_EM_DATA_ROOT", str(tmp_path / "emdata"))
    reset_local_hubs()

    async def main():
        hub = get_local_hub("em")
        await hub.start_http()
        tok = hub.issue_token("admin-user", workspace="ws-admin")
        w = BioEngineWorker(mode="single-machine", workspace_dir=tmp_path / "be", server_url="local://em", token=tok,
                            client_id="worker1", log_file="off", head_num_cpus=8, head_num_gpus=0,
                            monitoring_interval_seconds=0.5, data_server_url=None)
        await w.start(blocking=False)
        admin = await connect_to_server({"server_url": "local://em", "token": tok})
        svc = await admin.get_service(w.full_service_id)
        aid = await svc.deploy_app(artifact_id="em-mito-analyzer", application_id="em", disable_gpu=True,
                                   application_kwargs={"MitoAnalysisDeployment": {"features": [8, 16, 32]}})
        assert await w.apps_manager.wait_for(aid, timeout=240) == "RUNNING", \
            (await svc.get_app_status(application_ids=[aid]))["message"]
        st = await svc.get_app_status(application_ids=[aid])
        app = await admin.get_service(st["service_ids"][0]["websocket_service_id"])
        assert (await app.ping())["status"] == "ok"
        rng = np.random.default_rng(0)
        img = (rng.random((300, 340)) * 255).astype(np.uint8)
        r = await app.analyze(image=img.tolist(), pixel_size_nm=4.0, tile_size=128, overlap=32)
        assert r["image_shape"] == [300, 340] and len(r["labels"]) == 300
        assert set(r["properties"]) >= {"label", "area_um2", "aspect_ratio", "eccentricity", "centroid_y", "centroid_x"}
        assert r["n_mitochondria"] == len(r["properties"]["label"])
        buf = io.BytesIO()
        np.save(buf, (rng.random((4, 96, 96)) * 255).astype(np.uint8))
        rv = await app.analyze_volume(volume_npy_b64=base64.b64encode(buf.getvalue()).decode(), tile_size=64, overlap=16)
        assert rv["volume_shape"] == [4, 96, 96] and "instances" in rv
        # z-slab sharded over a gang of 2 / 3 ranks (gloo here, RCCL on GPUs): identical labels + stats
        blobs = np.zeros((9, 64, 64), np.float32)
        zz, yy, xx = np.mgrid[0:9, 0:64, 0:64]
        for cz, cy, cx in ((2, 20, 20), (4, 40, 45), (7, 15, 50), (6, 50, 12)):
            blobs += np.exp(-((zz - cz) ** 2 / 4 + (yy - cy) ** 2 / 30 + (xx - cx) ** 2 / 30))
        buf = io.BytesIO()
        np.save(buf, (blobs / blobs.max() * 255).astype(np.uint8))
        b64 = base64.b64encode(buf.getvalue()).decode()
        thr = 0.5
        one = await app.analyze_volume(volume_npy_b64=b64, tile_size=64, overlap=16, return_labels=True,
                                       input_is_probability=True)
        l1 = np.load(io.BytesIO(base64.b64decode(one["labels_npy_b64"])))
        assert l1.max() == 4 and one["n_components"] == 4
        for n in (2, 3):
            rn = await app.analyze_volume(volume_npy_b64=b64, tile_size=64, overlap=16, n_gpus=n, gather="rank0",
                                          return_labels=True, threshold=float(thr),
                                          input_is_probability=True)
            ln = np.load(io.BytesIO(base64.b64decode(rn["labels_npy_b64"])))
            assert np.array_equal(ln, l1), n
            assert rn["n_instances"] == one["n_instances"] and rn["instances"] == one["instances"]
            assert [r["z_range"] for r in rn["ranks"]][-1][1] == 9
        rs = await app.analyze_volume(volume_npy_b64=b64, tile_size=64, overlap=16, n_gpus=2, gather="sharded",
                                      threshold=float(thr), input_is_probability=True)
        parts = [np.load(f) for f in rs["label_shards"]["files"]]
        assert np.array_equal(np.concatenate(parts), l1)
        # volumes referenced by path (each rank reads only its slab): .npy memmap and local zarr,
        # touching objects split by the sharded 3-D watershed == the single-process split
        from bioengine_worker_amd.datasets.store import write_zarr_array

        data = tmp_path / "emdata"
        data.mkdir()
        zz, yy, xx = np.mgrid[0:40, 0:48, 0:48]
        touching = np.zeros((40, 48, 48), np.float32)
        for c in ((12, 20, 20), (21, 20, 22), (28, 30, 30), (20, 34, 12)):
            touching = np.maximum(touching, (((zz - c[0]) ** 2 + (yy - c[1]) ** 2 + (xx - c[2]) ** 2) < 36).astype(np.float32))
        np.save(data / "vol.npy", (touching * 255).astype(np.uint8))
        write_zarr_array(str(data / "vol.zarr"), (touching * 255).astype(np.uint8), chunks=(8, 24, 24))
        kw = dict(tile_size=64, overlap=16, input_is_probability=True, split_touching=True, closing_radius=1,
                  min_distance=3, min_voxels=20, return_labels=True)
        ref = await app.analyze_volume(volume_path="vol.npy", **kw)
        lref = np.load(io.BytesIO(base64.b64decode(ref["labels_npy_b64"])))
        assert ref["split_touching"] and ref["n_components"] >= 4  # the touching pair became two
        for src in ("vol.npy", "vol.zarr"):
            r2 = await app.analyze_volume(volume_path=src, n_gpus=2, gather="rank0", **kw)
            l2 = np.load(io.BytesIO(base64.b64decode(r2["labels_npy_b64"])))
            assert np.array_equal(l2, lref), src
        with pytest.raises(Exception):
            await app.analyze_volume(volume_path="../../etc/passwd", input_is_probability=True)
        await svc.stop_worker(blocking=True)
        await admin.disconnect()

    asyncio.run(asyncio.wait_for(main(), 600))
    reset_local_hubs()
