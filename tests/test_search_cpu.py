"""cell-image-search building blocks on CPU: oracle pre-processing, nuclei, vector index, app e2e."""
import asyncio
import base64
import io
from pathlib import Path

import numpy as np
import pytest
import torch

from bioengine_worker_amd.search import reference as ref
from bioengine_worker_amd.search.index import VectorIndex
from bioengine_worker_amd.search.ingestion import synthetic_cell_painting
from bioengine_worker_amd.search.preprocess import pil_bicubic_coeffs

ROOT = Path(__file__).resolve().parents[1]


def test_reference_nuclei_on_synthetic_field():
    img, meta = synthetic_cell_painting(3, size=720, n_cells=30)
    cents = ref.nucleus_centroids(img, n_crops=100)
    assert len(cents) >= 10
    crops = ref.extract_cell_crops(img, 224, 20)
    assert crops and crops[0].shape == (224, 224, 5)
    assert meta["compound"] in ref.__dict__.get("COMPOUNDS", meta["compound"]) or meta["compound"]


def test_otsu_matches_formula():
    rng = np.random.default_rng(0)
    im = np.concatenate([rng.normal(40, 5, 500), rng.normal(200, 10, 500)]).clip(0, 255).astype(np.uint8)
    t = ref.otsu_threshold_u8(im)
    lo, hi = im[:500].max(), im[500:].min()
    assert lo <= t < hi  # skimage returns the first bin of the optimal plateau


def test_pil_coefficients_sum_to_one():
    W, S = pil_bicubic_coeffs(300, 224)
    assert np.allclose(W.sum(1), 1.0, atol=1e-5) and S.min() >= 0 and S.max() < 300


def test_to_dinov2_matches_pil_pipeline():
    img = (np.random.default_rng(1).random((180, 200, 5)) * 4000).astype(np.uint16)
    rgb = ref.to_rgb_uint8(img)
    assert rgb.shape == (180, 200, 3)
    arr = ref.to_dinov2_array(rgb)
    assert arr.shape == (3, 224, 224) and abs(float(arr.mean())) < 3


def test_vector_index_flat_and_ivf():
    rng = np.random.default_rng(0)
    centers = rng.normal(size=(20, 32))
    x = centers[rng.integers(0, 20, 4000)] + 0.1 * rng.normal(size=(4000, 32))
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    idx = VectorIndex(dim=32, device="cpu")
    idx.add(x)
    q = x[:50]
    S, I = idx.search(q, 5)
    ref_I = np.argsort(-(q @ x.T), axis=1)[:, :5]
    assert (I[:, 0] == np.arange(50)).all() and (I == ref_I).mean() > 0.95
    ivf = VectorIndex(dim=32, device="cpu", nprobe=8)
    ivf.add(x)
    ivf.train_ivf(nlist=64)
    S2, I2 = ivf.search(q, 5)
    recall = np.mean([len(set(a) & set(b)) / 5 for a, b in zip(I2, ref_I)])
    assert recall > 0.8 and ivf.index_type.startswith("IVFFlat")


def test_vector_index_save_load(tmp_path):
    idx = VectorIndex(dim=16, device="cpu")
    v = np.random.default_rng(0).normal(size=(10, 16)).astype(np.float32)
    idx.add(v)
    info = idx.save(tmp_path)
    assert info["n_cells"] == 10
    idx2 = VectorIndex.load(tmp_path, device="cpu")
    assert idx2.ntotal == 10 and np.allclose(idx2.reconstruct_batch([3]), v[3], atol=1e-2)


@pytest.mark.end_to_end
def test_cell_image_search_app_e2e(tmp_path, monkeypatch):
    from bioengine_worker_amd.transport import connect_to_server
    from bioengine_worker_amd.transport.hub import get_local_hub, reset_local_hubs
    from bioengine_worker_amd.worker.worker import BioEngineWorker

    monkeypatch.setenv("BIOENGINE_LOCAL_ARTIFACT_PATH", str(ROOT / "apps"))
    monkeypatch.setenv("BIOENGINE_REPLICA_MODE", "local")
    monkeypatch.setenv("HOME", str(tmp_path / "home"))
    reset_local_hubs()

    async def main():
        hub = get_local_hub("cis")
        await hub.start_http()
        tok = hub.issue_token("admin-user", workspace="ws-admin")
        w = BioEngineWorker(mode="single-machine", workspace_dir=tmp_path / "be", server_url="local://cis", token=tok,
                            client_id="worker1", log_file="off", head_num_cpus=4, head_num_gpus=0,
                            monitoring_interval_seconds=0.5, data_server_url=None)
        await w.start(blocking=False)
        admin = await connect_to_server({"server_url": "local://cis", "token": tok})
        svc = await admin.get_service(w.full_service_id)
        aid = await svc.deploy_app(artifact_id="cell-image-search", application_id="cis", disable_gpu=True,
                                   application_kwargs={"CellImageSearch": {"model": "tiny-test"}})
        assert await w.apps_manager.wait_for(aid, timeout=240) == "RUNNING", \
            (await svc.get_app_status(application_ids=[aid]))["message"]
        s = await svc.get_app_status(application_ids=[aid])
        app = await admin.get_service(s["service_ids"][0]["websocket_service_id"])
        assert (await app.ping())["index_loaded"] is False
        r = await app.add_synthetic_dataset(n_images=2, n_crops_per_image=12)
        sid = r["session_id"]
        for _ in range(600):
            st = await app.get_ingestion_status(session_id=sid)
            if st["status"] in ("completed", "failed", "stopped"):
                break
            await asyncio.sleep(0.2)
        assert st["status"] == "completed", st
        stats = await app.get_index_stats()
        assert stats["indexed"] and stats["n_cells"] >= 12
        img, _ = synthetic_cell_painting(0, size=720, n_cells=30)
        buf = io.BytesIO()
        np.save(buf, img[200:424, 200:424])
        res = await app.search(image_b64=base64.b64encode(buf.getvalue()).decode(), top_k=5)
        assert len(res["results"]) == 5 and res["results"][0]["score"] >= res["results"][-1]["score"]
        assert res["results"][0]["thumbnail_b64"] and "compound" in res["results"][0]
        # concurrent queries are served through one batched embedding forward + one index scan
        b64 = base64.b64encode(buf.getvalue()).decode()
        many = await asyncio.gather(*[app.search(image_b64=b64, top_k=3 + i % 3) for i in range(12)])
        for i, r in enumerate(many):
            assert len(r["results"]) == 3 + i % 3
            assert r["results"][0]["faiss_idx"] == res["results"][0]["faiss_idx"]
        bs = await app.get_batch_stats()
        # one batched call per query group: pre-processing, embedding, scan and result lists
        assert bs["query"]["requests"] >= 13 and bs["query"]["mean_batch"] > 1.0, bs
        assert bs["query"]["batches"] < bs["query"]["requests"], bs
        assert res["query_thumbnail_b64"] and many[0]["query_thumbnail_b64"]
        # a malformed payload in the same batch fails only its own request: a truncated
        # .npy, a non-base64 .npy-looking string and a wrong-length embedding beside good queries
        raw = buf.getvalue()
        bad_npy = base64.b64encode(raw[:64]).decode()
        bad_b64 = b64[:8] + "!!!!" + b64[8:40] + "="
        mixed = await asyncio.gather(
            app.search(image_b64=b64, top_k=3), app.search(image_b64=bad_npy, top_k=3),
            app.search(image_b64=b64, top_k=4), app.search(embedding=[1.0] * 5, top_k=3),
            app.search(image_b64=bad_b64, top_k=3), app.search(image_b64=b64, top_k=5),
            return_exceptions=True)
        for j, k in ((0, 3), (2, 4), (5, 5)):
            assert not isinstance(mixed[j], BaseException), mixed[j]
            assert len(mixed[j]["results"]) == k
            assert mixed[j]["results"][0]["faiss_idx"] == res["results"][0]["faiss_idx"]
        for j in (1, 3, 4):
            assert isinstance(mixed[j], BaseException), mixed[j]
        emb = await app.search(embedding=[1.0] * int(stats.get("embed_dim", 768)), top_k=4)
        assert len(emb["results"]) == 4 and emb["query_thumbnail_b64"] == ""
        up = await app.get_umap_preview(n_samples=100)
        assert len(up["x"]) == stats["n_cells"] and up["method"] in ("pca", "umap")
        pq = await app.project_query_onto_umap(image_b64=base64.b64encode(buf.getvalue()).decode())
        assert "umap_x" in pq
        ds = await app.list_datasets()
        assert ds["datasets"][0]["status"] == "indexed"
        await svc.stop_worker(blocking=True)
        await admin.disconnect()

    asyncio.run(asyncio.wait_for(main(), 600))
    reset_local_hubs()


def test_compressed_tier_host_refine(tmp_path):
    """compress(): PQ codes on the index device, full vectors in host memory as the exact re-rank
    store; the refined top-k matches exact search, and save/load keeps the tier."""
    import torch

    from bioengine_worker_amd.search.index import VectorIndex

    g = torch.Generator().manual_seed(0)
    cent = torch.nn.functional.normalize(torch.randn(40, 64, generator=g), dim=1)
    x = torch.nn.functional.normalize(cent[torch.randint(0, 40, (4000,), generator=g)]
                                      + 0.3 * torch.randn(4000, 64, generator=g), dim=1)
    q = torch.nn.functional.normalize(x[:16] + 0.05 * torch.randn(16, 64, generator=g), dim=1)
    idx = VectorIndex(dim=64, device="cpu", index_type="flat")
    idx.add(x)
    _, exact = idx.search(q, 10)
    fp = idx.compress(pq_m=16, refine=20, nlist=16)
    assert idx.host_refine and idx.vecs.device.type == "cpu" and fp["host_bytes"] > 0 and fp["gpu_bytes"] > 0
    idx.pq.nprobe = 16
    _, got = idx.search(q, 10)
    rec = np.mean([len(set(a) & set(b)) / 10 for a, b in zip(exact, got)])
    assert rec >= 0.9, rec
    idx.save(tmp_path)
    back = VectorIndex.load(tmp_path, device="cpu")
    assert back.host_refine and back.pq is not None and back.refine == 20
    back.pq.nprobe = 16
    _, got2 = back.search(q, 10)
    assert (got2 == got).all()
