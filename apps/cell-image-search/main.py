"""Cell morphology similarity search on MI355X.

API parity with the reference app ``apps/cell-image-search/main.py`` (``CellImageSearch``,
``:1033-1519``): ping, get_index_stats, list_datasets, add_dataset, add_jump_cp_dataset,
remove_dataset, start_ingestion, get_ingestion_status, stop_ingestion, get_active_sessions, search,
get_umap_preview, project_query_onto_umap, enrich_metadata_with_compounds — plus
``add_synthetic_dataset`` / ``add_local_dataset`` for offline deployments and ``search`` by raw
array or precomputed embedding.

Everything heavy runs through ``bioengine_worker_amd.search``: GPU nucleus detection (Otsu +
union-find CCL kernels), batched percentile-stretch / PIL-bicubic / ImageNet normalisation kernels,
the DINOv2 ViT-B/14 engine (flash-attention + fused LayerNorm kernels, hipBLASLt GEMMs) and an
HBM-resident inner-product index.  DINOv2 weights: ``BIOENGINE_DINOV2_WEIGHTS`` (a
``dinov2_vitb14_pretrain.pth`` state dict, loaded ``weights_only=True``); random init offline.
"""
from __future__ import annotations

import asyncio
import base64
import io
import json
import os
import time
from datetime import datetime, timezone
from pathlib import Path
from uuid import uuid4

import numpy as np

from bioengine_worker_amd.serve.replica import BIG_STR, Utf8Str
from hypha_rpc.utils.schema import schema_method
from pydantic import Field
from ray import serve

from bioengine.utils import create_logger


def _registry_path(ws: str) -> Path:
    return Path(ws) / "datasets.json"


def _load_registry(ws: str) -> list:
    p = _registry_path(ws)
    return json.loads(p.read_text()) if p.exists() else []


def _save_registry(ws: str, reg: list) -> None:
    p = _registry_path(ws)
    p.parent.mkdir(parents=True, exist_ok=True)
    p.write_text(json.dumps(reg, indent=2, default=str))


def _upsert_registry(ws: str, entry: dict) -> None:
    reg = _load_registry(ws)
    for e in reg:
        if e.get("name") == entry.get("name"):
            e.update(entry)
            break
    else:
        reg.append(entry)
    _save_registry(ws, reg)


#: query batching: up to _QUERY_BATCH concurrent searches share one ViT forward + scan, with up to
#: _QUERY_CONC batches in flight, so one batch's result encoding / transport overlaps the next
#: batch's forward.  A single 64-wide batch at 64 concurrent clients serialises the whole closed
#: loop: 1,396 q/s, p99 167 ms; 32 x 3: 2,305 q/s, p99 108 ms; 16 x 4: 2,401 q/s, p50 24.8 /
#: p99 42.5 ms (MI355X, profiles/r04/search/search_batch_ab.jsonl)
_QUERY_BATCH = int(os.environ.get("BIOENGINE_SEARCH_MAX_BATCH", "16"))
_QUERY_CONC = int(os.environ.get("BIOENGINE_SEARCH_CONCURRENT_BATCHES", "4"))


def _is_npy_b64(s: str) -> bool:
    return s[:8] == base64.b64encode(b"\x93NUMPY")[:8].decode()


def _decode_image_b64(s: str) -> np.ndarray:
    data = base64.b64decode(s)
    if data[:6] == b"\x93NUMPY":
        return np.load(io.BytesIO(data))
    from PIL import Image

    return np.asarray(Image.open(io.BytesIO(data)))


@serve.deployment(
    ray_actor_options={"num_cpus": 4, "num_gpus": 1, "memory": int(8 * 1024 ** 3)},
    # queries are served in batches (one ViT forward + one scan per group): admit a full 64-query batch
    # (the reference's per-request path caps this replica at 10, main.py:1033-1050)
    max_ongoing_requests=64,
    max_queued_requests=256,
    health_check_period_s=60.0,
    health_check_timeout_s=60.0,
    graceful_shutdown_timeout_s=600.0,
)
class CellImageSearch:
    """Large-scale cell morphology similarity search engine."""

    def __init__(self, workspace_dir: str = "", auto_ingest: bool = False, n_synthetic_images: int = 8,
                 model: str = "vitb14") -> None:
        self._workspace_dir = workspace_dir
        self._model = model
        self._auto_ingest = auto_ingest
        self._n_synth = n_synthetic_images
        self._start_time = time.time()
        self._logger = create_logger("CellImageSearch")
        self._worker = None
        self._index = None
        self._metadata_df = None
        self._index_info: dict = {}
        self._thumbnails = None
        self._tasks: dict[str, asyncio.Future] = {}
        self._session_dataset_map: dict[str, str] = {}
        self._lock = asyncio.Lock()
        import threading

        self._gpu_lock = threading.Lock()  # engine / index calls from the batch threads

    # ------------------------------------------------------------------ lifecycle
    async def async_init(self) -> None:
        import torch

        from bioengine_worker_amd.search.ingestion import EmbedWorker, default_engine_factory

        if not self._workspace_dir:
            self._workspace_dir = os.path.join(os.environ.get("HOME", os.getcwd()), "cell_search_data")
        Path(self._workspace_dir).mkdir(parents=True, exist_ok=True)
        dev = "cuda:0" if torch.cuda.is_available() else "cpu"
        # ingestion embeds under the same lock as the query path, so it never runs inside the query
        # path's HIP-graph capture of the same engine (models/vit.py embed_graphed)
        self._worker = await asyncio.to_thread(EmbedWorker, dev, lambda d: default_engine_factory(d, self._model),
                                               64, self._gpu_lock)
        loaded = await self._try_load_index()
        if self._auto_ingest and not loaded:
            await self._start_dataset_ingestion({"name": "Synthetic Cell Painting", "type": "synthetic",
                                                 "config": {"n_images": self._n_synth, "n_crops_per_image": 40}})

    async def test_deployment(self) -> None:
        r = await self.ping()
        assert r["status"] == "ok"

    async def check_health(self) -> None:
        if self._worker is None:
            raise RuntimeError("embedding engine not loaded")

    async def _try_load_index(self) -> bool:
        from bioengine_worker_amd.search.index import VectorIndex
        from bioengine_worker_amd.search.ingestion import index_dir

        d = index_dir(self._workspace_dir)

        def load():
            import pandas as pd

            idx = VectorIndex.load(d)
            meta = pd.read_parquet(d / "metadata.parquet") if (d / "metadata.parquet").exists() else None
            info = json.loads((d / "index_info.json").read_text()) if (d / "index_info.json").exists() else {}
            th = np.load(d / "thumbnails.npy") if (d / "thumbnails.npy").exists() else None
            return idx, meta, info, th

        try:
            self._index, self._metadata_df, self._index_info, self._thumbnails = await asyncio.to_thread(load)
        except FileNotFoundError:
            return False
        await asyncio.to_thread(self._prepare_results_tables)
        return True

    def _prepare_results_tables(self) -> None:
        """Per-result lookups for the serving path: metadata as plain per-column Python lists
        (no pandas row access per result) and the base64 PNG thumbnails encoded at ingestion."""
        from bioengine_worker_amd.search.ingestion import index_dir, read_thumbnails_b64

        df = self._metadata_df
        self._meta_cols = [(c, df[c].tolist()) for c in df.columns] if df is not None else []
        self._meta_n = len(df) if df is not None else 0
        n = len(self._thumbnails) if self._thumbnails is not None else 0
        self._thumbs_b64 = read_thumbnails_b64(index_dir(self._workspace_dir), n) if n else None

    async def _start_dataset_ingestion(self, ds: dict) -> str:
        from bioengine_worker_amd.search import ingestion as ing

        now = datetime.now(timezone.utc)
        sid = now.strftime("%Y%m%d-%H%M%S") + "-" + uuid4().hex[:8]
        cfg = ds.get("config", {})
        name = ds.get("name", "unnamed")
        ing.write_status(self._workspace_dir, sid, ing.IngestionStatus.WAITING, f"Queued: {name}", dataset_name=name)
        _upsert_registry(self._workspace_dir, {"name": name, "type": ds.get("type"), "description": ds.get("description", ""),
                                               "zarr_url": ds.get("zarr_url", ""), "config": cfg, "status": "indexing",
                                               "session_id": sid, "date_added": now.isoformat(), "n_cells": 0})

        def job():
            return ing.run_ingestion(self._workspace_dir, sid, dataset=ds.get("type", "synthetic"),
                                     n_images=cfg.get("n_images", cfg.get("n_plates", 0) * 16),
                                     n_crops_per_image=cfg.get("n_crops_per_image", 80), zarr_url=ds.get("zarr_url"),
                                     local_dir=ds.get("local_dir"), arrays=ds.get("arrays"),
                                     rebuild_index=cfg.get("rebuild_index", False), dataset_name=name,
                                     workers=[self._worker])

        async def run():
            final = await asyncio.to_thread(job)
            await self._try_load_index()
            _upsert_registry(self._workspace_dir, {
                "name": name, "status": "indexed" if final.get("status") == "completed" else final.get("status"),
                "n_cells": final.get("n_embedded", 0), "date_indexed": datetime.now(timezone.utc).isoformat()})
            return final

        async with self._lock:
            self._tasks[sid] = asyncio.ensure_future(run())
            self._session_dataset_map[sid] = name
        return sid

    # ------------------------------------------------------------------ API
    @schema_method
    async def ping(self) -> dict:
        """Check connectivity and get deployment status."""
        return {"status": "ok", "uptime_seconds": round(time.time() - self._start_time, 1),
                "model": f"DINOv2 dinov2_{self._model} (MI355X HIP engine)", "index_loaded": self._index is not None,
                "n_cells_indexed": self._index.ntotal if self._index is not None else 0,
                "index_type": self._index_info.get("index_type", "none"), "workspace_dir": self._workspace_dir,
                "active_sessions": [s for s, t in self._tasks.items() if not t.done()]}

    @schema_method
    async def get_index_stats(self) -> dict:
        """Detailed statistics about the current vector index."""
        if self._index is None:
            return {"indexed": False, "n_cells": 0}
        n_comp = int(self._metadata_df["compound"].nunique()) if self._metadata_df is not None and \
            "compound" in self._metadata_df.columns else 0
        return {"indexed": True, "n_cells": self._index.ntotal, "n_compounds": n_comp, **self._index_info,
                "workspace_dir": self._workspace_dir}

    @schema_method
    async def list_datasets(self) -> dict:
        """All registered datasets and their indexing status."""
        reg = _load_registry(self._workspace_dir)
        active = {s for s, t in self._tasks.items() if not t.done()}
        for e in reg:
            if e.get("session_id") in active:
                e["status"] = "indexing"
        return {"datasets": reg, "active_sessions": sorted(active)}

    @schema_method
    async def add_dataset(self, name: str = Field(..., description="Human-readable dataset name."),
                          zarr_url: str = Field(..., description="HTTP URL of the Zarr store (datasets server)."),
                          description: str = Field("", description="Optional description."),
                          n_slices_per_volume: int = Field(200, ge=10, le=5000, description="2D slices per 3D volume."),
                          n_gpu_workers: int = Field(1, ge=1, le=64, description="GPU workers (one per GPU)."),
                          n_crops_per_slice: int = Field(50, ge=1, le=500, description="Crops per 2D slice.")) -> dict:
        """Register a Zarr dataset and start indexing it."""
        sid = await self._start_dataset_ingestion({"name": name, "type": "zarr", "zarr_url": zarr_url,
                                                   "description": description,
                                                   "config": {"n_images": n_slices_per_volume,
                                                              "n_crops_per_image": n_crops_per_slice}})
        return {"session_id": sid, "name": name, "zarr_url": zarr_url, "status": "queued",
                "message": f"Ingestion started. Poll get_ingestion_status('{sid}')."}

    @schema_method
    async def add_jump_cp_dataset(self, name: str = Field("JUMP Cell Painting", description="Dataset name."),
                                  n_plates: int = Field(10, ge=1, le=500, description="Plates to index."),
                                  n_gpu_workers: int = Field(1, ge=1, le=64, description="GPU workers.")) -> dict:
        """Index JUMP Cell Painting plates (needs BIOENGINE_JUMP_CP_ROOT offline)."""
        sid = await self._start_dataset_ingestion({"name": name, "type": "jump-cp",
                                                   "description": f"JUMP CP (cpg0016), {n_plates} plates.",
                                                   "config": {"n_plates": n_plates, "n_crops_per_image": 80}})
        return {"session_id": sid, "name": name, "status": "queued",
                "message": f"Ingestion started. Poll get_ingestion_status('{sid}')."}

    @schema_method
    async def add_synthetic_dataset(self, name: str = Field("Synthetic Cell Painting", description="Dataset name."),
                                    n_images: int = Field(8, ge=1, le=100000, description="Fields of view."),
                                    n_crops_per_image: int = Field(40, ge=1, le=500, description="Crops per image."),
                                    rebuild_index: bool = Field(False, description="Replace the index.")) -> dict:
        """Index synthetic Cell-Painting-like images (offline demo / benchmarking)."""
        sid = await self._start_dataset_ingestion({"name": name, "type": "synthetic",
                                                   "config": {"n_images": n_images, "n_crops_per_image": n_crops_per_image,
                                                              "rebuild_index": rebuild_index}})
        return {"session_id": sid, "name": name, "status": "queued"}

    @schema_method
    async def add_local_dataset(self, name: str = Field(..., description="Dataset name."),
                                local_dir: str = Field(..., description="Directory of .npy/.npz/.png/.tif images."),
                                n_crops_per_image: int = Field(80, ge=1, le=500, description="Crops per image.")) -> dict:
        """Index a directory of images on the worker's filesystem."""
        sid = await self._start_dataset_ingestion({"name": name, "type": "local", "local_dir": local_dir,
                                                   "config": {"n_images": 0, "n_crops_per_image": n_crops_per_image}})
        return {"session_id": sid, "name": name, "status": "queued"}

    @schema_method
    async def remove_dataset(self, name: str = Field(..., description="Dataset name to remove.")) -> dict:
        """Remove a dataset from the registry (does not delete indexed vectors)."""
        reg = [e for e in _load_registry(self._workspace_dir) if e.get("name") != name]
        _save_registry(self._workspace_dir, reg)
        return {"removed": name, "remaining": len(reg)}

    @schema_method
    async def start_ingestion(self, dataset: str = Field("synthetic", description="'synthetic', 'local', 'zarr' or 'jump-cp'."),
                              n_plates: int = Field(10, ge=1, le=500), zarr_url: str = Field(""),
                              n_crops_per_image: int = Field(80, ge=1, le=500), n_gpu_workers: int = Field(1, ge=1, le=64),
                              workspace_dir: str = Field(""), rebuild_index: bool = Field(False),
                              dataset_name: str = Field(""), local_dir: str = Field("")) -> dict:
        """Low-level ingestion start (prefer add_dataset / add_synthetic_dataset)."""
        name = dataset_name or f"{dataset} {datetime.now(timezone.utc).strftime('%Y-%m-%d %H:%M')}"
        sid = await self._start_dataset_ingestion({"name": name, "type": dataset, "zarr_url": zarr_url or None,
                                                   "local_dir": local_dir or None,
                                                   "config": {"n_images": n_plates * (16 if dataset == "jump-cp" else 1),
                                                              "n_crops_per_image": n_crops_per_image,
                                                              "rebuild_index": rebuild_index}})
        return {"session_id": sid, "status": "waiting", "dataset": dataset}

    @schema_method
    async def get_ingestion_status(self, session_id: str = Field(..., description="Session id.")) -> dict:
        """Real-time status of an ingestion job."""
        from bioengine_worker_amd.search.ingestion import read_status

        st = read_status(self._workspace_dir, session_id)
        t = self._tasks.get(session_id)
        if t is not None and t.done() and st.get("status") in ("running", "preparing", "building_index"):
            exc = t.exception()
            if exc:
                st["status"], st["message"] = "failed", str(exc)
        elif t is not None and not t.done() and st.get("status") == "completed":
            # the worker thread wrote "completed"; the new index is still being loaded into this
            # replica — report completion only once search can see it
            st["status"], st["message"] = "building_index", "Loading the new index"
        return st

    @schema_method
    async def stop_ingestion(self, session_id: str = Field(..., description="Session id to cancel.")) -> dict:
        """Cancel a running ingestion job (cooperative, checked per image)."""
        from bioengine_worker_amd.search.ingestion import read_status, request_stop

        request_stop(self._workspace_dir, session_id)
        name = self._session_dataset_map.get(session_id)
        if name:
            _upsert_registry(self._workspace_dir, {"name": name, "status": "stopped"})
        return read_status(self._workspace_dir, session_id)

    @schema_method
    async def get_active_sessions(self) -> dict:
        """All ingestion sessions of this replica with their status."""
        from bioengine_worker_amd.search.ingestion import read_status

        return {"sessions": [{"session_id": s, "dataset_name": self._session_dataset_map.get(s, ""),
                              "is_running": not t.done(), **read_status(self._workspace_dir, s)}
                             for s, t in list(self._tasks.items())]}

    async def _embed_query(self, image, plow, phigh) -> tuple[np.ndarray, np.ndarray]:
        from bioengine_worker_amd.search import reference as ref

        img = ref.to_hwc(np.asarray(image))
        rgb_f = asyncio.ensure_future(asyncio.to_thread(ref.to_rgb_uint8, img, None, plow, phigh))
        emb = await self._embed_batch((img, float(plow), float(phigh)))
        return emb, await rgb_f

    # ------------------------------------------------------------------ batched serving path
    # Concurrent search requests share ONE fp8 ViT-B/14 forward (up to 64 queries, the reference's
    # embedding batch, embedder.py:59-95) and ONE index scan, instead of one forward + one scan each
    # (the reference embeds and searches per request, main.py:1373-1418).  Two batches in flight:
    # the next batch stacks/uploads while the current one computes.
    @serve.batch(max_batch_size=64, batch_wait_timeout_s=0.002, max_concurrent_batches=2)
    async def _embed_batch(self, reqs: list) -> list:
        """reqs: [(image HWC ndarray, plow, phigh)] -> [embedding fp32 [D]]."""
        import torch

        from bioengine_worker_amd.search.preprocess import batch_to_dinov2

        groups: dict = {}
        for i, (img, pl, ph) in enumerate(reqs):
            groups.setdefault((img.shape, img.dtype.str, pl, ph), []).append(i)
        out = [None] * len(reqs)

        def run():
            for (_, _, pl, ph), idxs in groups.items():
                x = torch.from_numpy(np.ascontiguousarray(np.stack([reqs[i][0] for i in idxs])))
                with self._gpu_lock:
                    t = batch_to_dinov2(x.to(self._worker.device, non_blocking=True), None, pl, ph)
                    e = self._worker.engine.embed(t).float().cpu().numpy()
                for j, i in enumerate(idxs):
                    out[i] = e[j]
            return out

        return await asyncio.to_thread(run)

    @schema_method
    async def get_batch_stats(self) -> dict:
        """Continuous-batching statistics of the query path (batches, requests, batch-size histogram,
        mean queueing wait) for the embedding forward and the index scan."""
        from bioengine_worker_amd.serve.batching import batch_stats

        st = dict(self.__dict__.get("_stage_ms", {}))
        nb = max(1, st.get("batches", 0))
        stages = {k: round(v / nb, 3) for k, v in st.items() if k != "batches"}
        return {"query": batch_stats(self, "_query_batch") or {}, "embed": batch_stats(self, "_embed_batch") or {},
                "search": batch_stats(self, "_search_batch") or {},
                "query_stage_ms_per_batch": stages}

    @serve.batch(max_batch_size=64, batch_wait_timeout_s=0.001, max_concurrent_batches=2)
    async def _search_batch(self, reqs: list) -> list:
        """reqs: [(query fp32 [D], top_k)] -> [(scores [k], ids [k])]: one batched index search."""
        kmax = max(int(k) for _, k in reqs)
        q = np.stack([np.asarray(v, np.float32) for v, _ in reqs])

        def run():
            with self._gpu_lock:
                return self._index.search(q, kmax)

        S, I = await asyncio.to_thread(run)
        return [(S[i, :k], I[i, :k]) for i, (_, k) in enumerate(reqs)]

    def _thumb_b64(self, i: int) -> str:
        """PNG/base64 of an indexed cell's thumbnail, cached (results repeat across queries; the
        encode is the dominant per-result host cost)."""
        cache = self.__dict__.setdefault("_thumb_cache", {})
        v = cache.get(i)
        if v is None:
            from bioengine_worker_amd.search.ingestion import png_b64

            v = png_b64(self._thumbnails[i])
            if len(cache) >= 200_000:
                cache.clear()
            cache[i] = v
        return v

    def _results(self, scores, ids) -> list:
        cols = getattr(self, "_meta_cols", None)
        if cols is None or getattr(self, "_meta_n", -1) != (len(self._metadata_df) if self._metadata_df is not None else 0):
            self._prepare_results_tables()
            cols = self._meta_cols
        nmeta = self._meta_n
        tb = getattr(self, "_thumbs_b64", None)
        nth = len(self._thumbnails) if self._thumbnails is not None else 0
        out = []
        for rank, (s, i) in enumerate(zip(scores.tolist(), ids.tolist())):
            if i < 0:
                continue
            r = {"rank": rank + 1, "score": s, "faiss_idx": i}
            if i < nmeta:
                for c, col in cols:
                    r[c] = col[i]
            t = (tb[i] if tb is not None else self._thumb_b64(i)) if i < nth else ""
            if type(t) is str and len(t) >= BIG_STR and tb is not None:
                # cached UTF-8 form: the thumbnail leaves the replica without a per-response encode
                t = tb[i] = Utf8Str(t)
            r["thumbnail_b64"] = t
            out.append(r)
        return out

    # One batched call per group of concurrent queries: decode-free GPU pre-processing (percentile
    # stretch + bicubic resize + ImageNet norm, K18 kernels), ONE fp8 ViT-B/14 forward, ONE index
    # scan, the query thumbnails from the same resized uint8 tensor, and every request's result list
    # -- each request then does O(1) Python on the event loop (reference: per request decode, CPU
    # stretch, PIL thumbnail, single-image embed and FAISS search, main.py:1373-1418).
    @serve.batch(max_batch_size=_QUERY_BATCH, batch_wait_timeout_s=0.002, max_concurrent_batches=_QUERY_CONC)
    async def _query_batch(self, reqs: list) -> list:
        """reqs: [(image HWC ndarray | base64 .npy str | None, embedding [D] | None, plow, phigh, top_k)]
        -> [(results list, query thumbnail base64)].  Base64 .npy payloads are decoded here, for the
        whole batch at once on host threads outside the GIL (csrc/runtime/png.cpp), not per request
        on the event loop."""
        import torch

        from bioengine_worker_amd.search import reference as ref
        from bioengine_worker_amd.search.ingestion import b64decode_batch, png_b64_batch
        from bioengine_worker_amd.search.preprocess import batch_to_dinov2

        n = len(reqs)

        def run():
            dev = self._worker.device
            q = [None] * n
            thumbs = {}
            # one bad payload fails only its own request: its slot carries the exception, which the
            # batcher turns into that caller's error (serve/batching.py), and it leaves the batch
            err: dict = {}
            tm = [time.perf_counter()]
            imgs = [r[0] for r in reqs]
            enc = [i for i, im in enumerate(imgs) if isinstance(im, str)]
            if enc:
                for i, raw in zip(enc, b64decode_batch([imgs[i] for i in enc])):
                    try:
                        if raw is None:
                            raise ValueError("image_b64 is not valid base64")
                        imgs[i] = ref.to_hwc(np.load(io.BytesIO(memoryview(raw)), allow_pickle=False))
                    except Exception as e:  # noqa: BLE001
                        err[i] = ValueError(f"could not decode the query image: {e}")
            groups: dict = {}
            embs: dict = {}
            for i, (_, emb, pl, ph, _) in enumerate(reqs):
                if i in err:
                    continue
                try:
                    if emb is None:
                        im = imgs[i]
                        if not isinstance(im, np.ndarray) or im.ndim != 3 or im.shape[0] < 1 or im.shape[1] < 1:
                            raise ValueError(f"query image must be HxWxC, got {getattr(im, 'shape', type(im))}")
                        groups.setdefault((im.shape, im.dtype.str, pl, ph), []).append(i)
                    else:
                        v = np.asarray(emb, np.float32)
                        if v.shape != (self._index.dim,) or not np.isfinite(v).all():
                            raise ValueError(f"embedding must be {self._index.dim} finite floats, got shape {v.shape}")
                        embs[i] = v
                except Exception as e:  # noqa: BLE001
                    err[i] = e
            ok = [i for i in range(n) if i not in err]
            S = I = None
            with self._gpu_lock:
                tm.append(time.perf_counter())
                for (_, _, pl, ph), idxs in groups.items():
                    x = torch.from_numpy(np.ascontiguousarray(np.stack([imgs[i] for i in idxs]))).to(dev)
                    t, u8 = batch_to_dinov2(x, None, pl, ph, return_u8=True)
                    eng = self._worker.engine
                    e = (eng.embed_graphed(t) if hasattr(eng, "embed_graphed") else eng.embed(t)).float()
                    u8h = u8.permute(0, 2, 3, 1).contiguous().cpu().numpy()
                    for j, i in enumerate(idxs):
                        q[i] = e[j]
                        thumbs[i] = u8h[j]
                for i, v in embs.items():
                    v = torch.as_tensor(v, device=dev)
                    q[i] = v / v.norm().clamp_min(1e-9)
                tm.append(time.perf_counter())
                if ok:
                    kmax = max(int(reqs[i][4]) for i in ok)
                    S, I = self._index.search(torch.stack([q[i] for i in ok]), kmax)
                tm.append(time.perf_counter())
            res = [None] * n
            for row, i in enumerate(ok):
                k = int(reqs[i][4])
                res[i] = self._results(S[row, :k], I[row, :k])
            tm.append(time.perf_counter())
            # the batch's query thumbnails: one call into the host runtime's linear-time PNG encoder,
            # spread over host threads outside the GIL (csrc/runtime/png.cpp)
            order = sorted(thumbs)
            enc = dict(zip(order, (Utf8Str(v) for v in png_b64_batch(np.stack([thumbs[i] for i in order]))))) \
                if order else {}
            tm.append(time.perf_counter())
            st = self.__dict__.setdefault("_stage_ms", {"batches": 0, "decode": 0.0, "embed": 0.0, "scan": 0.0,
                                                        "results": 0.0, "thumbs": 0.0})
            st["batches"] += 1
            for k, a, b in (("decode", 0, 1), ("embed", 1, 2), ("scan", 2, 3), ("results", 3, 4), ("thumbs", 4, 5)):
                st[k] += (tm[b] - tm[a]) * 1e3
            return [err[i] if i in err else (res[i], enc.get(i, "")) for i in range(n)]

        return await asyncio.to_thread(run)

    @schema_method
    async def search(self, image_b64: str | None = Field(None, description="Base64 image (PNG/JPG/TIFF or .npy bytes)."),
                     image: list | None = Field(None, description="Image as a nested array (alternative to image_b64)."),
                     embedding: list | None = Field(None, description="Precomputed 768-d query embedding."),
                     top_k: int = Field(20, ge=1, le=100), plow: float = Field(1.0, ge=0.0, le=10.0),
                     phigh: float = Field(99.0, ge=90.0, le=100.0)) -> dict:
        """Top-K morphologically similar cells in the indexed database."""
        if self._index is None:
            return {"error": "No index loaded. Add a dataset first.", "results": []}
        t0 = time.time()
        from bioengine_worker_amd.search import reference as ref

        img = None
        if embedding is None:
            if image_b64 is not None and _is_npy_b64(image_b64):
                img = image_b64  # decoded with the rest of its batch (_query_batch)
            else:
                raw = await asyncio.to_thread(_decode_image_b64, image_b64) if image_b64 is not None \
                    else np.asarray(image)
                img = ref.to_hwc(np.asarray(raw))
        results, qthumb = await self._query_batch((img, embedding, float(plow), float(phigh), int(top_k)))
        return {"results": results, "query_thumbnail_b64": qthumb,
                "elapsed_ms": round((time.time() - t0) * 1000, 1), "n_cells_searched": self._index.ntotal, "top_k": top_k}

    @schema_method
    async def get_umap_preview(self, n_samples: int = Field(10_000, ge=100, le=100_000), color_by: str = Field("compound"),
                               force_recompute: bool = Field(False)) -> dict:
        """2-D projection of a sample of indexed cells (UMAP if installed, else GPU PCA)."""
        from bioengine_worker_amd.search.ingestion import index_dir
        from bioengine_worker_amd.search.projection import compute_projection

        labels = None
        if self._metadata_df is not None and color_by in self._metadata_df.columns:
            labels = self._metadata_df[color_by].astype(str).tolist()
        cache = index_dir(self._workspace_dir) / f"umap_cache_{color_by}.npz"
        return await asyncio.to_thread(compute_projection, self._index, labels, cache, n_samples, 42, force_recompute)

    @schema_method
    async def project_query_onto_umap(self, image_b64: str = Field(..., description="Base64 query image.")) -> dict:
        """Place a query on the projection at its nearest indexed neighbour."""
        if self._index is None:
            return {"error": "No index loaded."}
        q, _ = await self._embed_query(_decode_image_b64(image_b64), 1.0, 99.0)
        S, I = await asyncio.to_thread(self._index.search, q[None], 1)
        proj = await self.get_umap_preview()
        nn = int(I[0, 0])
        x = y = 0.0
        if nn >= 0 and proj["sample_idx"]:
            sidx = np.asarray(proj["sample_idx"])
            j = int(np.argmin(np.abs(sidx - nn)))
            x, y = proj["x"][j], proj["y"][j]
        meta = self._metadata_df.iloc[nn].to_dict() if self._metadata_df is not None and nn >= 0 else {}
        return {"umap_x": float(x), "umap_y": float(y), "nearest_score": float(S[0, 0]),
                "nearest_compound": meta.get("compound", "unknown"), "nearest_moa": meta.get("moa_class", "unknown")}

    @schema_method
    async def enrich_metadata_with_compounds(self, lookup_csv: str = Field("", description=(
            "CSV with columns source, plate, well, compound[, moa_class]; default <workspace>/compound_lookup.csv"))) -> dict:
        """Join compound / MOA annotations into the index metadata (no index rebuild)."""
        import pandas as pd

        from bioengine_worker_amd.search.ingestion import index_dir

        meta_path = index_dir(self._workspace_dir) / "metadata.parquet"
        if not meta_path.exists():
            return {"error": "No metadata.parquet found. Run ingestion first."}
        src = Path(lookup_csv or Path(self._workspace_dir) / "compound_lookup.csv")
        if not src.exists():
            return {"error": f"compound lookup table not found at {src} (the JUMP metadata download needs network)"}
        lk = pd.read_csv(src).astype(str)
        df = pd.read_parquet(meta_path)
        key = [c for c in ("source", "plate", "well") if c in lk.columns and c in df.columns]
        cols = [c for c in ("compound", "moa_class") if c in lk.columns]
        merged = df.drop(columns=[c for c in cols if c in df.columns]).merge(lk[key + cols], on=key, how="left")
        for c in cols:
            merged[c] = merged[c].fillna("unknown")
        merged.to_parquet(meta_path, index=False)
        self._metadata_df = merged
        self._prepare_results_tables()
        for p in index_dir(self._workspace_dir).glob("umap_cache*.npz"):
            p.unlink()
        n_after = int((merged["compound"] != "unknown").sum()) if "compound" in merged.columns else 0
        return {"status": "ok", "n_total": len(merged), "n_enriched": n_after, "n_unknown": len(merged) - n_after,
                "n_unique_compounds": int(merged["compound"].nunique()) if "compound" in merged.columns else 0,
                "enriched_pct": round(100 * n_after / max(len(merged), 1), 1)}
