"""Ingestion pipeline: images -> nucleus crops -> DINOv2 embeddings -> vector index.

Reference: apps/cell-image-search/ingestion.py:394-591 (Ray-task version) and main.py:704-968
(head-node embedder pool).  MI355X design: one embedding worker per visible GPU (a thread owning
that GPU's :class:`ViTEngine`), image decoding on a CPU thread pool that stays ahead of the GPUs,
crops + pre-processing + embedding all on the GPU (no host round trip per crop), embeddings kept
on-device until the index build.  Status and stop handling follow the reference session layout:
``<workspace>/sessions/<id>/status.json`` and ``stop_requested``.

Sources: ``synthetic`` (Cell-Painting-like 5-channel images, used offline and by tests/bench),
``local`` (a directory of .npy/.npz/.png/.tif images, optional metadata.csv), ``arrays``
(in-memory), ``zarr`` (2-D slices of a volume served by the datasets server), ``jump-cp`` (needs
the public S3 bucket; offline it requires ``BIOENGINE_JUMP_CP_ROOT`` pointing to a local mirror).
"""
from __future__ import annotations

import base64
import io
import json
import logging
import os
import queue
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from enum import Enum
from pathlib import Path
from typing import Any, Callable, Iterator

import numpy as np
import torch

from .index import VectorIndex

log = logging.getLogger("cell-image-search")


class IngestionStatus(str, Enum):
    WAITING = "waiting"
    PREPARING = "preparing"
    RUNNING = "running"
    BUILDING_INDEX = "building_index"
    COMPLETED = "completed"
    STOPPED = "stopped"
    FAILED = "failed"


def session_dir(ws: str, sid: str) -> Path:
    return Path(ws) / "sessions" / sid


def write_status(ws: str, sid: str, status: IngestionStatus, message: str, n_embedded: int = 0, n_total: int = 0,
                 throughput_per_sec: float = 0.0, elapsed_seconds: float = 0.0, dataset_name: str = "",
                 log_lines: list[str] | None = None, **extra: Any) -> dict:
    p = session_dir(ws, sid) / "status.json"
    p.parent.mkdir(parents=True, exist_ok=True)
    old: dict = {}
    if p.exists():
        try:
            old = json.loads(p.read_text())
        except Exception:  # noqa: BLE001
            old = {}
    tail = list(old.get("log_tail", []))
    if log_lines:
        tail = (tail + list(log_lines))[-20:]
    d = {**old, "status": status.value, "message": message, "dataset_name": dataset_name or old.get("dataset_name", ""),
         "n_embedded": n_embedded, "n_total": n_total, "progress_pct": round(100.0 * n_embedded / max(n_total, 1), 1),
         "throughput_per_sec": round(throughput_per_sec, 1), "elapsed_seconds": round(elapsed_seconds, 1),
         "eta_seconds": round((n_total - n_embedded) / max(throughput_per_sec, 0.1)), "log_tail": tail,
         "updated_at": time.time(), **extra}
    tmp = p.with_suffix(".json.tmp")
    tmp.write_text(json.dumps(d, indent=2, default=str))
    tmp.replace(p)
    return d


def read_status(ws: str, sid: str) -> dict:
    p = session_dir(ws, sid) / "status.json"
    if not p.exists():
        return {"status": IngestionStatus.WAITING.value, "message": "Not started"}
    try:
        return json.loads(p.read_text())
    except Exception:  # noqa: BLE001
        return {"status": "unknown", "message": "Error reading status"}


def request_stop(ws: str, sid: str) -> None:
    p = session_dir(ws, sid) / "stop_requested"
    p.parent.mkdir(parents=True, exist_ok=True)
    p.write_text("1")


def is_stop_requested(ws: str, sid: str) -> bool:
    return (session_dir(ws, sid) / "stop_requested").exists()


# ------------------------------------------------------------------ sources

COMPOUNDS = ["DMSO", "staurosporine", "nocodazole", "taxol", "cytochalasin-D", "brefeldin-A", "tunicamycin",
             "rapamycin"]
MOA = {"DMSO": "control", "staurosporine": "kinase inhibitor", "nocodazole": "tubulin destabilizer",
       "taxol": "tubulin stabilizer", "cytochalasin-D": "actin disruptor", "brefeldin-A": "golgi disruptor",
       "tunicamycin": "glycosylation inhibitor", "rapamycin": "mTOR inhibitor"}


def synthetic_cell_painting(i: int, size: int = 1080, n_cells: int = 60, seed: int = 0) -> tuple[np.ndarray, dict]:
    """A 5-channel uint16 field of view (DNA, ER, RNA, AGP, Mito) with ~n_cells cells; the
    compound modulates cell size/texture so embeddings carry signal."""
    rng = np.random.default_rng(seed * 100003 + i)
    comp = COMPOUNDS[i % len(COMPOUNDS)]
    k = COMPOUNDS.index(comp)
    img = rng.normal(300, 30, (size, size, 5)).clip(0, None)
    yy, xx = np.mgrid[0:size, 0:size]
    for _ in range(n_cells):
        cy, cx = rng.uniform(40, size - 40, 2)
        r_nuc = rng.uniform(9, 14) * (1 + 0.08 * k)
        r_cell = r_nuc * rng.uniform(1.8, 2.6)
        y0, y1 = int(max(cy - 3 * r_cell, 0)), int(min(cy + 3 * r_cell, size))
        x0, x1 = int(max(cx - 3 * r_cell, 0)), int(min(cx + 3 * r_cell, size))
        d2 = (yy[y0:y1, x0:x1] - cy) ** 2 + (xx[y0:y1, x0:x1] - cx) ** 2
        nuc = np.exp(-d2 / (2 * r_nuc ** 2))
        cell = np.exp(-d2 / (2 * r_cell ** 2))
        img[y0:y1, x0:x1, 0] += 3000 * (nuc > 0.5) * (0.8 + 0.2 * nuc)
        img[y0:y1, x0:x1, 1] += 1200 * cell * (1 + 0.3 * np.sin(d2 / (5 + k)))
        img[y0:y1, x0:x1, 2] += 900 * cell * nuc
        img[y0:y1, x0:x1, 3] += 1500 * cell * (1 + 0.5 * (k % 3 == 0) * np.cos(xx[y0:y1, x0:x1] / 3.0))
        img[y0:y1, x0:x1, 4] += 800 * cell
    meta = {"source": "synthetic", "plate": f"SYN{i // 16:04d}", "well": f"r{(i % 16) // 4:02d}c{i % 4:02d}",
            "site": i, "compound": comp, "moa_class": MOA[comp], "image_path": f"synthetic://{i}"}
    return img.astype(np.uint16), meta


def _decode_file(p: Path) -> np.ndarray:
    if p.suffix == ".npy":
        return np.load(p)
    if p.suffix == ".npz":
        z = np.load(p)
        return z[z.files[0]]
    from PIL import Image

    return np.asarray(Image.open(p))


def iter_source(dataset: str, n_images: int, zarr_url: str | None = None, arrays=None, local_dir: str | None = None,
                n_slices: int = 200) -> tuple[int, Callable[[int], tuple[np.ndarray, dict]]]:
    """Returns (n_images, loader(i) -> (image HxWxC, metadata))."""
    if dataset == "synthetic":
        return n_images, lambda i: synthetic_cell_painting(i)
    if dataset == "arrays":
        arrs = list(arrays or [])
        return len(arrs), lambda i: (np.asarray(arrs[i]), {"source": "arrays", "image_path": f"array://{i}"})
    if dataset in ("local", "jump-cp"):
        root = local_dir or (os.environ.get("BIOENGINE_JUMP_CP_ROOT") if dataset == "jump-cp" else None)
        if not root or not Path(root).is_dir():
            raise RuntimeError(
                "JUMP Cell Painting lives in the public S3 bucket s3://cellpainting-gallery; this worker has no "
                "network access — set BIOENGINE_JUMP_CP_ROOT to a local mirror (directory of images)"
                if dataset == "jump-cp" else f"local dataset directory not found: {root}")
        files = sorted(p for p in Path(root).rglob("*") if p.suffix.lower() in (".npy", ".npz", ".png", ".tif", ".tiff"))
        meta_rows = {}
        mcsv = Path(root) / "metadata.csv"
        if mcsv.exists():
            import pandas as pd

            for r in pd.read_csv(mcsv).to_dict("records"):
                meta_rows[str(r.get("image_path", ""))] = r
        files = files[: n_images] if n_images else files

        def load(i):
            p = files[i]
            rel = str(p.relative_to(root))
            m = {"source": dataset, "image_path": rel, "plate": p.parent.name, "well": p.stem}
            m.update(meta_rows.get(rel, {}))
            return _decode_file(p), m
        return len(files), load
    if dataset == "zarr":
        if not zarr_url:
            raise ValueError("zarr dataset needs zarr_url")
        from ..datasets.store import HttpZarrStore, read_zarr_array
        import asyncio

        store = HttpZarrStore(zarr_url)
        vol = asyncio.run(read_zarr_array(store))
        if vol.ndim == 2:
            vol = vol[None]
        z = np.linspace(0, vol.shape[0] - 1, min(n_slices, vol.shape[0])).astype(int)
        z = z[: n_images] if n_images else z
        return len(z), lambda i: (vol[z[i]], {"source": zarr_url, "image_path": f"{zarr_url}#z={z[i]}", "slice": int(z[i])})
    raise ValueError(f"unknown dataset type {dataset!r}")


# ------------------------------------------------------------------ pipeline

def _thumbs(crops_u8: torch.Tensor, size: int = 96) -> np.ndarray:
    t = torch.nn.functional.interpolate(crops_u8.float(), size=(size, size), mode="area")
    return t.round().clamp(0, 255).to(torch.uint8).permute(0, 2, 3, 1).cpu().numpy()


def png_b64(rgb: np.ndarray, compress_level: int = 6) -> str:
    from PIL import Image

    buf = io.BytesIO()
    Image.fromarray(rgb, mode="RGB").save(buf, format="PNG", compress_level=compress_level)
    return base64.b64encode(buf.getvalue()).decode()


def png_b64_batch(rgb: np.ndarray, threads: int = 8) -> list[str]:
    """Base64 PNGs of uint8 RGB images [n, h, w, 3] from the host runtime's linear-time encoder
    (``csrc/runtime/png.cpp``: filter-0 rows in stored deflate blocks -- no compression search, so a
    224x224 thumbnail costs a fraction of a millisecond instead of PIL's 6-11 ms; the whole batch
    runs on host threads outside the GIL).  Falls back to PIL when the runtime is not built."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    if rgb.ndim != 4 or rgb.shape[-1] != 3:
        raise ValueError(f"expected [n, h, w, 3] uint8, got {rgb.shape}")
    n, h, w, _ = rgb.shape
    if n == 0:
        return []
    try:
        from ..ops import _native

        lib = _native.runtime()
        cap = int(lib.be_rt_png_b64_cap(h, w))
        if cap <= 0:
            raise ValueError("image too large")
        out = np.empty(cap * n, np.uint8)
        lens = np.empty(n, np.int64)
        _native.rt_call("be_rt_png_b64_batch", rgb.ctypes.data, n, h, w, out.ctypes.data, cap, lens.ctypes.data,
                        int(threads))
        return [out[i * cap: i * cap + int(lens[i])].tobytes().decode("ascii") for i in range(n)]
    except (OSError, AttributeError, ImportError, ValueError) as e:
        if isinstance(e, ValueError) and "too large" not in str(e):
            raise
        return [png_b64(rgb[i], 1) for i in range(n)]


def b64decode_batch(strings: list, threads: int = 8) -> list:
    """Decoded bytes (uint8 ndarray views) of base64 strings, decoded by the host runtime on host
    threads outside the GIL (``csrc/runtime/png.cpp``); falls back to :func:`base64.b64decode`."""
    n = len(strings)
    if n == 0:
        return []
    try:
        import ctypes

        from ..ops import _native

        lib = _native.runtime()
        # the ASCII bytes of each string: attached to strings received out of band (serve/replica.py
        # Utf8Str), else one encode
        raw = [np.frombuffer(s.utf8, np.uint8) if hasattr(s, "utf8") else
               np.frombuffer(s.encode("ascii") if isinstance(s, str) else s, np.uint8) for s in strings]
        ptrs = (ctypes.c_void_p * n)(*[r.ctypes.data for r in raw])
        lens = np.array([r.size for r in raw], np.int64)
        cap = int(lens.max()) * 3 // 4 + 3
        out = np.empty(cap * n, np.uint8)
        olen = np.empty(n, np.int64)
        lib.be_rt_b64decode_batch.argtypes = None  # variadic-safe: pass ctypes objects as they are
        rc = lib.be_rt_b64decode_batch(ptrs, lens.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(n),
                                       out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(cap),
                                       olen.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(int(threads)))
        if rc != 0 or (olen < 0).any():
            raise ValueError("b64 decode failed")
        return [out[i * cap: i * cap + int(olen[i])] for i in range(n)]
    except (OSError, AttributeError, ImportError, UnicodeEncodeError, ValueError):
        # per item, so one malformed payload yields None in its own slot, not a failed batch
        res = []
        for s in strings:
            try:
                res.append(np.frombuffer(base64.b64decode(s, validate=False), np.uint8))
            except (ValueError, TypeError):
                res.append(None)
        return res


THUMBS_B64 = "thumbnails_b64.txt"


def write_thumbnails_b64(out: Path, thumbs: np.ndarray, start: int = 0) -> None:
    """Result thumbnails as base64 PNG, one per line, encoded once at ingestion (the reference stores
    them as base64 strings too, ``apps/cell-image-search/main.py:1404-1408``): serving a result
    is then a list lookup, never an encode.  ``start`` > 0 appends the thumbnails from that row."""
    mode = "a" if start > 0 and (out / THUMBS_B64).exists() else "w"
    rows = range(start if mode == "a" else 0, len(thumbs))
    with open(out / THUMBS_B64, mode) as f:
        for i in rows:
            f.write(png_b64(thumbs[i]) + "\n")


def read_thumbnails_b64(out: Path, n: int) -> list | None:
    p = Path(out) / THUMBS_B64
    if not p.exists():
        return None
    lines = p.read_text().splitlines()
    return lines if len(lines) == n else None


class EmbedWorker:
    """Owns one GPU's ViT engine; embeds crop batches."""

    def __init__(self, device, engine_factory: Callable[[Any], Any], batch_size: int = 64, gpu_lock=None):
        import contextlib

        self.device = torch.device(device)
        self.engine = engine_factory(self.device)
        self.batch_size = batch_size
        # held around every engine call: an app that also serves queries from this engine (and
        # captures HIP graphs of it) passes its own lock so ingestion never runs inside a capture
        self.gpu_lock = gpu_lock if gpu_lock is not None else contextlib.nullcontext()

    def process(self, image: np.ndarray, n_crops: int, rgb_channels=None):
        from . import reference as ref
        from .nuclei import extract_cell_crops
        from .preprocess import batch_to_dinov2

        img = torch.from_numpy(np.ascontiguousarray(ref.to_hwc(image)))
        if self.device.type == "cuda":
            img = img.to(self.device, non_blocking=True)
        crops = extract_cell_crops(img, 224, n_crops)
        if crops.shape[0] == 0:
            return None, None
        embs = []
        thumbs = []
        for i in range(0, crops.shape[0], self.batch_size):
            c = crops[i:i + self.batch_size]
            x = batch_to_dinov2(c.to(self.device), rgb_channels)
            with self.gpu_lock:
                embs.append(self.engine.embed(x))
            # thumbnails of the displayed RGB composite (ImageNet de-normalised)
            mean = torch.tensor([0.485, 0.456, 0.406], device=x.device)[None, :, None, None]
            std = torch.tensor([0.229, 0.224, 0.225], device=x.device)[None, :, None, None]
            u8 = ((x.float() * std + mean) * 255.0).round().clamp(0, 255)
            thumbs.append(_thumbs(u8))
        return torch.cat(embs), np.concatenate(thumbs)


def default_engine_factory(device, model: str = "vitb14", precision: str | None = None):
    """DINOv2 engine; ``model`` = vits14/vitb14/vitl14/vitg14, or ``tiny-test`` (2 blocks, for CPU tests).

    ``precision``: ``"fp8"`` (default on GPU: e4m3 GEMMs, cosine >= 0.99 to bf16, 1.11x faster —
    profiles/README.md) or ``"bf16"``; ``BIOENGINE_EMBED_PRECISION`` overrides the default."""
    from ..models.vit import ViT, ViTConfig, ViTEngine

    weights = os.environ.get("BIOENGINE_DINOV2_WEIGHTS")
    cfg = ViTConfig(embed_dim=128, depth=2, num_heads=2) if model == "tiny-test" else ViTConfig.dinov2(model)
    net = ViT(cfg)
    if weights and Path(weights).exists():
        sd = torch.load(weights, map_location="cpu", weights_only=True)
        net.load_state_dict(sd, strict=False)
    else:
        net.randomize_(0)
    if precision is None:
        precision = os.environ.get("BIOENGINE_EMBED_PRECISION") or (
            "fp8" if torch.device(device).type == "cuda" else "bf16")
    return ViTEngine(net.eval(), device, precision=precision)


def run_ingestion(workspace_dir: str, session_id: str, dataset: str = "synthetic", n_images: int = 8,
                  n_crops_per_image: int = 80, zarr_url: str | None = None, arrays=None, local_dir: str | None = None,
                  rebuild_index: bool = False, dataset_name: str = "", devices: list | None = None,
                  workers: list | None = None, engine_factory=default_engine_factory, rgb_channels=None,
                  io_threads: int = 4) -> dict:
    """Blocking ingestion (run it in a thread).  Returns the final status dict."""
    ws = workspace_dir
    t0 = time.time()
    name = dataset_name or dataset
    upd = lambda st, msg, **kw: write_status(ws, session_id, st, msg, dataset_name=name, elapsed_seconds=time.time() - t0,
                                             **kw)
    try:
        upd(IngestionStatus.PREPARING, "Listing images", log_lines=[f"source={dataset}"])
        n, loader = iter_source(dataset, n_images, zarr_url, arrays, local_dir)
        if workers is None:
            if devices is None:
                devices = ([f"cuda:{i}" for i in range(torch.cuda.device_count())] if torch.cuda.is_available()
                           else ["cpu"])
            workers = [EmbedWorker(d, engine_factory) for d in devices]
        n_total_expected = n * n_crops_per_image
        upd(IngestionStatus.RUNNING, f"Embedding {n} images on {len(workers)} device(s)", n_total=n_total_expected)
        results: list = [None] * n
        lock = threading.Lock()
        done = {"cells": 0, "images": 0}
        stop = threading.Event()
        pool = ThreadPoolExecutor(max_workers=io_threads, thread_name_prefix="ingest-io")
        futs = [pool.submit(loader, i) for i in range(n)]
        work_q: queue.Queue = queue.Queue()
        for i in range(n):
            work_q.put(i)
        last = [0.0]

        def gpu_loop(w: EmbedWorker):
            while not stop.is_set():
                try:
                    i = work_q.get_nowait()
                except queue.Empty:
                    return
                if is_stop_requested(ws, session_id):
                    stop.set()
                    return
                img, meta = futs[i].result()
                emb, th = w.process(img, n_crops_per_image, rgb_channels)
                with lock:
                    if emb is not None:
                        results[i] = (emb.cpu(), th, meta)
                        done["cells"] += emb.shape[0]
                    done["images"] += 1
                    el = time.time() - t0
                    if time.time() - last[0] > 1.0:
                        last[0] = time.time()
                        upd(IngestionStatus.RUNNING, f"{done['images']}/{n} images, {done['cells']} cells",
                            n_embedded=done["cells"], n_total=n_total_expected,
                            throughput_per_sec=done["cells"] / max(el, 1e-3))

        threads = [threading.Thread(target=gpu_loop, args=(w,), daemon=True) for w in workers]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        pool.shutdown(wait=False, cancel_futures=True)
        if stop.is_set():
            return upd(IngestionStatus.STOPPED, "Stopped by user", n_embedded=done["cells"], n_total=n_total_expected)
        upd(IngestionStatus.BUILDING_INDEX, "Building index", n_embedded=done["cells"], n_total=n_total_expected)
        embs, thumbs, rows = [], [], []
        for r in results:
            if r is None:
                continue
            e, th, meta = r
            embs.append(e)
            thumbs.append(th)
            rows.extend([dict(meta, cell_idx=j) for j in range(e.shape[0])])
        if not embs:
            raise RuntimeError("no cells were extracted")
        E = torch.cat(embs).float()
        info = build_or_append(ws, E, rows, np.concatenate(thumbs), rebuild=rebuild_index)
        el = time.time() - t0
        return upd(IngestionStatus.COMPLETED, f"Indexed {E.shape[0]} cells ({info['index_type']})",
                   n_embedded=int(E.shape[0]), n_total=int(E.shape[0]), throughput_per_sec=E.shape[0] / max(el, 1e-3),
                   index_info=info)
    except Exception as e:  # noqa: BLE001
        log.exception("ingestion failed")
        return upd(IngestionStatus.FAILED, f"{type(e).__name__}: {e}")


def index_dir(ws: str) -> Path:
    return Path(ws) / "cell_search"


def build_or_append(ws: str, E: torch.Tensor, rows: list[dict], thumbs: np.ndarray, rebuild: bool = False) -> dict:
    import pandas as pd

    out = index_dir(ws)
    out.mkdir(parents=True, exist_ok=True)
    df_new = pd.DataFrame(rows)
    if not rebuild and (out / "vectors.npy").exists():
        idx = VectorIndex.load(out)
        df_old = pd.read_parquet(out / "metadata.parquet") if (out / "metadata.parquet").exists() else pd.DataFrame()
        th_old = np.load(out / "thumbnails.npy") if (out / "thumbnails.npy").exists() else np.zeros((0,) + thumbs.shape[1:],
                                                                                                     np.uint8)
        idx.add(E)
        df = pd.concat([df_old, df_new], ignore_index=True)
        thumbs = np.concatenate([th_old, thumbs])
    else:
        idx = VectorIndex(dim=E.shape[1])
        idx.add(E)
        df = df_new
    for c in ("compound", "moa_class"):
        if c not in df.columns:
            df[c] = "unknown"
    df = df.astype({c: str for c in df.columns if df[c].dtype == object})
    info = idx.save(out)
    df.to_parquet(out / "metadata.parquet", index=False)
    n_old = 0 if rebuild else len(thumbs) - len(rows)
    np.save(out / "thumbnails.npy", thumbs.astype(np.uint8))
    if n_old and read_thumbnails_b64(out, n_old) is None:
        n_old = 0  # no (or a stale) encoded file: encode everything
    write_thumbnails_b64(out, thumbs.astype(np.uint8), n_old)
    for p in out.glob("umap_cache*.npz"):
        p.unlink()
    return info
