"""Cellpose fine-tuning + inference app on the MI355X-native Cellpose implementation.

API parity with the reference app ``apps/cellpose-finetuning/main.py`` (CellposeFinetune,
``:3633-5144``): ``start_training`` (artifact folder / glob / metadata pairing, ``n_samples``,
``rescale``, CLAHE, label), ``stop_training``, ``get_training_status`` (stale-session
normalisation), ``restart_training`` (re-reads the session from disk), ``list_training_sessions``,
``delete_training_session`` (owner-checked), ``export_model`` (BioImage.IO package created, uploaded
and committed into a collection artifact), ``list_models_by_dataset``, ``infer`` and
``debug_task_info``.  The default and reference model is ``cpsam`` (Cellpose-SAM, ViT-L/8);
``cyto3`` (CPnet U-Net) is also built in.

MI355X design:
* inference: ``CellposeRunner`` batches the tiles of every request in a continuous batch
  (``@serve.batch``) through the HIP Cellpose-SAM / CPnet engines and batched mask recovery;
* training: ``train/session.py`` on the HIP CPSAM training engine (flash-attention fwd/bwd, fused
  LN/GELU backward, fused AdamW, HIP-graph step) in a thread of this replica, or -- with
  ``n_gpus > 1`` -- as a gang-scheduled data-parallel job (``serve/gang.py``): one process per GPU,
  gradient buckets all-reduced over RCCL/xGMI while backward runs.
* offline there are no pretrained checkpoints: ``BIOENGINE_CPSAM_WEIGHTS`` / ``BIOENGINE_CYTO3_WEIGHTS``
  load real weights, otherwise the built-ins are random and every response says ``weights: random``.
"""
from __future__ import annotations

import asyncio
import base64
import io
import json
import logging
import os
import shutil
import threading
import time
import uuid
from concurrent.futures import ThreadPoolExecutor
from datetime import datetime, timezone
from pathlib import Path
from typing import Any

import numpy as np
from hypha_rpc.utils.schema import schema_method
from pydantic import Field
from ray import serve

from bioengine_worker_amd.cellpose.datasets import (  # noqa: F401  (re-exported: reference test surface)
    HubArtifact,
    create_dataset_split,
    decode_image,
    list_artifact_files,
    list_artifact_files_recursive,
    list_matching_artifact_paths,
    make_training_pairs,
    make_training_pairs_from_metadata,
    match_image_annotation_pairs,
    read_image,
)
from bioengine_worker_amd.cellpose.model_store import BUILTIN_MODELS
from bioengine_worker_amd.profiling import trace
from bioengine_worker_amd.serve.batching import offload
from bioengine_worker_amd.train.session import now_iso, read_status, to_chw, write_status  # noqa: F401

log = logging.getLogger("ray.serve")
STATUS_STALE_SECONDS = 300.0
DEFAULT_COLLECTION = "bioimage-io/colab-annotations"
TRAINING_PARAMS_FILENAME = "training_params.json"


def sessions_root() -> Path:
    p = Path(os.environ.get("HOME", ".")) / "sessions"
    p.mkdir(parents=True, exist_ok=True)
    return p


def session_dir(sid: str) -> Path:
    return sessions_root() / sid


def normalize_session_id(session_id: Any) -> str:
    if isinstance(session_id, dict):
        session_id = session_id.get("session_id", session_id.get("id", ""))
    s = str(session_id).strip().replace("\\", "/")
    if s.endswith("/status.json"):
        s = s[: -len("/status.json")]
    return Path(s).name


def _opt(v):
    """Reference ``normalize_optional_param``: '', 'none', 'null' and pydantic FieldInfo mean None."""
    if v is None or type(v).__name__ == "FieldInfo":
        return None
    if isinstance(v, str) and v.strip().lower() in ("", "none", "null"):
        return None
    return v


def _user_id(context) -> str | None:
    if isinstance(context, dict) and isinstance(context.get("user"), dict):
        return context["user"].get("id")
    return None


def image_chw(img: np.ndarray, nchan: int) -> np.ndarray:
    """[H,W] / [H,W,C] / [C,H,W] -> [nchan, H, W] in the image's OWN dtype (uint8/uint16 stay
    integers: half / a quarter of the float32 bytes through the replica ring and over PCIe; the GPU
    converts while normalising)."""
    a = np.asarray(img)
    if a.ndim == 2:
        a = a[None]
    elif a.ndim == 3 and a.shape[-1] <= 4 and a.shape[0] > 4:
        a = np.moveaxis(a, -1, 0)
    if a.dtype not in (np.uint8, np.uint16, np.float16, np.float32):
        a = a.astype(np.float32)
    if a.shape[0] < nchan:
        a = np.concatenate([a, np.zeros((nchan - a.shape[0],) + a.shape[1:], a.dtype)], 0)
    return np.ascontiguousarray(a[:nchan])


class HWCImage:
    """An [H, W, C] image with C == the model's channel count, passed through batching untransposed:
    the GPU path stages it as is (a plain copy into pinned memory) and permutes to CHW on the device
    after the H2D; the host-side HWC -> CHW copy it replaces cost ~0.4 ms per 512^2 2-channel uint16
    image, a third of the served c=1 overhead."""

    __slots__ = ("a",)

    def __init__(self, a: np.ndarray):
        self.a = a

    @property
    def shape(self):
        h, w, c = self.a.shape
        return (c, h, w)

    @property
    def dtype(self):
        return self.a.dtype

    def chw(self) -> np.ndarray:
        return np.ascontiguousarray(np.moveaxis(self.a, -1, 0))


def image_for_batch(img, nchan: int, gpu: bool):
    """``image_chw`` for the batcher; on the GPU path an [H, W, nchan] image of a staged dtype stays
    HWC (see :class:`HWCImage`)."""
    a = np.asarray(img)
    if (gpu and a.ndim == 3 and a.shape[-1] == nchan and a.shape[0] > 4 and
            a.dtype in (np.uint8, np.uint16, np.float16, np.float32)):
        return HWCImage(a)
    return image_chw(a, nchan)


def mask_png_payload(mask: np.ndarray) -> dict:
    """JSON-safe mask overlay (reference ``encode_mask_png_payload``): RGBA PNG where each label
    gets a fixed colour, alpha 150 on objects; vectorised with a per-label colour table."""
    from PIL import Image

    m = np.squeeze(np.asarray(mask))
    if m.ndim != 2:
        raise ValueError(f"Expected 2D mask, got shape={m.shape}")
    lab = m.astype(np.int64)
    ids = np.unique(lab)
    ids = ids[ids > 0]
    rgba = np.zeros(lab.shape + (4,), np.uint8)
    fg = lab > 0
    v = lab[fg]
    rgba[fg] = np.stack([(v * 123) % 255, (v * 231) % 255, (v * 73) % 255, np.full_like(v, 150)], -1).astype(np.uint8)
    buf = io.BytesIO()
    Image.fromarray(rgba, mode="RGBA").save(buf, format="PNG", optimize=True)
    return {"encoding": "mask_png_base64", "width": int(lab.shape[1]), "height": int(lab.shape[0]),
            "object_count": int(ids.size), "png_base64": base64.b64encode(buf.getvalue()).decode("ascii")}


def flow_rgb(dP: np.ndarray) -> np.ndarray:
    """cellpose ``dx_to_circ``: flow angle -> hue, magnitude -> value, as uint8 RGB [H, W, 3]."""
    dy, dx = dP[0], dP[1]
    mag = np.sqrt(dy * dy + dx * dx)
    mag = np.clip(mag / max(float(np.percentile(mag, 99)), 1e-6), 0, 1)
    ang = np.arctan2(dy, dx) + np.pi
    r = np.clip((np.cos(ang) + 1) / 2, 0, 1) * mag
    g = np.clip((np.cos(ang + 2 * np.pi / 3) + 1) / 2, 0, 1) * mag
    b = np.clip((np.cos(ang + 4 * np.pi / 3) + 1) / 2, 0, 1) * mag
    return (np.stack([r, g, b], -1) * 255).astype(np.uint8)


def clahe_image(img: np.ndarray, device=None) -> np.ndarray:
    """Reference CLAHE pre-processing (grayscale uint8, clip 3.0, 16x16 tiles; main.py:273-308):
    HIP kernel on a GPU device, the OpenCV-semantics numpy oracle otherwise."""
    import torch

    from bioengine_worker_amd.ops.clahe import clahe_u8, to_gray_u8

    g = torch.from_numpy(to_gray_u8(img))
    if device is not None and torch.device(device).type == "cuda":
        g = g.to(device)
    return clahe_u8(g, 3.0, (16, 16)).cpu().numpy()


@serve.deployment(
    ray_actor_options={"num_gpus": 1, "num_cpus": 4, "memory": 12 * 1024 ** 3},
    # one GPU-pinned replica by default (the reference app's single replica); a node-level deployment
    # sets BIOENGINE_CELLPOSE_REPLICAS to its GPU count and the router spreads requests over them
    num_replicas=int(os.environ.get("BIOENGINE_CELLPOSE_REPLICAS", "1")),
    max_ongoing_requests=64,  # >= 2 full continuous batches in flight at the replica
    max_queued_requests=256,
    health_check_period_s=30.0,
    health_check_timeout_s=60.0,
    graceful_shutdown_timeout_s=300.0,
)
class CellposeFinetune:
    def __init__(self, default_model: str = "cpsam", max_batch_size: int = 16, cpsam_arch: str = "vit_l",
                 dataset_cache_dir: str | None = None) -> None:
        sessions_root()
        self.default_model = default_model
        self.max_batch_size = max_batch_size
        self.cpsam_arch = cpsam_arch
        self.cache_dir = Path(dataset_cache_dir or Path(os.environ.get("HOME", ".")) / "datasets")
        self.pretrained_models = list(BUILTIN_MODELS)
        self.executors: dict[str, ThreadPoolExecutor] = {}
        self.tasks: dict[str, asyncio.Future] = {}
        self._lock = asyncio.Lock()
        self._weights: dict[str, str] = {}
        self._gpu_lock = threading.Lock()
        self._mask_lock = threading.Lock()  # mask recovery of one batch overlaps the next batch's network

    # ------------------------------------------------------------------ models
    def _device(self):
        import torch

        return torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")

    def _build_net(self, model_id: str):
        from bioengine_worker_amd.cellpose.model_store import resolve_net

        net, src = resolve_net(model_id, sessions_root(), self.cpsam_arch)
        self._weights[model_id] = src
        return net

    @serve.multiplexed(max_num_models_per_replica=4)
    async def _runner(self, model_id: str):
        from bioengine_worker_amd.cellpose.pipeline import CellposeRunner

        net = await asyncio.to_thread(self._build_net, model_id)
        return await asyncio.to_thread(CellposeRunner, net, self._device())

    async def _hub(self):
        from hypha_rpc import connect_to_server

        return await connect_to_server({"server_url": os.environ.get("HYPHA_SERVER_URL"),
                                        "token": os.environ.get("HYPHA_TOKEN")})

    async def resolve_model_id(self, model: str) -> str:
        """Built-in name, local session id, or a published model artifact (downloaded into a local
        session directory once, reference ``ensure_published_model_local_session``)."""
        if model in BUILTIN_MODELS:
            return model
        sid = normalize_session_id(model)
        if (session_dir(sid) / "models" / "model").exists():
            return sid
        if "/" in str(model):
            return await self._fetch_published(str(model))
        raise ValueError(f"Model identifier '{model}' is not a known pretrained model or a valid session ID / "
                         "published artifact reference.")

    async def _fetch_published(self, ref: str) -> str:
        """``ws/alias`` or ``https://server/<ws>/artifacts/<alias>`` -> local session holding its weights."""
        if "/artifacts/" in ref:
            head, alias = ref.rstrip("/").split("/artifacts/", 1)
            aid = f"{head.rstrip('/').split('/')[-1]}/{alias.split('/')[0]}"
        else:
            aid = ref.strip("/")
        sid = "published-" + aid.replace("/", "--")
        d = session_dir(sid)
        if (d / "models" / "model").exists():
            return sid
        server = await self._hub()
        try:
            art = HubArtifact(await server.get_service("public/artifact-manager"), aid)
            (d / "models").mkdir(parents=True, exist_ok=True)
            await art.get(["model_weights.pth"], [str(d / "models" / "model")])
        finally:
            await server.disconnect()
        write_status(d, status_type="completed", message=f"Published model {aid}", published_artifact_id=aid,
                     created_at=now_iso())
        return sid

    # ------------------------------------------------------------------ lifecycle
    #: batch sizes the replica runs once at start-up, largest first (BE_CELLPOSE_PREWARM=0 skips it):
    #: EVERY size the batcher can form (1..32), not only powers of two -- the c = 64 serving tail of
    #: round 6 came as ~30 ms stalls at the first batch of a new size (3, 5, ...: allocator growth and
    #: per-shape plans on the request path; profiles/r06/README.md §4)
    PREWARM_BATCHES = tuple(range(32, 0, -1))

    async def async_init(self) -> None:
        await self._runner(self.default_model)
        if os.environ.get("BE_CELLPOSE_PREWARM", "1") != "0":
            await self._prewarm(int(os.environ.get("BE_CELLPOSE_PREWARM_SIZE", "512")))

    async def _prewarm(self, size: int = 512) -> None:
        """Run every continuous-batching size once before the replica takes traffic.  The first batch
        of a new size pays one-time costs on the request path: pinned host staging blocks, device
        allocator growth for that batch's work buffers, the engine's per-shape plans.  At c = 64 the
        first two 32-image batches paid ~110 ms each, which put ~1 % of all requests (the router p99)
        at ~143 ms (BENCH_r05).  Largest first, so the caching allocators keep the biggest blocks
        and smaller batches are carved from them."""
        import torch

        if not torch.cuda.is_available() and os.environ.get("BE_CELLPOSE_PREWARM") != "force":
            return  # CPU replicas pay none of these costs ("force": the CPU test of this path)
        from bioengine_worker_amd.cellpose.pipeline import synthetic_cells

        imgs = [synthetic_cells(1, size, size, ncells=40, seed=s)[0] for s in range(4)]
        for b in self.PREWARM_BATCHES:
            await asyncio.gather(*[self.infer(input_arrays=[imgs[i % 4]], model=self.default_model)
                                   for i in range(b)])

    async def test_deployment(self) -> None:
        from bioengine_worker_amd.cellpose.pipeline import synthetic_cells

        img = synthetic_cells(1, 128, 128, ncells=8)[0]
        out = await self.infer(input_arrays=[img], model=self.default_model)
        assert out[0]["output"].shape == (128, 128)

    # ------------------------------------------------------------------ inference (continuous batching)
    @serve.batch(max_batch_size=32, batch_wait_timeout_s=0.005, max_concurrent_batches=2)
    async def _segment_batch(self, reqs: list) -> list:
        """reqs: [(model_id, image CHW, params dict, want_flows)] -> [(masks, flows | None)].

        Two batches are in flight: while one batch's kernels run (under the GPU lock, on the
        default stream), the other stacks its images or copies its masks back on a side stream
        into pinned memory, so host work and PCIe transfers hide behind GPU compute."""
        from bioengine_worker_amd.profiling import trace

        out = [None] * len(reqs)
        groups: dict = {}
        for i, (mid, img, prm, want_flows) in enumerate(reqs):
            key = (mid, img.shape, img.dtype.str, isinstance(img, HWCImage), tuple(sorted(prm.items())))
            groups.setdefault(key, []).append(i)
        for (mid, shape, _, _, prm_items), idxs in groups.items():
            runner = await self._runner(mid)
            prm = dict(prm_items)
            flows_needed = any(reqs[i][3] for i in idxs)

            def run():
                import torch

                with trace.span("app.stack", images=len(idxs)):
                    batch = self._stage_batch([reqs[i][1] for i in idxs], runner)
                if torch.is_tensor(batch) and batch.is_cuda:  # H2D issued on the copy stream
                    torch.cuda.current_stream(batch.device).wait_stream(self._h2d_stream)
                    batch.record_stream(torch.cuda.current_stream(batch.device))
                with trace.span("app.eval", images=len(idxs)):
                    if hasattr(runner, "eval_locked"):
                        # network under the GPU lock, mask recovery under its own lock on a second
                        # stream: the other in-flight batch's network overlaps this batch's masks
                        m, f, _, ev = runner.eval_locked(batch, self._gpu_lock, self._mask_lock, **prm)
                    else:
                        with self._gpu_lock:
                            m, f, _ = runner.eval(batch, **prm)
                            ev = None
                            if m.is_cuda:
                                ev = torch.cuda.Event()
                                ev.record()
                with trace.span("app.d2h", images=len(idxs)):
                    if not m.is_cuda:
                        return m.numpy(), (f.numpy() if flows_needed else None)
                    if getattr(self, "_d2h_stream", None) is None:
                        self._d2h_stream = torch.cuda.Stream(m.device)
                    st = self._d2h_stream
                    # Labels are renumbered 1..n with every mask >= min_size pixels, so an image of
                    # fewer than 65536 * min_size pixels cannot overflow uint16 (512^2 at the default
                    # min_size 15): no overflow reduction and no second copy to wait for.
                    min_size = int(prm.get("min_size", 15) or 0)
                    fits = min_size > 0 and m[0].numel() < 65536 * min_size
                    with torch.cuda.stream(st):
                        st.wait_event(ev)
                        # uint16 masks (cellpose's dtype when labels fit): low 16 bits + an overflow
                        # flag, so the copy-back needs a single host sync
                        m16 = m.to(torch.int16)
                        mh = torch.empty(m.shape, dtype=torch.int16, pin_memory=True)
                        mh.copy_(m16, non_blocking=True)
                        over = oh = None
                        if not fits:
                            over = (m > 65535).any().reshape(1)
                            oh = torch.empty(1, dtype=torch.bool, pin_memory=True)
                            oh.copy_(over, non_blocking=True)
                        fh = f.to("cpu", non_blocking=True) if flows_needed else None
                        for t in (m, m16) + ((over,) if over is not None else ()) + ((f,) if f is not None else ()):
                            t.record_stream(st)
                    st.synchronize()
                    if oh is not None and bool(oh[0]):  # more than 65535 objects in an image: int32 labels
                        return m.cpu().numpy(), (fh.numpy() if fh is not None else None)
                    return mh.numpy().view(np.uint16), (fh.numpy() if fh is not None else None)

            masks, flows = await offload(run)
            for j, i in enumerate(idxs):
                out[i] = (masks[j], flows[j] if flows is not None and reqs[i][3] else None)
        return out

    def _stage_batch(self, images: list, runner):
        """Stack the batch straight into pinned host memory (one copy) and start its H2D on a copy
        stream before taking the GPU lock, so the transfer overlaps the other in-flight batch's
        kernels instead of sitting on the critical path."""
        import torch

        dev = getattr(runner, "device", None)
        hwc = isinstance(images[0], HWCImage)
        if dev is None or torch.device(dev).type != "cuda":
            return np.stack([im.chw() for im in images] if hwc else images)
        arrs = [im.a for im in images] if hwc else images
        a0 = arrs[0]
        tdt = torch.from_numpy(np.empty(0, a0.dtype)).dtype
        host = torch.empty((len(arrs),) + tuple(a0.shape), dtype=tdt, pin_memory=True)
        np.stack(arrs, out=host.numpy())
        if getattr(self, "_h2d_stream", None) is None:
            self._h2d_stream = torch.cuda.Stream(dev)
        with torch.cuda.stream(self._h2d_stream):
            x = host.to(dev, non_blocking=True)
            return x.permute(0, 3, 1, 2).contiguous() if hwc else x

    async def _images_from_artifact(self, artifact: str, paths: list[str]) -> list[np.ndarray]:
        server = await self._hub()
        try:
            art = HubArtifact(await server.get_service("public/artifact-manager"), artifact)
            d = self.cache_dir / artifact.replace("/", "--")
            loc = [str(d / p.lstrip("/")) for p in paths]
            await art.get([p for p in paths], loc)
            return [read_image(p) for p in loc]
        finally:
            await server.disconnect()

    @schema_method
    async def infer(
        self,
        artifact: str | None = Field(None, description="Artifact 'workspace/alias' containing the source images."),
        image_paths: list | None = Field(None, description="Artifact-relative image paths to segment."),
        input_arrays: list | None = Field(None, description="Images as arrays ([H,W], [H,W,C] or [C,H,W])."),
        model: str = Field("cpsam", description="Built-in model ('cpsam', 'cyto3'), a session id of a fine-tuned "
                                                "model, or a published model artifact id."),
        diameter: float | None = Field(None, description="Approximate object diameter (rescale to the model's 30 px)."),
        flow_threshold: float = Field(0.4, description="Flow error threshold (QC)."),
        cellprob_threshold: float = Field(0.0, description="Cell probability threshold."),
        niter: int | None = Field(None, description="Flow-dynamics iterations (default 200)."),
        return_flows: bool = Field(False, description="Also return [RGB flow, dY/dX flows, cell probability]."),
        json_safe: bool = Field(False, description="Masks as PNG overlay payloads instead of arrays."),
        enable_clahe: bool = Field(False, description="CLAHE pre-processing (brightfield / phase contrast)."),
    ) -> list:
        """Segment images; returns one {input_path, output(, flows)} per image."""
        if isinstance(artifact, dict):
            w = artifact
            artifact = w.get("artifact", w.get("artifact_id", w.get("id")))
            image_paths, input_arrays = w.get("image_paths", image_paths), w.get("input_arrays", input_arrays)
            model, diameter = w.get("model", model), w.get("diameter", diameter)
            flow_threshold = w.get("flow_threshold", flow_threshold)
            cellprob_threshold = w.get("cellprob_threshold", cellprob_threshold)
            niter, return_flows = w.get("niter", niter), w.get("return_flows", return_flows)
            json_safe, enable_clahe = w.get("json_safe", json_safe), w.get("enable_clahe", enable_clahe)
        model = _opt(model) or self.default_model
        model_id = await self.resolve_model_id(model)
        if _opt(input_arrays) is not None:
            images = [np.asarray(a) for a in input_arrays]
            names = [f"input_arrays[{i}]" for i in range(len(images))]
        elif _opt(artifact) is not None:
            names = list(image_paths or [])
            images = await self._images_from_artifact(artifact, names)
        else:
            raise ValueError("Provide input_arrays or artifact + image_paths")
        if enable_clahe:
            images = [clahe_image(im, self._device()) for im in images]
        runner = await self._runner(model_id)
        prm = {"diameter": _opt(diameter), "flow_threshold": float(flow_threshold),
               "cellprob_threshold": float(cellprob_threshold), "niter": int(_opt(niter) or 200)}
        on_gpu = str(getattr(runner, "device", "cpu")).startswith("cuda")
        chw = [image_for_batch(im, runner.nchan, on_gpu) for im in images]
        with trace.span("app.batched", images=len(chw)):
            if len(chw) == 1:
                res = [await self._segment_batch((model_id, chw[0], prm, bool(return_flows)))]
            else:
                res = await asyncio.gather(*[self._segment_batch((model_id, c, prm, bool(return_flows))) for c in chw])
        out = []
        for name, (m, f) in zip(names, res):
            item = {"input_path": name, "output": mask_png_payload(m) if json_safe else m}
            if return_flows:
                fl = [flow_rgb(f[:2]), f[:2], f[2]]
                item["flows"] = [x.tolist() for x in fl] if json_safe else fl
            out.append(item)
        if self._weights.get(model_id) == "random" and out:
            out[0]["weights"] = "random"
        return out

    # ------------------------------------------------------------------ training
    async def _prepare_data(self, sid: str, params: dict, arrays: dict | None) -> None:
        """Write the session's ``pairs.json``: artifact pairs (cached downloads) or saved arrays."""
        d = session_dir(sid)
        if arrays is not None:
            data = d / "data"
            data.mkdir(parents=True, exist_ok=True)
            pairs = {"train": [], "test": []}
            for split in ("train", "test"):
                for i, (im, lab) in enumerate(zip(arrays.get(f"{split}_images") or [], arrays.get(f"{split}_labels") or [])):
                    ip, lp = data / f"{split}_{i:04d}_img.npy", data / f"{split}_{i:04d}_masks.npy"
                    np.save(ip, np.asarray(im))
                    np.save(lp, np.asarray(lab).astype(np.int32))
                    pairs[split].append({"image": str(ip), "annotation": str(lp)})
        else:
            aid = params["artifact_id"]
            server = await self._hub()
            try:
                art = HubArtifact(await server.get_service("public/artifact-manager"), aid)
                cache = self.cache_dir / aid.replace("/", "--")
                tr, te = await make_training_pairs(art, params, cache)
            finally:
                await server.disconnect()
            split = create_dataset_split(tr, te)
            pairs = {"train": [{"image": str(a), "annotation": str(b)} for a, b in
                               zip(split["train_files"], split["train_labels_files"])],
                     "test": [{"image": str(a), "annotation": str(b)} for a, b in
                              zip(split["test_files"] or [], split["test_labels_files"] or [])]}
        if params.get("n_samples") is not None and arrays is not None:
            pairs["train"] = pairs["train"][: int(params["n_samples"])]
        (d / "pairs.json").write_text(json.dumps(pairs, indent=1))

    async def _run_session(self, sid: str, params: dict, arrays: dict | None, source: str | None) -> None:
        d = session_dir(sid)
        try:
            if source is not None and (session_dir(source) / "pairs.json").exists():
                if (session_dir(source) / "data").exists():
                    shutil.copytree(session_dir(source) / "data", d / "data", dirs_exist_ok=True)
                txt = (session_dir(source) / "pairs.json").read_text().replace(str(session_dir(source) / "data"),
                                                                               str(d / "data"))
                (d / "pairs.json").write_text(txt)
            else:
                write_status(d, status_type="preparing", message="Downloading and pairing training data")
                await self._prepare_data(sid, params, arrays)
            n_gpus = int(params.get("n_gpus") or 1)
            if n_gpus > 1:
                from bioengine_worker_amd.train.session import run_dp_session

                write_status(d, message=f"Waiting for {n_gpus} GPUs (data-parallel gang)")
                # a rank failure restarts a fresh gang at n_gpus - 1 from the last epoch checkpoint
                res = await run_dp_session(d, params, n_gpus, self.cpsam_arch, max_restarts=params.get("max_restarts"),
                                           name=f"train-{sid[-8:]}")
                write_status(d, rank_weight_digests=[r.get("weights_sha256") for r in res])
            else:
                from bioengine_worker_amd.train.session import train_session

                loop = asyncio.get_running_loop()
                await loop.run_in_executor(self.executors[sid], train_session, d, params, self._device(), 0, 1, None,
                                           self.cpsam_arch)
        except Exception as e:  # noqa: BLE001
            log.exception("session %s failed", sid)
            write_status(d, status_type="failed", message=f"{type(e).__name__}: {e}")

    async def _launch(self, sid: str, params: dict, arrays: dict | None = None, source: str | None = None):
        async with self._lock:
            self.executors[sid] = ThreadPoolExecutor(max_workers=1, thread_name_prefix=f"train-{sid[-8:]}")
            self.tasks[sid] = asyncio.ensure_future(self._run_session(sid, params, arrays, source))

    @schema_method
    async def start_training(
        self,
        artifact: str | None = Field(None, description="Dataset artifact 'workspace/alias' with images and annotations."),
        train_images: str | None = Field(None, description="Folder ('images/') or glob ('images/*/*.tif') of training images."),
        train_annotations: str | None = Field(None, description="Folder or glob of annotations; the '*' parts must "
                                                                "match the images' (e.g. 'annotations/*/*_mask.ome.tif')."),
        metadata_dir: str | None = Field(None, description="Folder of JSON files listing image/annotation pairs."),
        test_images: str | None = Field(None, description="Folder or glob of test images (enables validation)."),
        test_annotations: str | None = Field(None, description="Folder or glob of test annotations."),
        model: str = Field("cpsam", description="Model to fine-tune: built-in, session id or published artifact."),
        n_samples: int | None = Field(None, description="Random subset of this many training pairs."),
        n_epochs: int = Field(10, description="Number of training epochs."),
        learning_rate: float = Field(1e-6, description="AdamW learning rate."),
        weight_decay: float = Field(1e-4, description="AdamW weight decay."),
        min_train_masks: int = Field(5, description="Drop training images with fewer masks."),
        validation_interval: int | None = Field(None, description="Validate every N epochs (and at epoch 1); default 10."),
        enable_clahe: bool = Field(False, description="CLAHE pre-processing of training and test images."),
        rescale: bool = Field(False, description="Rescale crops by each image's estimated cell diameter."),
        label: str | None = Field(None, description="Annotation label (saved with the session, used as a filter)."),
        batch_size: int = Field(1, description="Crops per optimisation step and GPU (reference: 1)."),
        n_gpus: int = Field(1, description="Data-parallel GPUs (a gang of one process per GPU, RCCL all-reduce)."),
        train_arrays: list | None = Field(None, description="Training images as arrays (instead of an artifact)."),
        label_arrays: list | None = Field(None, description="Instance label arrays for train_arrays."),
        test_arrays: list | None = Field(None, description="Test images as arrays."),
        test_label_arrays: list | None = Field(None, description="Instance label arrays for test_arrays."),
        context: dict | None = Field(None, description="Authentication context (injected)."),
    ) -> dict:
        """Start asynchronous fine-tuning; returns the initial session status with its ``session_id``."""
        if isinstance(artifact, dict):
            w = artifact
            artifact = w.get("artifact", w.get("artifact_id", w.get("id")))
            train_images, train_annotations = w.get("train_images", train_images), w.get("train_annotations", train_annotations)
            metadata_dir, test_images = w.get("metadata_dir", metadata_dir), w.get("test_images", test_images)
            test_annotations, model = w.get("test_annotations", test_annotations), w.get("model", model)
            n_samples, n_epochs = w.get("n_samples", n_samples), w.get("n_epochs", n_epochs)
            learning_rate, weight_decay = w.get("learning_rate", learning_rate), w.get("weight_decay", weight_decay)
            min_train_masks = w.get("min_train_masks", min_train_masks)
            validation_interval = w.get("validation_interval", validation_interval)
            enable_clahe, rescale = bool(w.get("enable_clahe", enable_clahe)), bool(w.get("rescale", rescale))
            label, context = w.get("label", label), w.get("context", context)
        artifact, metadata_dir = _opt(artifact), _opt(metadata_dir)
        train_images, train_annotations = _opt(train_images), _opt(train_annotations)
        test_images, test_annotations = _opt(test_images), _opt(test_annotations)
        arrays = None
        if _opt(train_arrays) is not None:
            if label_arrays is None or len(label_arrays) != len(train_arrays):
                raise ValueError("label_arrays must give one label image per train_arrays entry")
            arrays = {"train_images": list(train_arrays), "train_labels": list(label_arrays),
                      "test_images": list(test_arrays or []), "test_labels": list(test_label_arrays or [])}
        elif metadata_dir is None:
            if not isinstance(train_images, str) or not train_images:
                raise ValueError("train_images must be a non-empty string when metadata_dir is not provided")
            if not isinstance(train_annotations, str) or not train_annotations:
                raise ValueError("train_annotations must be a non-empty string when metadata_dir is not provided")
        if arrays is None and not artifact:
            raise ValueError("artifact is required (or pass train_arrays / label_arrays)")
        if (test_images is None) != (test_annotations is None):
            raise ValueError("test_images and test_annotations must be provided together")
        model_id = await self.resolve_model_id(_opt(model) or "cpsam")
        sid = datetime.now(timezone.utc).strftime("%Y-%m-%d-%H%M%S") + "-" + uuid.uuid4().hex[:8]
        params = {"artifact_id": artifact, "train_images": train_images, "train_annotations": train_annotations,
                  "metadata_dir": metadata_dir, "test_images": test_images, "test_annotations": test_annotations,
                  "model": model_id, "n_epochs": int(_opt(n_epochs) or 10),
                  "learning_rate": float(_opt(learning_rate) or 1e-6),
                  "weight_decay": float(weight_decay if _opt(weight_decay) is not None else 1e-4),
                  "server_url": os.environ.get("HYPHA_SERVER_URL"),
                  "n_samples": int(n_samples) if _opt(n_samples) is not None else None, "session_id": sid,
                  "min_train_masks": int(min_train_masks if _opt(min_train_masks) is not None else 5),
                  "validation_interval": int(validation_interval) if _opt(validation_interval) is not None else None,
                  "enable_clahe": bool(enable_clahe), "rescale": bool(rescale),
                  "label": (str(label).strip() or None) if _opt(label) is not None else None,
                  "batch_size": int(batch_size or 1), "n_gpus": int(n_gpus or 1),
                  "data_source": "arrays" if arrays is not None else "artifact"}
        d = session_dir(sid)
        d.mkdir(parents=True)
        (d / TRAINING_PARAMS_FILENAME).write_text(json.dumps(params, indent=2, default=str))
        write_status(d, status_type="preparing", message="Preparing for training...", dataset_artifact_id=artifact,
                     model=model_id, n_samples=params["n_samples"], n_epochs=params["n_epochs"],
                     learning_rate=params["learning_rate"], weight_decay=params["weight_decay"],
                     min_train_masks=params["min_train_masks"], validation_interval=params["validation_interval"],
                     user_id=_user_id(context), label=params["label"], created_at=now_iso(), train_losses=[],
                     test_losses=[], test_metrics=[], n_gpus=params["n_gpus"])
        await self._launch(sid, params, arrays)
        return dict(read_status(d), session_id=sid)

    @schema_method
    async def stop_training(self, session_id: str = Field(..., description="Session id.")) -> dict:
        """Request a cooperative stop (checked after every batch)."""
        sid = normalize_session_id(session_id)
        st = read_status(session_dir(sid))
        (session_dir(sid) / "stop").touch()
        if st.get("status_type") not in ("running", "preparing", "waiting"):
            return {"session_id": sid, "status_type": st.get("status_type"), "message": "session is not running"}
        return {"session_id": sid, "status_type": "stopping", "message": "stop requested"}

    def _normalize_status(self, sid: str, st: dict) -> dict:
        tl = st.get("train_losses")
        st["current_loss"] = float(tl[-1]) if tl else st.get("current_loss")
        if str(st.get("status_type", "unknown")).lower() not in ("waiting", "preparing", "running"):
            return st
        t = self.tasks.get(sid)
        if t is not None and not t.done():
            return st
        if (session_dir(sid) / "stop").exists():
            st["status_type"], st["message"] = "stopped", "Training session stopped by user."
            return st
        age = time.time() - (session_dir(sid) / "status.json").stat().st_mtime
        if age >= STATUS_STALE_SECONDS:
            st["status_type"] = "stopped"
            st["message"] = ("Training was interrupted (likely due to service restart). Use restart_training to "
                             "resume with the saved checkpoint.")
        return st

    @schema_method
    async def get_training_status(self, session_id: str = Field(..., description="Session id.")) -> dict:
        """Status document of a session (losses, metrics, progress)."""
        sid = normalize_session_id(session_id)
        st = await asyncio.to_thread(read_status, session_dir(sid))
        return dict(self._normalize_status(sid, st), session_id=sid)

    @schema_method
    async def restart_training(
        self,
        session_id: str = Field(..., description="Stopped / failed / completed session to continue."),
        n_epochs: int | None = Field(None, description="Epochs for the continued run (default: the original)."),
        resume_optimizer: bool = Field(False, description="Also restore AdamW moments, step and RNG (exact resume)."),
        context: dict | None = Field(None, description="Injected caller context."),
    ) -> dict:
        """Start a new session from ``session_id``'s checkpoint with its saved parameters and data
        (everything is re-read from disk, so it works after replica restarts)."""
        if isinstance(session_id, dict):
            n_epochs = session_id.get("n_epochs", n_epochs)
        sid = normalize_session_id(session_id)
        st = self._normalize_status(sid, read_status(session_dir(sid)))
        if str(st.get("status_type")).lower() not in ("stopped", "unknown", "failed", "completed"):
            raise ValueError(f"Session {sid} has status '{st.get('status_type')}'. Only stopped/unknown/failed/"
                             "completed sessions can be restarted.")
        pfile = session_dir(sid) / TRAINING_PARAMS_FILENAME
        if not pfile.exists():
            raise ValueError(f"Cannot restart session {sid}: {TRAINING_PARAMS_FILENAME} not found")
        params = json.loads(pfile.read_text())
        has_ck = (session_dir(sid) / "models" / "model").exists()
        new = datetime.now(timezone.utc).strftime("%Y-%m-%d-%H%M%S") + "-" + uuid.uuid4().hex[:8]
        params.update(session_id=new, model=sid if has_ck else params.get("model", "cpsam"),
                      n_epochs=int(_opt(n_epochs) or params.get("n_epochs", 10)))
        ts = session_dir(sid) / "models" / "trainer_state.pt"
        params["resume_trainer_state"] = str(ts) if (resume_optimizer and ts.exists()) else None
        d = session_dir(new)
        d.mkdir(parents=True)
        (d / TRAINING_PARAMS_FILENAME).write_text(json.dumps(params, indent=2, default=str))
        write_status(d, status_type="preparing", message=f"Continued from {sid}", continued_from=sid,
                     last_continued_time=now_iso(), dataset_artifact_id=params.get("artifact_id"),
                     model=params["model"], n_epochs=params["n_epochs"], learning_rate=params.get("learning_rate"),
                     weight_decay=params.get("weight_decay"), label=params.get("label"),
                     user_id=_user_id(context) or st.get("user_id"), created_at=now_iso(),
                     inherited_train_losses=list(st.get("train_losses") or []),
                     inherited_test_losses=list(st.get("test_losses") or []), train_losses=[], test_losses=[],
                     test_metrics=[])
        await self._launch(new, params, source=sid if (session_dir(sid) / "pairs.json").exists() else None)
        return dict(read_status(d), session_id=new, restarted_from=sid,
                    last_continued_time=read_status(d)["last_continued_time"])

    @schema_method
    async def list_training_sessions(
        self,
        status_types: list | None = Field(None, description="Filter by status types."),
        dataset_artifact_ids: list | None = Field(None, description="Filter by dataset artifact."),
        labels: list | None = Field(None, description="Filter by label."),
        limit: int | None = Field(None, description="Most recent N sessions."),
    ) -> dict:
        """All sessions (newest first) with their status documents."""
        out = {}
        for d in sorted(sessions_root().iterdir(), reverse=True):
            if not (d / "status.json").exists() or d.name.startswith("published-"):
                continue
            st = self._normalize_status(d.name, json.loads((d / "status.json").read_text()))
            if status_types and st.get("status_type") not in status_types:
                continue
            if dataset_artifact_ids and st.get("dataset_artifact_id") not in dataset_artifact_ids:
                continue
            if labels and st.get("label") not in labels:
                continue
            out[d.name] = st
            if limit and len(out) >= limit:
                break
        return out

    @schema_method
    async def delete_training_session(self, session_id: str = Field(..., description="Session id."),
                                      context: dict | None = Field(None, description="Injected caller context.")) -> dict:
        """Delete a session (only its creator may)."""
        sid = normalize_session_id(session_id)
        st = read_status(session_dir(sid))
        uid = _user_id(context)
        if st.get("user_id") is not None and uid != st["user_id"]:  # no caller id -> refused too
            raise PermissionError(f"Session '{sid}' belongs to another user")
        t = self.tasks.get(sid)
        if t is not None and not t.done() and st.get("status_type") in ("completed", "failed", "stopped"):
            await asyncio.wait([t], timeout=30)  # final status is written just before the task returns
        if t is not None and not t.done():
            (session_dir(sid) / "stop").touch()
            raise RuntimeError("session is running; it has been asked to stop, retry the deletion when stopped")
        shutil.rmtree(session_dir(sid))
        self.tasks.pop(sid, None)
        ex = self.executors.pop(sid, None)
        if ex is not None:
            ex.shutdown(wait=False)
        return {"deleted": sid, "session_id": sid}

    # ------------------------------------------------------------------ export
    def _package(self, sid: str, out: Path, model_name: str, description: str | None, authors, uploader) -> tuple[dict, list]:
        """Write the BioImage.IO package of a session into ``out``; returns (rdf, file names)."""
        import hashlib

        import torch
        import yaml

        from bioengine_worker_amd.cellpose.model_store import load_checkpoint

        d = session_dir(sid)
        st = read_status(d)
        params = json.loads((d / TRAINING_PARAMS_FILENAME).read_text()) if (d / TRAINING_PARAMS_FILENAME).exists() else {}
        ck = torch.load(d / "models" / "model", map_location="cpu", weights_only=True)
        shutil.copy(d / "models" / "model", out / "model_weights.pth")
        shutil.copy(d / TRAINING_PARAMS_FILENAME, out / TRAINING_PARAMS_FILENAME) if (d / TRAINING_PARAMS_FILENAME).exists() \
            else (out / TRAINING_PARAMS_FILENAME).write_text("{}")
        shutil.copy(d / "status.json", out / "training_history.json")
        (out / "model.py").write_text(MODEL_PY)
        # test sample: a crop of the first training image (or synthetic) and the model's flows on it
        dev = self._device()
        net = load_checkpoint(d / "models" / "model").eval().to(dev)
        bs = int(getattr(net, "bsize", 224))
        nchan = 3 if ck["arch"] == "cpsam" else net.nchan
        x = np.zeros((1, nchan, bs, bs), np.float32)
        try:
            pairs = json.loads((d / "pairs.json").read_text())
            img = to_chw(read_image(pairs["train"][0]["image"]), nchan)
            from bioengine_worker_amd.cellpose.reference import normalize99

            img = normalize99(img)[:, :bs, :bs]
            x[0, :, : img.shape[1], : img.shape[2]] = img
        except Exception:  # noqa: BLE001
            x[0] = np.random.default_rng(0).random((nchan, bs, bs), dtype=np.float32)
        with torch.no_grad():
            y = net(torch.from_numpy(x).to(dev))[0].float().cpu().numpy()
        np.save(out / "input_sample.npy", x)
        np.save(out / "output_sample.npy", y)
        self._cover(x[0], y[0], out / "cover.png")
        tl = st.get("train_losses") or []
        (out / "README.md").write_text(
            f"# {model_name}\n\n{'Cellpose-SAM' if ck['arch'] == 'cpsam' else 'Cellpose CPnet'} model fine-tuned on "
            f"bioengine-worker-amd (MI355X).\n\n- Session: `{sid}`\n- Training images: {st.get('n_train', 'N/A')}\n"
            f"- Test images: {st.get('n_test', 0)}\n- Epochs: {st.get('total_epochs', 'N/A')}\n"
            f"- Final training loss: {tl[-1]:.4f}\n" if tl else f"# {model_name}\n")
        sha = lambda f: hashlib.sha256((out / f).read_bytes()).hexdigest()
        axes_in = [{"type": "batch"}, {"type": "channel", "channel_names": [f"c{i}" for i in range(nchan)]},
                   {"type": "space", "id": "y", "size": bs}, {"type": "space", "id": "x", "size": bs}]
        axes_out = [{"type": "batch"}, {"type": "channel", "channel_names": ["flow_y", "flow_x", "cellprob"]},
                    {"type": "space", "id": "y", "size": bs}, {"type": "space", "id": "x", "size": bs}]
        rdf = {
            "format_version": "0.5.6", "type": "model", "name": model_name,
            "description": ("Cellpose model fine-tuned on a custom dataset with bioengine-worker-amd (MI355X). "
                            + (description or "")).strip(),
            "authors": authors or [{"name": "bioengine-worker-amd"}], "uploader": uploader,
            "license": "BSD-3-Clause", "tags": ["cellpose", "segmentation", "instance-segmentation", "2d"],
            "documentation": "README.md", "covers": ["cover.png"],
            "cite": [{"text": "Pachitariu, Rariden & Stringer (2025). Cellpose-SAM.", "doi": "10.1101/2025.04.28.651001"}],
            "inputs": [{"id": "raw", "axes": axes_in, "test_tensor": {"source": "input_sample.npy",
                                                                     "sha256": sha("input_sample.npy")}}],
            "outputs": [{"id": "flows", "axes": axes_out, "test_tensor": {"source": "output_sample.npy",
                                                                         "sha256": sha("output_sample.npy")}}],
            "weights": {"pytorch_state_dict": {
                "source": "model_weights.pth", "sha256": sha("model_weights.pth"),
                "architecture": {"callable": "CellposeNet", "source": "model.py", "sha256": sha("model.py"),
                                 "kwargs": {"arch": ck["arch"], "arch_kwargs": dict(ck.get("arch_kwargs") or {})}},
                "pytorch_version": torch.__version__.split("+")[0]}},
            "training_data": {"id": params.get("artifact_id")} if params.get("artifact_id") else None,
            "training_dataset_id": params.get("artifact_id"),
            "config": {"bioengine": {"session_id": sid, "train_losses": tl, "diam_mean": 30.0,
                                     "learning_rate": params.get("learning_rate"), "n_epochs": st.get("total_epochs")}},
        }
        rdf = {k: v for k, v in rdf.items() if v is not None}
        (out / "rdf.yaml").write_text(yaml.safe_dump(json.loads(json.dumps(rdf, default=str)), sort_keys=False))
        files = ["model_weights.pth", "model.py", "input_sample.npy", "output_sample.npy", "cover.png", "README.md",
                 "rdf.yaml", TRAINING_PARAMS_FILENAME, "training_history.json"]
        return rdf, files

    @staticmethod
    def _cover(x: np.ndarray, y: np.ndarray, path: Path) -> None:
        from PIL import Image

        g = x[0]
        g = ((g - g.min()) / max(float(np.ptp(g)), 1e-6) * 255).astype(np.uint8)
        prob = 1.0 / (1.0 + np.exp(-y[2]))
        rgb = np.concatenate([np.stack([g] * 3, -1), np.stack([(prob * 255).astype(np.uint8), g // 2, g // 2], -1)], 1)
        Image.fromarray(rgb).save(path)

    @schema_method
    async def export_model(
        self,
        session_id: str = Field(..., description="Training session to export."),
        model_name: str | None = Field(None, description="Model name (default cellpose-<session prefix>)."),
        description: str | None = Field(None, description="Text appended to the RDF description."),
        authors: list | None = Field(None, description="[{name, affiliation}]"),
        uploader: dict | None = Field(None, description="{name, email}"),
        collection: str = Field(DEFAULT_COLLECTION, description="Collection artifact 'workspace/alias' to upload to."),
    ) -> dict:
        """Package the session as a BioImage.IO model (weights, model.py, test tensors, cover, docs,
        rdf.yaml) and create + upload + commit it as a model artifact in ``collection``."""
        import tempfile

        import httpx

        if isinstance(session_id, dict):
            w = session_id
            model_name, description = w.get("model_name", model_name), w.get("description", description)
            authors, uploader = w.get("authors", authors), w.get("uploader", uploader)
            collection = w.get("collection", collection)
        sid = normalize_session_id(session_id)
        st = read_status(session_dir(sid))
        if not (session_dir(sid) / "models" / "model").exists():
            raise ValueError(f"Session '{sid}' has no trained weights")
        collection = str(_opt(collection) or DEFAULT_COLLECTION)
        model_name = _opt(model_name) or f"cellpose-{sid[:8]}"
        if authors:
            for a in authors:
                if not isinstance(a, dict) or not a.get("name"):
                    raise ValueError("every author needs a 'name'")
        if uploader is not None and (not isinstance(uploader, dict) or not uploader.get("name") or
                                     not uploader.get("email")):
            raise ValueError("uploader needs 'name' and 'email'")
        out = Path(tempfile.mkdtemp(prefix=f"cellpose_export_{sid}_"))
        try:
            rdf, files = await asyncio.to_thread(self._package, sid, out, model_name, _opt(description), authors,
                                                 uploader)
            server = await self._hub()
            try:
                am = await server.get_service("public/artifact-manager")
                ws, alias = collection.split("/", 1) if "/" in collection else (None, collection)
                try:
                    col = await am.read(collection)
                except Exception as e:  # noqa: BLE001
                    raise ValueError(f"Collection '{collection}' does not exist. Please create it first or use an "
                                     "existing collection.") from e
                art = await am.create(type="model", alias=model_name, parent_id=col["id"], manifest=rdf, stage=True)
                aid = str(art["id"] if isinstance(art, dict) else art)
                async with httpx.AsyncClient(timeout=120) as c:
                    for f in files:
                        url = await am.put_file(aid, file_path=f)
                        r = await c.put(url, content=(out / f).read_bytes())
                        r.raise_for_status()
                await am.commit(aid)
                if rdf.get("training_dataset_id"):
                    try:
                        await am.edit(aid, config={"training_dataset_id": rdf["training_dataset_id"]})
                    except Exception as e:  # noqa: BLE001
                        log.warning("could not tag %s with its training dataset: %s", aid, e)
            finally:
                await server.disconnect()
            base = (st.get("server_url") or os.environ.get("HYPHA_SERVER_URL") or "").rstrip("/")
            url = f"{base}/{aid.split('/')[0]}/artifacts/{aid.split('/')[-1]}"
            write_status(session_dir(sid), exported_artifact_id=aid, model_modified=False)
            return {"artifact_id": aid, "model_name": model_name, "status": "exported", "artifact_url": url,
                    "download_url": f"{url}/create-zip-file", "files": files}
        except Exception as e:  # noqa: BLE001
            raise RuntimeError(f"Model export failed: {e}") from e
        finally:
            shutil.rmtree(out, ignore_errors=True)

    @schema_method
    async def list_models_by_dataset(
        self,
        dataset_id: str = Field(..., description="Dataset artifact id."),
        collection: str = Field(DEFAULT_COLLECTION, description="Collection to search."),
    ) -> list:
        """Exported models whose training_dataset_id is ``dataset_id``."""
        server = await self._hub()
        try:
            am = await server.get_service("public/artifact-manager")
            col = await am.read(collection)
            arts = await am.list(parent_id=col["id"], filters={"type": "model"})
        finally:
            await server.disconnect()
        base = (os.environ.get("HYPHA_SERVER_URL") or "").rstrip("/")
        out = []
        for a in arts:
            if a.get("type", "model") != "model":
                continue
            man, cfg = a.get("manifest") or {}, a.get("config") or {}
            if (man.get("training_dataset_id") or cfg.get("training_dataset_id")) == dataset_id:
                mid = a["id"]
                out.append({"id": mid, "name": a.get("alias", mid.split("/")[-1]), "created_at": a.get("created_at"),
                            "url": f"{base}/{mid.split('/')[0]}/artifacts/{mid.split('/')[-1]}"})
        return out

    @schema_method
    async def debug_task_info(self) -> dict:
        """Background training tasks and their state."""
        return {sid: {"done": t.done(), "cancelled": t.cancelled(),
                      "error": (repr(t.exception()) if t.done() and not t.cancelled() and t.exception() else None)}
                for sid, t in self.tasks.items()}

    @schema_method
    async def get_batch_stats(self) -> dict:
        """Continuous-batching statistics of inference on this replica (observability extension)."""
        from bioengine_worker_amd.serve.batching import batch_stats

        return batch_stats(self, "_segment_batch") or {}


MODEL_PY = '''"""Architecture of an exported bioengine-worker-amd Cellpose model (BioImage.IO
pytorch_state_dict ``architecture``).  Requires the ``bioengine_worker_amd`` package."""
import torch


class CellposeNet(torch.nn.Module):
    def __init__(self, arch: str = "cpsam", arch_kwargs: dict | None = None):
        super().__init__()
        from bioengine_worker_amd.cellpose.model_store import new_net

        self.net = new_net(arch, arch_kwargs or {})

    def load_state_dict(self, sd, strict: bool = True):
        if isinstance(sd, dict) and "state_dict" in sd:
            sd = sd["state_dict"]
        return self.net.load_state_dict(sd, strict=strict)

    def forward(self, x):
        return self.net(x)[0]
'''
