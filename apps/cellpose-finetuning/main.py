"""Cellpose fine-tuning + inference app on the MI355X-native Cellpose implementation.

API parity with the reference app ``apps/cellpose-finetuning/main.py`` (CellposeFinetune,
``:3633-5144``): ``start_training``, ``stop_training``, ``get_training_status``,
``restart_training``, ``list_training_sessions``, ``delete_training_session`` (owner-checked),
``export_model`` (BioImage.IO RDF + weights), ``list_models_by_dataset``, ``infer``,
``debug_task_info``.  Session layout on disk matches the reference: ``sessions/<id>/status.json``
(status_type, message, losses, metrics, progress, hyper-parameters), ``training_params.json``,
``models/model`` (weights), ``info.txt``, and a ``stop`` marker file for cooperative stops.

Compute runs on the framework's HIP kernels: inference through ``CellposeRunner`` (fused CPnet
convs, batched tiling and mask recovery) with cross-request continuous batching
(``@serve.batch``), training through ``CellposeTrainer`` (HIP augmentation, fused loss, fused
AdamW) in a background thread per session.  Built-in model: ``cyto3`` (CPnet architecture; random
initialisation offline — load real weights with ``model=<path to a cellpose state_dict>``).
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

import numpy as np
from hypha_rpc.utils.schema import schema_method
from pydantic import Field
from ray import serve

log = logging.getLogger("ray.serve")
BUILTIN_MODELS = ("cyto3",)
STATUS_TYPES = ("waiting", "preparing", "running", "completed", "failed", "stopped")


def sessions_root() -> Path:
    p = Path(os.environ.get("HOME", ".")) / "sessions"
    p.mkdir(parents=True, exist_ok=True)
    return p


def _sid(session_id: str) -> str:
    s = str(session_id).strip().replace("\\", "/")
    if s.endswith("/status.json"):
        s = s[: -len("/status.json")]
    return Path(s).name


def _now() -> str:
    return datetime.now(timezone.utc).isoformat()


def read_status(sid: str) -> dict:
    p = sessions_root() / sid / "status.json"
    if not p.exists():
        raise ValueError(f"Unknown training session '{sid}'")
    return json.loads(p.read_text())


def write_status(sid: str, **fields) -> dict:
    d = sessions_root() / sid
    d.mkdir(parents=True, exist_ok=True)
    p = d / "status.json"
    st = json.loads(p.read_text()) if p.exists() else {}
    if (d / "stop").exists() and fields.get("status_type") in ("running", "preparing"):
        fields["status_type"], fields["message"] = "stopped", "Training session stopped by user."
    st.update({k: v for k, v in fields.items() if v is not None})
    st["updated_at"] = _now()
    tmp = p.with_suffix(".tmp")
    with open(tmp, "w") as f:
        json.dump(st, f, default=float)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, p)
    return st


def _decode_image(data: bytes, name: str) -> np.ndarray:
    if name.endswith(".npy"):
        return np.load(io.BytesIO(data), allow_pickle=False)
    from PIL import Image

    img = Image.open(io.BytesIO(data))
    frames = []
    try:
        i = 0
        while True:
            img.seek(i)
            frames.append(np.array(img))
            i += 1
    except EOFError:
        pass
    return frames[0] if len(frames) == 1 else np.stack(frames)


def to_chw(img: np.ndarray, nchan: int = 2) -> np.ndarray:
    a = np.asarray(img)
    if a.ndim == 2:
        a = a[None]
    elif a.ndim == 3 and a.shape[-1] <= 4 and a.shape[0] > 4:
        a = np.moveaxis(a, -1, 0)
    if a.dtype not in (np.uint8, np.uint16, np.float16, np.float32):
        a = a.astype(np.float32)  # integer/float samples keep their width: the GPU converts
    if a.shape[0] < nchan:
        a = np.concatenate([a, np.zeros((nchan - a.shape[0],) + a.shape[1:], a.dtype)], 0)
    return np.ascontiguousarray(a[:nchan])


def clahe(img: np.ndarray, clip: float = 3.0, tiles: int = 16, device=None) -> np.ndarray:
    """Reference CLAHE pre-processing (grayscale uint8, cv2-style CLAHE 3.0 / 16x16 tiles; main.py:273-308).
    Runs the HIP kernel when ``device`` is a GPU, the numpy oracle otherwise."""
    import torch

    from bioengine_worker_amd.ops.clahe import clahe_u8, to_gray_u8

    g = torch.from_numpy(to_gray_u8(img))
    if device is not None and torch.device(device).type == "cuda":
        g = g.to(device)
    return clahe_u8(g, clip, (tiles, tiles)).cpu().numpy()


def encode_png_b64(mask: np.ndarray) -> str:
    from PIL import Image

    m = np.asarray(mask)
    img = Image.fromarray(m.astype(np.uint16 if m.max() < 65536 else np.int32))
    buf = io.BytesIO()
    img.save(buf, format="PNG")
    return base64.b64encode(buf.getvalue()).decode()


@serve.deployment(
    ray_actor_options={"num_gpus": 1, "num_cpus": 4, "memory": 12 * 1024 ** 3},
    max_ongoing_requests=64,  # >= 2 full continuous batches in flight at the replica
    max_queued_requests=256,
    health_check_period_s=30.0,
    health_check_timeout_s=60.0,
    graceful_shutdown_timeout_s=300.0,
)
class CellposeFinetune:
    def __init__(self, default_model: str = "cyto3", max_batch_size: int = 16) -> None:
        sessions_root()
        self.default_model = default_model
        self.max_batch_size = max_batch_size
        self.executors: dict[str, ThreadPoolExecutor] = {}
        self.tasks: dict[str, asyncio.Future] = {}
        self._lock = asyncio.Lock()
        self._runners: dict[str, object] = {}
        self._gpu_lock = threading.Lock()

    # ------------------------------------------------------------------ model handling
    def _device(self):
        import torch

        return torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")

    def _build_net(self, model_id: str):
        import torch

        from bioengine_worker_amd.models.cpnet import CPnet

        net = CPnet()
        if model_id in BUILTIN_MODELS:
            net.randomize_(0)
            return net
        p = sessions_root() / _sid(model_id) / "models" / "model"
        if not p.exists() and Path(model_id).exists():
            p = Path(model_id)
        if not p.exists():
            raise ValueError(f"Model identifier '{model_id}' is not a known pretrained model or session id")
        sd = torch.load(p, map_location="cpu", weights_only=True)
        net.load_state_dict(sd.get("state_dict", sd) if isinstance(sd, dict) else sd)
        return net

    @serve.multiplexed(max_num_models_per_replica=4)
    async def _runner(self, model_id: str):
        from bioengine_worker_amd.cellpose.pipeline import CellposeRunner

        net = await asyncio.to_thread(self._build_net, model_id)
        return CellposeRunner(net=net, device=self._device())

    # ------------------------------------------------------------------ lifecycle
    async def async_init(self) -> None:
        await self._runner(self.default_model)

    async def test_deployment(self) -> None:
        from bioengine_worker_amd.cellpose.pipeline import synthetic_cells

        img = synthetic_cells(1, 128, 128, ncells=8)[0]
        out = await self.infer(input_arrays=[img], model=self.default_model)
        assert out[0]["output"].shape == (128, 128)

    # ------------------------------------------------------------------ inference (continuous batching)
    @serve.batch(max_batch_size=32, batch_wait_timeout_s=0.005)
    async def _segment_batch(self, reqs: list) -> list:
        """reqs: [(model_id, image CHW, params dict, want_flows)] -> [(masks, flows | None)]."""
        from bioengine_worker_amd.profiling import trace

        out = [None] * len(reqs)
        groups: dict = {}
        for i, (mid, img, prm, want_flows) in enumerate(reqs):
            key = (mid, img.shape, img.dtype.str, tuple(sorted(prm.items())))
            groups.setdefault(key, []).append(i)
        for (mid, shape, _, prm_items), idxs in groups.items():
            runner = await self._runner(mid)
            with trace.span("app.stack", images=len(idxs)):
                batch = np.stack([reqs[i][1] for i in idxs])
            prm = dict(prm_items)
            flows_needed = any(reqs[i][3] for i in idxs)

            def run():
                with self._gpu_lock:
                    with trace.span("app.eval", images=len(idxs)):
                        m, f, _ = runner.eval(batch, **prm)
                    with trace.span("app.d2h", images=len(idxs)):
                        m = m.cpu()
                        f = f.cpu().numpy() if flows_needed else None  # 12 B/pixel D2H only on request
                return m.numpy(), f

            masks, flows = await asyncio.to_thread(run)
            for j, i in enumerate(idxs):
                out[i] = (masks[j], flows[j] if flows is not None and reqs[i][3] else None)
        return out

    async def _fetch_artifact_files(self, artifact: str, paths: list[str]) -> list[np.ndarray]:
        import httpx
        from hypha_rpc import connect_to_server

        server = await connect_to_server({"server_url": os.environ.get("HYPHA_SERVER_URL"),
                                          "token": os.environ.get("HYPHA_TOKEN")})
        try:
            am = await server.get_service("public/artifact-manager")
            out = []
            async with httpx.AsyncClient(timeout=120) as c:
                for p in paths:
                    url = await am.get_file(artifact, file_path=p)
                    r = await c.get(url)
                    r.raise_for_status()
                    out.append(_decode_image(r.content, p))
            return out
        finally:
            await server.disconnect()

    @schema_method
    async def infer(
        self,
        artifact: str | None = Field(None, description="Artifact 'workspace/alias' holding the images."),
        image_paths: list | None = Field(None, description="Image paths inside the artifact."),
        input_arrays: list | None = Field(None, description="Images as arrays ([H,W], [H,W,C] or [C,H,W])."),
        model: str = Field("cyto3", description="Built-in model name, training session id, or weights path."),
        diameter: float | None = Field(None, description="Object diameter in pixels (rescale to the model's 30 px)."),
        flow_threshold: float = Field(0.4, description="Flow error threshold (QC)."),
        cellprob_threshold: float = Field(0.0, description="Cell probability threshold."),
        niter: int | None = Field(None, description="Flow-dynamics iterations (default 200)."),
        return_flows: bool = Field(False, description="Also return dY/dX flows and cell probability."),
        json_safe: bool = Field(False, description="Return masks as base64 PNG instead of arrays."),
        enable_clahe: bool = Field(False, description="CLAHE pre-processing (brightfield)."),
    ) -> list:
        """Segment images; returns one {input_path, output(, flows)} per image."""
        if input_arrays is not None:
            images = [np.asarray(a) for a in input_arrays]
            names = [f"input_arrays[{i}]" for i in range(len(images))]
        elif artifact is not None:
            names = list(image_paths or [])
            images = await self._fetch_artifact_files(artifact, names)
        else:
            raise ValueError("Provide input_arrays or artifact + image_paths")
        if enable_clahe:
            images = [clahe(im, device=self._device()) for im in images]
        prm = {"diameter": diameter, "flow_threshold": flow_threshold, "cellprob_threshold": cellprob_threshold,
               "niter": niter or 200}
        chw = [to_chw(im) for im in images]
        res = await asyncio.gather(*[self._segment_batch((model or self.default_model, c, prm, bool(return_flows)))
                                     for c in chw])
        out = []
        for name, (m, f) in zip(names, res):
            item = {"input_path": name, "output": encode_png_b64(m) if json_safe else m.astype(np.int32)}
            if return_flows:
                item["flows"] = f.tolist() if json_safe else f
            out.append(item)
        return out

    # ------------------------------------------------------------------ training
    async def _load_training_data(self, artifact, train_images, train_annotations, train_arrays, label_arrays):
        if train_arrays is not None:
            imgs = [to_chw(a) for a in train_arrays]
            labs = [np.asarray(l).astype(np.int32) for l in label_arrays]
        else:
            if not artifact or not train_images or not train_annotations:
                raise ValueError("Provide train_arrays/label_arrays or artifact + train_images + train_annotations")
            raw = await self._fetch_artifact_files(artifact, list(train_images))
            lab = await self._fetch_artifact_files(artifact, list(train_annotations))
            imgs = [to_chw(a) for a in raw]
            labs = [np.asarray(l).astype(np.int32) for l in lab]
        if len(imgs) != len(labs):
            raise ValueError(f"{len(imgs)} images but {len(labs)} annotations")
        return imgs, labs

    def _train_blocking(self, sid: str, imgs, labs, test_imgs, test_labs, params: dict, resume: dict | None):
        import torch

        from bioengine_worker_amd.cellpose.reference import normalize99
        from bioengine_worker_amd.train.cellpose_train import TrainConfig, build_trainer, labels_to_flows, run_training

        dev = self._device()
        try:
            write_status(sid, status_type="preparing", message="Computing flow targets")
            keep = [i for i, l in enumerate(labs) if len(np.unique(l)) - 1 >= params["min_train_masks"]]
            if not keep:
                raise ValueError("no training image has enough masks")
            imgs = [imgs[i] for i in keep]
            labs = [labs[i] for i in keep]
            Hm = min(i.shape[1] for i in imgs)
            Wm = min(i.shape[2] for i in imgs)

            def prep(ims, lbs):
                x = torch.from_numpy(np.stack([normalize99(i[:, :Hm, :Wm]) for i in ims])).float().to(dev)
                lab = torch.from_numpy(np.stack([l[:Hm, :Wm] for l in lbs])).to(dev)
                return x, labels_to_flows(lab)

            tx, tl = prep(imgs, labs)
            vx, vl = prep(test_imgs, test_labs) if test_imgs else (None, None)
            bsize = min(params.get("bsize", 256), Hm, Wm)
            cfg = TrainConfig(batch_size=params["batch_size"], bsize=bsize, lr=params["learning_rate"],
                              weight_decay=params["weight_decay"], validation_interval=params["validation_interval"],
                              min_train_masks=params["min_train_masks"])
            net = self._build_net(params["model"])
            trainer = build_trainer(cfg, dev, net=net)
            start_epoch = 0
            if resume is not None:
                trainer.load_state_dict(resume)
            hist = read_status(sid)
            write_status(sid, status_type="running", message="Training", n_train=len(imgs),
                         n_test=len(test_imgs or []), total_epochs=params["n_epochs"], start_time=hist.get("start_time") or _now())
            losses_prev = list(hist.get("train_losses") or [])
            stop_file = sessions_root() / sid / "stop"
            t_last = [0.0]

            def on_batch(ep, k, nb, loss, el, _):
                if time.time() - t_last[0] > 1.0 or k == nb - 1:
                    t_last[0] = time.time()
                    write_status(sid, current_epoch=ep, current_batch=k + 1, total_batches=nb, elapsed_seconds=el,
                                 current_loss=float(loss))

            def on_epoch(ep, tr, te, el, metrics):
                st = read_status(sid)
                tl_ = list(st.get("train_losses") or losses_prev) + [float(tr)]
                tm = list(st.get("test_metrics") or []) + [metrics]
                write_status(sid, train_losses=tl_, test_losses=list(st.get("test_losses") or []) + [te],
                             test_metrics=tm, current_epoch=ep, elapsed_seconds=el)
                mdir = sessions_root() / sid / "models"
                mdir.mkdir(exist_ok=True)
                torch.save({"state_dict": trainer.net.state_dict()}, mdir / "model")
                torch.save(trainer.state_dict(), mdir / "trainer_state.pt")

            out = run_training(trainer, tx, tl, params["n_epochs"], vx, vl, batch_callback=on_batch,
                               epoch_callback=on_epoch, stop_check=stop_file.exists, start_epoch=start_epoch)
            mdir = sessions_root() / sid / "models"
            mdir.mkdir(exist_ok=True)
            torch.save({"state_dict": trainer.net.state_dict()}, mdir / "model")
            torch.save(trainer.state_dict(), mdir / "trainer_state.pt")
            if out.get("stopped"):
                write_status(sid, status_type="stopped", message="Training session stopped by user.")
            else:
                if test_imgs:
                    write_status(sid, message="Computing instance metrics on the test images")
                    try:
                        write_status(sid, instance_metrics=self._instance_metrics(trainer.net, test_imgs, test_labs, dev))
                    except Exception as e:  # noqa: BLE001 — metrics are best-effort, as in the reference
                        log.warning("session %s: could not compute instance metrics: %s", sid, e)
                write_status(sid, status_type="completed", message="Training completed", model_modified=True)
        except Exception as e:  # noqa: BLE001
            log.exception("training failed")
            write_status(sid, status_type="failed", message=f"{type(e).__name__}: {e}")

    @staticmethod
    def _instance_metrics(net, test_imgs, test_labs, dev) -> dict:
        """Full Cellpose eval of the fine-tuned net on every test image, then image-mean AP at IoU
        0.5 / 0.75 / 0.9 (reference main.py:1977-2029, cellpose metrics.average_precision)."""
        from bioengine_worker_amd.cellpose.metrics import instance_metrics
        from bioengine_worker_amd.cellpose.pipeline import CellposeRunner

        net.eval()
        runner = CellposeRunner(net=net, device=dev)
        preds = []
        for img in test_imgs:
            masks, _, _ = runner.eval(np.asarray(img)[None])
            preds.append(masks[0].cpu())
        return instance_metrics([np.asarray(l, np.int32) for l in test_labs], [p.numpy() for p in preds])

    async def _launch(self, sid: str, imgs, labs, test_imgs, test_labs, params: dict, resume=None):
        ex = ThreadPoolExecutor(max_workers=1, thread_name_prefix=f"train-{sid[:8]}")
        self.executors[sid] = ex
        if not hasattr(self, "_cached_data"):
            self._cached_data = {}
        self._cached_data[sid] = (imgs, labs, test_imgs, test_labs)  # enables restart_training
        loop = asyncio.get_running_loop()
        self.tasks[sid] = loop.run_in_executor(ex, self._train_blocking, sid, imgs, labs, test_imgs, test_labs,
                                               params, resume)

    @schema_method
    async def start_training(
        self,
        artifact: str | None = Field(None, description="Dataset artifact 'workspace/alias'."),
        train_images: list | None = Field(None, description="Training image paths in the artifact."),
        train_annotations: list | None = Field(None, description="Label-image paths (same order as train_images)."),
        test_images: list | None = Field(None, description="Validation image paths."),
        test_annotations: list | None = Field(None, description="Validation label paths."),
        train_arrays: list | None = Field(None, description="Training images as arrays (instead of an artifact)."),
        label_arrays: list | None = Field(None, description="Instance label arrays for train_arrays."),
        test_arrays: list | None = Field(None, description="Validation images as arrays (instead of test_images)."),
        test_label_arrays: list | None = Field(None, description="Instance label arrays for test_arrays."),
        model: str = Field("cyto3", description="Initial model (built-in name or session id)."),
        n_epochs: int = Field(10, description="Epochs."),
        learning_rate: float = Field(1e-6, description="AdamW learning rate."),
        weight_decay: float = Field(1e-4, description="AdamW weight decay."),
        batch_size: int = Field(8, description="Crops per step."),
        min_train_masks: int = Field(5, description="Drop training images with fewer masks."),
        validation_interval: int = Field(10, description="Validate every N epochs (and at epoch 1)."),
        enable_clahe: bool = Field(False, description="CLAHE pre-processing."),
        label: str | None = Field(None, description="Free-form session label."),
        context: dict | None = Field(None, description="Injected caller context."),
    ) -> dict:
        """Start a fine-tuning session in the background; returns {session_id}."""
        imgs, labs = await self._load_training_data(artifact, train_images, train_annotations, train_arrays, label_arrays)
        test_imgs, test_labs = [], []
        if test_images and test_annotations and artifact:
            test_imgs, test_labs = await self._load_training_data(artifact, test_images, test_annotations, None, None)
        elif test_arrays and test_label_arrays:
            test_imgs, test_labs = await self._load_training_data(None, None, None, test_arrays, test_label_arrays)
        if enable_clahe:
            imgs = [to_chw(clahe(i, device=self._device())) for i in imgs]
        sid = f"{datetime.now().strftime('%Y-%m-%d-%H%M%S')}-{uuid.uuid4().hex[:8]}"
        uid = (context or {}).get("user", {}).get("id")
        params = {"model": model, "n_epochs": n_epochs, "learning_rate": learning_rate, "weight_decay": weight_decay,
                  "batch_size": batch_size, "min_train_masks": min_train_masks,
                  "validation_interval": validation_interval, "bsize": 256}
        d = sessions_root() / sid
        d.mkdir(parents=True)
        (d / "training_params.json").write_text(json.dumps(dict(params, artifact=artifact, label=label), default=str))
        write_status(sid, status_type="waiting", message="Queued", dataset_artifact_id=artifact, user_id=uid,
                     label=label, model=model, n_epochs=n_epochs, learning_rate=learning_rate,
                     weight_decay=weight_decay, created_at=_now(), train_losses=[], test_losses=[], test_metrics=[])
        async with self._lock:
            await self._launch(sid, imgs, labs, test_imgs, test_labs, params)
        return {"session_id": sid}

    @schema_method
    async def stop_training(self, session_id: str = Field(..., description="Session id.")) -> dict:
        """Request a cooperative stop (checked after every batch)."""
        sid = _sid(session_id)
        read_status(sid)
        (sessions_root() / sid / "stop").touch()
        return {"session_id": sid, "message": "stop requested"}

    @schema_method
    async def get_training_status(self, session_id: str = Field(..., description="Session id.")) -> dict:
        """Status document of a session (losses, metrics, progress)."""
        sid = _sid(session_id)
        st = read_status(sid)
        tl = st.get("train_losses") or []
        st.setdefault("current_loss", float(tl[-1]) if tl else None)
        if st.get("status_type") in ("waiting", "preparing", "running"):
            t = self.tasks.get(sid)
            if t is None or t.done():
                age = time.time() - (sessions_root() / sid / "status.json").stat().st_mtime
                if age > 300:
                    st["status_type"], st["message"] = "failed", "Session is stale (no active training task)."
        st["session_id"] = sid
        return st

    @schema_method
    async def restart_training(self, session_id: str = Field(..., description="Session to continue."),
                               n_epochs: int | None = Field(None, description="Epochs for the continued run."),
                               context: dict | None = Field(None, description="Injected caller context.")) -> dict:
        """Continue a session from its last checkpoint (optimizer state and RNG restored exactly)."""
        import torch

        sid = _sid(session_id)
        st = read_status(sid)
        params = json.loads((sessions_root() / sid / "training_params.json").read_text())
        ts = sessions_root() / sid / "models" / "trainer_state.pt"
        if not ts.exists():
            raise ValueError(f"Session '{sid}' has no checkpoint")
        raise_if_running = self.tasks.get(sid)
        if raise_if_running is not None and not raise_if_running.done():
            raise RuntimeError(f"Session '{sid}' is still running")
        resume = torch.load(ts, map_location="cpu", weights_only=True)
        new = f"{datetime.now().strftime('%Y-%m-%d-%H%M%S')}-{uuid.uuid4().hex[:8]}"
        shutil.copytree(sessions_root() / sid, sessions_root() / new)
        (sessions_root() / new / "stop").unlink(missing_ok=True)
        params["n_epochs"] = int(n_epochs or params["n_epochs"])
        (sessions_root() / new / "training_params.json").write_text(json.dumps(params))
        write_status(new, status_type="waiting", message=f"Continued from {sid}", continued_from=sid,
                     last_continued_time=_now(), n_epochs=params["n_epochs"])
        data = self._cached_data.get(sid) if hasattr(self, "_cached_data") else None
        if data is None:
            raise ValueError("training data for the original session is no longer cached; start a new session")
        await self._launch(new, *data, params, resume)
        return {"session_id": new, "continued_from": sid}

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
            if not (d / "status.json").exists():
                continue
            st = json.loads((d / "status.json").read_text())
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
        sid = _sid(session_id)
        st = read_status(sid)
        uid = (context or {}).get("user", {}).get("id")
        if st.get("user_id") and uid and st["user_id"] != uid:
            raise PermissionError(f"Session '{sid}' belongs to another user")
        t = self.tasks.get(sid)
        if t is not None and not t.done() and st.get("status_type") in ("completed", "failed", "stopped"):
            # the final status is written before the task returns: let it finish its teardown
            await asyncio.wait([t], timeout=30)
        if t is not None and not t.done():
            (sessions_root() / sid / "stop").touch()
            raise RuntimeError("session is running; it has been asked to stop, retry the deletion when stopped")
        shutil.rmtree(sessions_root() / sid)
        return {"deleted": sid}

    @schema_method
    async def list_models_by_dataset(self, dataset_id: str = Field(..., description="Dataset artifact id.")) -> list:
        """Completed sessions trained on a dataset."""
        res = []
        for sid, st in (await self.list_training_sessions(dataset_artifact_ids=[dataset_id])).items():
            if st.get("status_type") == "completed":
                res.append({"session_id": sid, "label": st.get("label"), "train_losses": st.get("train_losses")})
        return res

    @schema_method
    async def export_model(self, session_id: str = Field(..., description="Completed session."),
                           model_name: str | None = Field(None, description="Model name."),
                           description: str | None = Field(None, description="Model description."),
                           authors: list | None = Field(None, description="[{name, affiliation}]"),
                           uploader: dict | None = Field(None, description="{email, name}"),
                           collection: str | None = Field(None, description="Target collection artifact id.")) -> dict:
        """Package a trained session as a BioImage.IO model (rdf.yaml 0.5 + state_dict) under the session dir."""
        import hashlib

        import yaml

        sid = _sid(session_id)
        st = read_status(sid)
        w = sessions_root() / sid / "models" / "model"
        if not w.exists():
            raise ValueError(f"Session '{sid}' has no trained weights")
        out = sessions_root() / sid / "export"
        out.mkdir(exist_ok=True)
        shutil.copy(w, out / "weights.pt")
        sha = hashlib.sha256((out / "weights.pt").read_bytes()).hexdigest()
        rdf = {"format_version": "0.5.6", "type": "model", "name": model_name or f"cellpose-{sid}",
               "description": description or "Cellpose CPnet fine-tuned on bioengine-worker-amd (MI355X)",
               "authors": authors or [{"name": "bioengine-worker-amd"}], "uploader": uploader,
               "license": "MIT", "tags": ["cellpose", "segmentation", "instance-segmentation"],
               "inputs": [{"id": "raw", "axes": [{"type": "batch"}, {"type": "channel", "channel_names": ["c0", "c1"]},
                                                  {"type": "space", "id": "y", "size": {"min": 16, "step": 16}},
                                                  {"type": "space", "id": "x", "size": {"min": 16, "step": 16}}]}],
               "outputs": [{"id": "flows", "axes": [{"type": "batch"}, {"type": "channel",
                                                                        "channel_names": ["dy", "dx", "cellprob"]},
                                                    {"type": "space", "id": "y"}, {"type": "space", "id": "x"}]}],
               "weights": {"pytorch_state_dict": {"source": "weights.pt", "sha256": sha,
                                                  "architecture": {"callable": "CPnet",
                                                                   "import_from": "bioengine_worker_amd.models.cpnet",
                                                                   "kwargs": {}}}},
               "config": {"bioengine": {"session_id": sid, "train_losses": st.get("train_losses")}}}
        (out / "rdf.yaml").write_text(yaml.safe_dump(rdf, sort_keys=False))
        return {"session_id": sid, "path": str(out), "files": sorted(p.name for p in out.iterdir()),
                "collection": collection}

    @schema_method
    async def debug_task_info(self) -> dict:
        """Background training tasks and their state."""
        return {sid: {"done": t.done(), "cancelled": t.cancelled()} for sid, t in self.tasks.items()}

    @schema_method
    async def get_batch_stats(self) -> dict:
        """Continuous-batching statistics of inference on this replica (batch-size histogram,
        mean queue wait) — observability extension, not in the reference."""
        from bioengine_worker_amd.serve.batching import batch_stats

        return batch_stats(self, "_segment_batch") or {}
