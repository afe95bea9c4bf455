"""One cellpose fine-tuning session, end to end, on local files -- the body of ``start_training``.

The reference runs ``finetune_cellpose`` -> ``train_seg_with_callbacks`` in a one-thread executor
inside its single GPU replica (``apps/cellpose-finetuning/main.py:1716-2201``).  Here the same session
body is a plain function of ``(session_dir, params)`` so it runs either

* in a thread of the app replica (one GPU), or
* as every rank of a gang-scheduled multi-GPU job (``serve/gang.py``): each rank calls
  :func:`train_session` with its ``rank``/``world``; the trainer all-reduces gradient buckets over
  RCCL (``nccl``) or gloo, rank 0 alone writes status, checkpoints and metrics.

Session directory layout (reference-compatible): ``status.json`` (status_type, message, losses,
metrics, progress), ``training_params.json``, ``pairs.json`` (local image/annotation files),
``models/model`` (checkpoint: arch + state_dict), ``models/trainer_state.pt`` (exact resume),
``info.txt`` and a ``stop`` marker for cooperative stops.
"""
from __future__ import annotations

import json
import logging
import os
import time
from datetime import datetime, timezone
from pathlib import Path

import numpy as np
import torch

log = logging.getLogger("bioengine.train.session")
STATUS_TYPES = ("waiting", "preparing", "running", "completed", "failed", "stopped", "unknown")


def _save_atomic(obj, path: Path) -> None:
    """torch.save to a temporary file in the same directory, then rename it over ``path``: a rank
    that dies mid-write (what elastic restart recovers from) never leaves a truncated resume state."""
    path = Path(path)
    tmp = path.with_name(f"{path.name}.tmp{os.getpid()}")
    torch.save(obj, tmp)
    os.replace(tmp, path)


def now_iso() -> str:
    return datetime.now(timezone.utc).isoformat()


def read_status(session_dir: Path) -> dict:
    p = Path(session_dir) / "status.json"
    if not p.exists():
        raise ValueError(f"Unknown training session '{Path(session_dir).name}'")
    return json.loads(p.read_text())


def write_status(session_dir: Path, **fields) -> dict:
    """Merge ``fields`` into status.json atomically (tmp + fsync + rename, reference main.py:1155)."""
    d = Path(session_dir)
    d.mkdir(parents=True, exist_ok=True)
    p = d / "status.json"
    st = json.loads(p.read_text()) if p.exists() else {}
    if (d / "stop").exists() and fields.get("status_type") in ("running", "preparing"):
        fields["status_type"], fields["message"] = "stopped", "Training session stopped by user."
    st.update({k: v for k, v in fields.items() if v is not None})
    st["updated_at"] = now_iso()
    tmp = p.with_name(f"status.{os.getpid()}.tmp")
    with open(tmp, "w") as f:
        json.dump(st, f, default=float)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, p)
    return st


def log_info(session_dir: Path, msg: str) -> None:
    with open(Path(session_dir) / "info.txt", "a") as f:
        f.write(f"{now_iso()} {msg}\n")


def cell_diameter(labels: np.ndarray) -> float:
    """cellpose ``utils.diameters``: median sqrt(area) / (sqrt(pi) / 2) over the instances."""
    _, counts = np.unique(labels.astype(np.int32), return_counts=True)
    counts = counts[1:]
    if counts.size == 0:
        return 0.0
    return float(np.median(np.sqrt(counts)) / (np.sqrt(np.pi) / 2))


def to_chw(img: np.ndarray, nchan: int) -> np.ndarray:
    a = np.asarray(img)
    if a.ndim == 2:
        a = a[None]
    elif a.ndim == 3 and a.shape[-1] <= 4 and a.shape[0] > 4:
        a = np.moveaxis(a, -1, 0)
    a = a.astype(np.float32)
    if a.shape[0] < nchan:
        a = np.concatenate([a, np.zeros((nchan - a.shape[0],) + a.shape[1:], np.float32)], 0)
    return np.ascontiguousarray(a[:nchan])


def load_pairs(pairs: list[dict], nchan: int, enable_clahe: bool = False, device=None):
    """Local (image, annotation) files -> lists of CHW float images and int32 label maps."""
    from ..cellpose.datasets import read_image, read_labels

    imgs, labs = [], []
    for pr in pairs:
        im = read_image(pr["image"])
        if enable_clahe:
            from ..ops.clahe import clahe_u8, to_gray_u8

            g = torch.from_numpy(to_gray_u8(im))
            if device is not None and torch.device(device).type == "cuda":
                g = g.to(device)
            im = clahe_u8(g, 3.0, (16, 16)).cpu().numpy()
        imgs.append(to_chw(im, nchan))
        lab = read_labels(pr["annotation"])
        if lab.shape != imgs[-1].shape[1:]:
            raise ValueError(f"annotation {pr['annotation']} shape {lab.shape} != image {imgs[-1].shape[1:]}")
        labs.append(lab)
    return imgs, labs


def _prep(imgs, labs, device):
    """normalize99 per image (cellpose ``normalize_img``) + labels -> [instances, flowY, flowX] on device."""
    from ..cellpose.reference import normalize99
    from .cellpose_train import labels_to_flows

    xs, ys = [], []
    for im, lab in zip(imgs, labs):
        xs.append(torch.from_numpy(normalize99(im)).float().to(device))
        ys.append(labels_to_flows(torch.from_numpy(lab.astype(np.int32))[None].to(device))[0])
    return xs, ys


def train_session(session_dir: str | Path, params: dict, device=None, rank: int = 0, world: int = 1,
                  group=None, cpsam_arch: str = "vit_l") -> dict:
    """Run one fine-tuning session (blocking).  ``params``: the session's training_params plus
    ``model`` (built-in / session id / checkpoint path).  Returns the final status dict (rank 0)."""
    from ..cellpose.model_store import resolve_net, save_checkpoint
    from .cellpose_train import TrainConfig, build_trainer, run_training

    sdir = Path(session_dir)
    lead = rank == 0
    dev = torch.device(device) if device is not None else (
        torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
    stop_file = sdir / "stop"
    try:
        pairs = json.loads((sdir / "pairs.json").read_text())
        net, weights = resolve_net(params["model"], sdir.parent, cpsam_arch)
        nchan = 3 if type(net).__name__ == "CPSAM" else net.nchan
        if lead:
            write_status(sdir, status_type="preparing", message="Loading training data", init_weights=weights)
        imgs, labs = load_pairs(pairs["train"], nchan, params.get("enable_clahe", False), dev)
        timgs, tlabs = load_pairs(pairs.get("test") or [], nchan, params.get("enable_clahe", False), dev)
        mtm = int(params.get("min_train_masks", 5))
        keep = [i for i, l in enumerate(labs) if len(np.unique(l)) - 1 >= mtm]
        if not keep:
            raise ValueError(f"no training image has at least min_train_masks={mtm} masks")
        imgs, labs = [imgs[i] for i in keep], [labs[i] for i in keep]
        diams = [cell_diameter(l) for l in labs]
        tx, tl = _prep(imgs, labs, dev)
        vx, vl = _prep(timgs, tlabs, dev) if timgs else (None, None)
        with torch.no_grad():
            net.diam_labels.fill_(float(np.mean(diams)) if diams else 30.0)
        bsize = int(getattr(net, "bsize", 0) or params.get("bsize", 256))
        cfg = TrainConfig(batch_size=int(params.get("batch_size", 1)), bsize=bsize,
                          lr=float(params.get("learning_rate", 1e-6)),
                          weight_decay=float(params.get("weight_decay", 1e-4)),
                          validation_interval=int(params.get("validation_interval") or 10), min_train_masks=mtm,
                          seed=int(params.get("seed", 0)))
        trainer = build_trainer(cfg, dev, world_size=world, rank=rank, net=net, group=group)
        resume = params.get("resume_trainer_state")
        if resume and Path(resume).exists():
            trainer.load_state_dict(torch.load(resume, map_location="cpu", weights_only=True))
        # "continue": the SAME session picks up after its last completed epoch (elastic restart of a
        # data-parallel gang at a smaller world); otherwise a resumed state seeds a new session
        start_epoch = trainer.epoch if (params.get("continue_session") and resume and Path(resume).exists()) else 0
        trainer.epoch = start_epoch
        n_epochs = int(params.get("n_epochs", 10))
        hist = read_status(sdir)
        prev_losses = list(hist.get("inherited_train_losses") or [])
        if lead and start_epoch > 0:
            st = read_status(sdir)
            write_status(sdir, status_type="running", message=f"Training (resumed at epoch {start_epoch}, world {world})",
                         world_size=world, train_losses=list(st.get("train_losses") or [])[:start_epoch + len(prev_losses)],
                         test_losses=list(st.get("test_losses") or [])[:start_epoch + len(prev_losses)],
                         test_metrics=list(st.get("test_metrics") or [])[:start_epoch])
            log_info(sdir, f"resumed at epoch {start_epoch} with world {world}")
        elif lead:
            write_status(sdir, status_type="running", message="Training", n_train=len(imgs), n_test=len(timgs),
                         total_epochs=n_epochs, start_time=hist.get("start_time") or now_iso(), world_size=world,
                         train_losses=prev_losses, test_losses=list(hist.get("inherited_test_losses") or []),
                         test_metrics=[])
            log_info(sdir, f"training {params['model']} on {len(imgs)} images ({len(timgs)} test), "
                           f"{n_epochs} epochs, world {world}, device {dev}")
        t_last = [0.0]
        t_start = time.time()

        fi = params.get("fault_injection") or {}
        kill_at = int(fi.get("at_batch", -1)) if (fi.get("kill_rank") == rank and not params.get("continue_session")) else -1
        nstep = [0]

        def on_batch(ep, k, nb, loss, el, _):
            nstep[0] += 1
            if nstep[0] == kill_at:  # test hook: this rank crashes like a lost GPU / OOM-killed process
                os._exit(137)
            if lead and (time.time() - t_last[0] > 1.0 or k == nb - 1):
                t_last[0] = time.time()
                write_status(sdir, current_epoch=ep, current_batch=k + 1, total_batches=nb, elapsed_seconds=el,
                             current_loss=float(loss))

        def on_epoch(ep, tr, te, el, metrics):
            if not lead:
                return
            st = read_status(sdir)
            write_status(sdir, train_losses=list(st.get("train_losses") or []) + [float(tr)],
                         test_losses=list(st.get("test_losses") or []) + [te],
                         test_metrics=list(st.get("test_metrics") or []) + [metrics], current_epoch=ep,
                         elapsed_seconds=el, samples_per_sec=round(ep * len(imgs) / max(el, 1e-9), 3))
            save_checkpoint(sdir / "models" / "model", trainer.net)
            _save_atomic(trainer.state_dict(), sdir / "models" / "trainer_state.pt")

        out = run_training(trainer, tx, tl, n_epochs, vx, vl, batch_callback=on_batch, epoch_callback=on_epoch,
                           stop_check=stop_file.exists, diams=diams, rescale=bool(params.get("rescale", False)),
                           start_epoch=start_epoch)
        digest = weights_digest(trainer)
        if not lead:
            return {"rank": rank, "weights_sha256": digest}
        write_status(sdir, weights_sha256=digest)
        save_checkpoint(sdir / "models" / "model", trainer.net)
        _save_atomic(trainer.state_dict(), sdir / "models" / "trainer_state.pt")
        if out.get("stopped"):
            return write_status(sdir, status_type="stopped", message="Training session stopped by user.")
        if timgs:
            write_status(sdir, message="Computing instance metrics on the test images")
            try:
                write_status(sdir, instance_metrics=instance_metrics(trainer.net, timgs, tlabs, dev))
            except Exception as e:  # noqa: BLE001 -- metrics are best effort, as in the reference
                log.warning("instance metrics failed: %s", e)
        log_info(sdir, f"completed in {time.time() - t_start:.1f} s")
        return write_status(sdir, status_type="completed", message="Training completed", model_modified=True)
    except Exception as e:  # noqa: BLE001
        log.exception("training session %s failed", sdir.name)
        if lead and world > 1 and _is_peer_failure(e):
            # a collective failed because another rank died: the gang supervisor decides (elastic
            # restart at world - 1, run_dp_session); do not mark the session failed
            write_status(sdir, message=f"collective failed ({type(e).__name__}); waiting for the gang supervisor")
            raise
        if lead:
            return write_status(sdir, status_type="failed", message=f"{type(e).__name__}: {e}")
        raise


def _is_peer_failure(e: BaseException) -> bool:
    import torch.distributed as dist

    if isinstance(e, tuple(t for t in (getattr(dist, "DistBackendError", None), getattr(dist, "DistNetworkError", None))
                          if t is not None)):
        return True
    msg = str(e).lower()
    return any(k in msg for k in ("connection closed", "connection reset", "gloo", "nccl", "rccl", "broken pipe",
                                  "peer", "timed out"))


async def run_dp_session(session_dir: str | Path, params: dict, n_gpus: int, cpsam_arch: str = "vit_l",
                         max_restarts: int | None = None, name: str | None = None, gpus_per_rank: int = 1) -> list:
    """Data-parallel session as a gang (``serve/gang.py``) with elastic restart.

    When a rank dies (process exit, signal, OOM kill) the gang supervisor tears the whole job down;
    a FRESH gang of ``world - 1`` processes is then started from the session's last
    ``models/trainer_state.pt`` (weights, AdamW moments, step, RNG, completed epochs) and continues
    the same session -- never an exec of a process that used the GPU.  Per-rank batch stays fixed,
    so the global batch shrinks with the world.  A user stop or an error the lead rank recorded is
    not retried.  Returns the final gang's per-rank results."""
    from ..serve.gang import GangError, run_gang

    sdir = Path(session_dir)
    world = int(n_gpus)
    restarts = 0
    max_restarts = max(0, world - 1) if max_restarts is None else int(max_restarts)
    p = dict(params)
    while True:
        try:
            return await run_gang("bioengine_worker_amd.train.session:train_session_rank",
                                  {"session_dir": str(sdir), "params": p, "cpsam_arch": cpsam_arch},
                                  world_size=world, gpus_per_rank=gpus_per_rank, cpus_per_rank=1.0,
                                  timeout_s=p.get("timeout_s"), name=(name or "train") + (f"-r{restarts}" if restarts else ""))
        except GangError as e:
            st = read_status(sdir)
            if (sdir / "stop").exists() or st.get("status_type") in ("failed", "stopped", "completed") \
                    or world <= 1 or restarts >= max_restarts:
                raise
            ckpt = sdir / "models" / "trainer_state.pt"
            restarts += 1
            world -= 1
            if ckpt.exists():
                p["resume_trainer_state"] = str(ckpt)
                p["continue_session"] = True
            log.warning("session %s: gang failed (%s); elastic restart %d at world %d", sdir.name,
                        str(e).splitlines()[0], restarts, world)
            write_status(sdir, message=f"Rank failure; restarting at world {world} from "
                                       f"{'epoch ' + str(_ckpt_epoch(ckpt)) if ckpt.exists() else 'the start'}",
                         elastic_restarts=restarts, world_size=world,
                         elastic_events=list(st.get("elastic_events") or []) + [
                             {"time": now_iso(), "error": str(e).splitlines()[0][:300], "new_world": world}])


def _ckpt_epoch(ckpt: Path) -> int:
    try:
        return int(torch.load(ckpt, map_location="cpu", weights_only=True).get("epoch", 0))
    except Exception:  # noqa: BLE001
        return 0


def weights_digest(trainer) -> str:
    import hashlib

    return hashlib.sha256(trainer.fp.flat.detach().cpu().numpy().tobytes()).hexdigest()


def train_session_rank(rank: int, world: int, session_dir: str, params: dict, cpsam_arch: str = "vit_l") -> dict:
    """Gang target (``serve/gang.py``): one data-parallel rank of a fine-tuning session.  The
    process group is already initialised (RCCL with GPUs, gloo otherwise)."""
    import torch.distributed as dist

    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    st = train_session(session_dir, params, dev, rank=rank, world=world, cpsam_arch=cpsam_arch)
    return {"rank": rank, "weights_sha256": st.get("weights_sha256"), "status_type": st.get("status_type")}


def instance_metrics(net, test_imgs, test_labs, device) -> dict:
    """Full Cellpose eval of the fine-tuned net on every test image, then AP at IoU 0.5/0.75/0.9
    (reference main.py:1977-2029)."""
    from ..cellpose.metrics import instance_metrics as im
    from ..cellpose.pipeline import CellposeRunner

    runner = CellposeRunner(net=net.eval(), device=device)
    preds = []
    for img in test_imgs:
        masks, _, _ = runner.eval(np.asarray(img)[None])
        preds.append(masks[0].cpu().numpy())
    return im([np.asarray(l, np.int32) for l in test_labs], preds)
