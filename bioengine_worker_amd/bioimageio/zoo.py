"""Model zoo access and the on-disk model cache (reference ModelCache,
apps/model-runner/entry_deployment.py:72-1009).

Sources, in order: a local zoo directory (``BIOENGINE_MODEL_ZOO``: one sub-directory per model id
holding ``rdf.yaml`` and its files — the offline stand-in for bioimage.io), then the hub's
artifact manager collection ``bioimage-io/bioimage.io`` (files fetched through presigned URLs).
The cache keeps one directory per model id under ``cache_dir`` with the reference's
cross-replica coordination: atomic ``os.rename`` publication of a finished download, a
``.downloading`` marker other replicas wait on, ``.last_access`` files for LRU eviction, and
in-use leases that make a package non-evictable while a request holds it.

Crash recovery (reference ``entry_deployment.py:384-411, 833-837``): leases and download markers
record their owner (host, pid) and start time.  A lease older than :data:`LEASE_MAX_AGE_S` or whose
owner process on this host has exited no longer blocks eviction; a download marker whose owner has
exited, or that is older than :data:`DOWNLOAD_TIMEOUT_S`, is removed and the download claimed again --
a replica that dies mid-download no longer leaves every later request waiting out the timeout.
"""
from __future__ import annotations

import asyncio
import json
import os
import shutil
import time
from pathlib import Path

import socket
import uuid

import yaml

#: an in-use lease older than this no longer blocks eviction (the reference's 10 minutes)
LEASE_MAX_AGE_S = 600.0
#: a download marker older than this is stale whatever its owner
DOWNLOAD_TIMEOUT_S = float(os.environ.get("BIOENGINE_MODEL_DOWNLOAD_TIMEOUT_S", "1800"))
_HOST = socket.gethostname()


def _owner() -> dict:
    return {"host": _HOST, "pid": os.getpid(), "t": time.time()}


def _pid_alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    return True


def _owner_stale(info: dict | None, max_age: float, mtime: float) -> bool:
    """An owner record is stale when its process (on this host) is gone or it is older than max_age."""
    t = float(info.get("t", mtime)) if info else mtime
    if time.time() - t > max_age:
        return True
    if info and info.get("host") == _HOST and isinstance(info.get("pid"), int):
        return not _pid_alive(int(info["pid"]))
    return False


def _read_owner(p: Path) -> dict | None:
    try:
        return json.loads(p.read_text())
    except (OSError, ValueError):
        return None


def lease_live(p: Path) -> bool:
    try:
        mt = p.stat().st_mtime
    except OSError:
        return False
    return not _owner_stale(_read_owner(p), LEASE_MAX_AGE_S, mt)


def local_zoo_root() -> Path | None:
    p = os.environ.get("BIOENGINE_MODEL_ZOO")
    return Path(p) if p and Path(p).is_dir() else None


def list_local_models() -> dict[str, dict]:
    root = local_zoo_root()
    out = {}
    if root is None:
        return out
    for d in sorted(root.iterdir()):
        f = d / "rdf.yaml"
        if f.exists():
            try:
                rdf = yaml.safe_load(f.read_text())
            except Exception:  # noqa: BLE001
                continue
            out[str(rdf.get("id") or d.name)] = {"dir": d, "rdf": rdf}
    return out


def search_local(keywords: list[str] | None, limit: int = 10) -> list[dict]:
    res = []
    for mid, m in list_local_models().items():
        rdf = m["rdf"]
        text = " ".join([mid, str(rdf.get("name", "")), str(rdf.get("description", ""))] +
                        [str(t) for t in rdf.get("tags", [])]).lower()
        if keywords and not all(k.lower() in text for k in keywords):
            continue
        res.append({"model_id": mid, "description": rdf.get("description", "")})
        if len(res) >= limit:
            break
    return res


class PackageLease:
    """Async context manager marking a cached package as in use (not evictable)."""

    def __init__(self, cache: "ModelCache", model_id: str, path: Path, latest_remote_modified: float | None):
        self.cache, self.model_id, self.source, self.latest_remote_modified = cache, model_id, path, latest_remote_modified
        self._lease: Path | None = None

    @property
    def rdf_path(self) -> Path:
        return self.source / "rdf.yaml"

    async def __aenter__(self):
        self._lease = self.source / f".in_use.{os.getpid()}.{uuid.uuid4().hex[:12]}"
        self._lease.write_text(json.dumps(_owner()))
        (self.source / ".last_access").write_text(str(time.time()))
        return self

    async def __aexit__(self, *exc):
        if self._lease is not None:
            self._lease.unlink(missing_ok=True)
        (self.source / ".last_access").write_text(str(time.time()))


class ModelCache:
    def __init__(self, cache_dir: str | Path | None = None, cache_size_in_gb: float = 50.0, replica_id: str = "r0",
                 fetch_remote=None):
        self.cache_dir = Path(cache_dir or Path(os.environ.get("HOME", ".")) / "models")
        self.cache_dir.mkdir(parents=True, exist_ok=True)
        self.cache_size_bytes = int(cache_size_in_gb * 1024 ** 3)
        self.replica_id = replica_id
        self.fetch_remote = fetch_remote  # async (model_id, dest_dir, stage) -> latest_modified | None

    def _dir(self, model_id: str) -> Path:
        return self.cache_dir / model_id.replace("/", "__")

    @staticmethod
    def _size(d: Path) -> int:
        return sum(p.stat().st_size for p in d.rglob("*") if p.is_file())

    def cached_models(self) -> list[dict]:
        out = []
        for d in self.cache_dir.iterdir():
            if d.is_dir() and (d / "rdf.yaml").exists():
                la = d / ".last_access"
                out.append({"model_id": d.name, "path": str(d), "size_bytes": self._size(d),
                            "last_access": float(la.read_text()) if la.exists() else 0.0,
                            "in_use": any(lease_live(p) for p in d.glob(".in_use.*"))})
        return out

    async def ensure_space(self, needed: int) -> None:
        for _ in range(5):
            models = sorted(self.cached_models(), key=lambda m: m["last_access"])
            used = sum(m["size_bytes"] for m in models)
            if used + needed <= self.cache_size_bytes:
                return
            for m in models:
                if used + needed <= self.cache_size_bytes:
                    return
                if m["in_use"]:
                    continue
                shutil.rmtree(m["path"], ignore_errors=True)
                used -= m["size_bytes"]
            await asyncio.sleep(0.2)
        if sum(m["size_bytes"] for m in self.cached_models()) + needed > self.cache_size_bytes:
            raise RuntimeError("model cache full (all cached packages in use)")

    @staticmethod
    def _reclaim_stale_marker(marker: Path) -> bool:
        """Remove a download marker left by a dead downloader (or older than the download timeout);
        True when it was removed and the caller may claim the download."""
        try:
            mt = marker.stat().st_mtime
        except OSError:
            return True  # gone meanwhile
        info = _read_owner(marker / "owner.json")
        if info is None and time.time() - mt < 5.0:
            return False  # just created; its owner record follows the mkdir
        if not _owner_stale(info, DOWNLOAD_TIMEOUT_S, mt):
            return False
        # Atomic reclaim: rename the stale marker to a tombstone unique to this waiter.  Of several
        # waiters that judged the same marker stale, only one rename succeeds; the others see it gone
        # (and then race on the mkdir, which is atomic).  A rmtree of the marker path itself could
        # delete a FRESH marker another waiter had just reclaimed and re-created.
        tomb = marker.with_name(f"{marker.name}.stale.{os.getpid()}.{uuid.uuid4().hex[:8]}")
        try:
            os.rename(marker, tomb)
        except OSError:
            return True  # someone else reclaimed (or the owner finished): retry the mkdir
        # the renamed directory must still be the one judged stale: a marker re-created between the
        # check and the rename carries a different owner record -- put it back untouched
        if _read_owner(tomb / "owner.json") != info:
            try:
                os.rename(tomb, marker)
                return False
            except OSError:
                pass  # a third marker exists now; the tombstone is ours to drop
        shutil.rmtree(tomb, ignore_errors=True)
        return True

    async def get_model_package(self, model_id: str, stage: bool = False, skip_cache: bool = False,
                                allow_unpublished: bool = True) -> PackageLease:
        if "://" in model_id:
            raise ValueError("model_id must be a model id, not a URL")
        d = self._dir(model_id)
        marker = self.cache_dir / f".{d.name}.downloading"
        if skip_cache and d.exists():
            shutil.rmtree(d, ignore_errors=True)
        for _ in range(600):
            if (d / "rdf.yaml").exists() and not marker.exists():
                meta = d / ".source.json"
                lm = json.loads(meta.read_text()).get("latest_remote_modified") if meta.exists() else None
                return PackageLease(self, model_id, d, lm)
            try:
                marker.mkdir()  # atomic: only one replica downloads
            except FileExistsError:
                if self._reclaim_stale_marker(marker):
                    continue
                await asyncio.sleep(0.1)
                continue
            (marker / "owner.json").write_text(json.dumps(_owner()))
            try:
                tmp = self.cache_dir / f".{d.name}.{self.replica_id}.tmp"
                shutil.rmtree(tmp, ignore_errors=True)
                local = list_local_models().get(model_id)
                latest = None
                if local is not None:
                    await self.ensure_space(self._size(local["dir"]))
                    shutil.copytree(local["dir"], tmp)
                    latest = max(p.stat().st_mtime for p in local["dir"].rglob("*") if p.is_file())
                elif self.fetch_remote is not None:
                    tmp.mkdir(parents=True)
                    latest = await self.fetch_remote(model_id, tmp, stage)
                else:
                    raise ValueError(f"model '{model_id}' not found (no local zoo entry, no remote source)")
                (tmp / ".source.json").write_text(json.dumps({"model_id": model_id, "latest_remote_modified": latest}))
                if d.exists():
                    shutil.rmtree(d, ignore_errors=True)
                os.rename(tmp, d)
            finally:
                shutil.rmtree(marker, ignore_errors=True)
        raise TimeoutError(f"timed out waiting for model '{model_id}' download")
