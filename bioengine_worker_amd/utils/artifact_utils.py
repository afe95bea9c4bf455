"""App artifacts: file lists, manifest validation, staged upload + version semantics.

Mirrors the reference's app-artifact workflow (``bioengine/utils/artifact_utils.py``):

* ``create_file_list_from_directory`` (``:13-97``) — text files as ``text``, binaries as ``base64``;
* ``ensure_applications_collection`` (``:100-167``) — ``<ws>/applications`` with public read;
* ``validate_manifest`` (``:216-259``) / ``validate_artifact_id`` (``:263-317``);
* ``stage_artifact`` (``:320-478``) — a manifest version not yet present branches a new version
  snapshot; re-saving the latest version updates it in place; re-saving an *older* version raises;
* presigned uploads (``:481-548``), commit (``:580-609``), static-site URL (``:612-628``);
* ``create_application_from_files`` (``:632-790``) orchestrating the above, pruning files that
  are no longer part of the app.
"""
from __future__ import annotations

import base64
import logging
from pathlib import Path, PurePosixPath
from typing import Any

import httpx
import yaml

REQUIRED_FIELDS = ("name", "id", "id_emoji", "description", "type", "deployments")
_log = logging.getLogger("bioengine.artifacts")


def create_file_list_from_directory(directory_path: str | Path, _artifact_id_suffix: str | None = None) -> list[dict]:
    root = Path(directory_path)
    if not root.is_dir():
        raise ValueError(f"Not a directory: {root}")
    files = []
    for p in sorted(root.rglob("*")):
        if not p.is_file() or "__pycache__" in p.parts:
            continue
        rel = p.relative_to(root).as_posix()
        try:
            content, kind = p.read_text(encoding="utf-8"), "text"
        except UnicodeDecodeError:
            content, kind = base64.b64encode(p.read_bytes()).decode("ascii"), "base64"
        if rel == "manifest.yaml" and _artifact_id_suffix:
            m = yaml.safe_load(content)
            if not isinstance(m, dict) or "id" not in m:
                raise ValueError("manifest.yaml must be a mapping with an 'id'")
            m["id"] = f"{m['id']}-{_artifact_id_suffix}"
            content = yaml.safe_dump(m, sort_keys=False)
        files.append({"name": rel, "content": content, "type": kind})
    return files


def validate_manifest(manifest: dict) -> None:
    if not isinstance(manifest, dict):
        raise ValueError("Manifest must be a mapping")
    for f in REQUIRED_FIELDS:
        if f not in manifest:
            raise ValueError(f"Manifest is missing required field: '{f}'")
    if manifest["type"] != "ray-serve":
        raise ValueError(f"Invalid manifest type: '{manifest['type']}'. Expected 'ray-serve'.")
    deps = manifest["deployments"]
    if not isinstance(deps, list) or not deps:
        raise ValueError("Manifest 'deployments' must be a non-empty list of 'python_file:ClassName' entries")
    for d in deps:
        if not isinstance(d, str) or ":" not in d:
            raise ValueError(f"Invalid deployment entry '{d}': expected 'python_file:ClassName'")


def validate_artifact_id(manifest: dict, workspace: str, artifact_id: str | None = None) -> str:
    if artifact_id is None:
        alias = manifest.get("id")
        if not alias:
            raise ValueError("No artifact_id given and manifest has no 'id'")
        if (not alias.islower() and any(c.isalpha() for c in alias)) or "_" in alias or "/" in alias \
                or not alias.replace("-", "_").isidentifier():
            raise ValueError(f"Invalid artifact alias: '{alias}'. Use lowercase letters, numbers and hyphens.")
        return f"{workspace}/{alias}"
    full = artifact_id if "/" in artifact_id else f"{workspace}/{artifact_id}"
    if not full.startswith(f"{workspace}/"):
        raise ValueError(f"Artifact ID '{full}' does not belong to workspace '{workspace}'")
    return full


def load_manifest_from_files(files: list[dict]) -> dict:
    for f in files:
        if f.get("name") == "manifest.yaml":
            content = f["content"]
            if f.get("type") == "base64":
                content = base64.b64decode(content).decode()
            m = yaml.safe_load(content)
            validate_manifest(m)
            return m
    raise ValueError("Application files must include 'manifest.yaml'")


async def ensure_applications_collection(artifact_manager, workspace: str, logger=None) -> str:
    logger = logger or _log
    cid = f"{workspace}/applications"
    try:
        coll = await artifact_manager.read(cid)
        cfg = dict(coll.get("config") or {})
        perms = dict(cfg.get("permissions") or {})
        if perms.get("*") != "r":
            perms["*"] = "r"
            cfg["permissions"] = perms
            await artifact_manager.edit(artifact_id=cid, config=cfg)
    except Exception as e:  # noqa: BLE001
        if "does not exist" not in str(e):
            raise
        await artifact_manager.create(type="collection", alias="applications",
                                      manifest={"name": "Applications", "description": "BioEngine applications"},
                                      config={"permissions": {"*": "r"}})
        logger.info(f"Created collection '{cid}'")
    return cid


def _view_config(manifest: dict) -> dict | None:
    fe = manifest.get("frontend_entry")
    if not fe:
        return None
    p = PurePosixPath(fe)
    parent = str(p.parent)
    return {"branch": "main", "root_directory": "" if parent == "." else parent, "headers": {}, "index": p.name}


async def stage_artifact(artifact_manager, workspace: str, manifest: dict, logger=None, permissions: dict | None = None):
    """Put the app artifact in staging. Returns (artifact, version_is_new)."""
    logger = logger or _log
    aid = validate_artifact_id(manifest, workspace)
    coll = f"{workspace}/applications"
    vc = _view_config(manifest)
    mver = manifest.get("version")
    existing = None
    try:
        existing = await artifact_manager.read(aid)
        if existing.get("parent_id") != coll:
            await artifact_manager.delete(artifact_id=aid)
            existing = None
    except Exception as e:  # noqa: BLE001
        if "does not exist" not in str(e):
            raise
    if existing is not None:
        cfg = dict(existing.get("config") or {})
        if permissions:
            cfg["permissions"] = permissions
        if vc is not None:
            cfg["view_config"] = vc
        versions = [v["version"] for v in (existing.get("versions") or [])]
        version_is_new = bool(mver and mver not in versions)
        if not version_is_new and versions and mver and mver != versions[-1]:
            raise ValueError(f"Cannot re-save artifact '{aid}' at version '{mver}': a newer version "
                             f"'{versions[-1]}' already exists. Bump the version in manifest.yaml "
                             f"(existing versions: {versions}).")
        kw = {"artifact_id": aid, "manifest": manifest, "type": "application", "stage": True,
              "version": "new" if version_is_new else None}
        if cfg:
            kw["config"] = cfg
        art = await artifact_manager.edit(**kw)
        return art, version_is_new
    cfg = {}
    if permissions:
        cfg["permissions"] = permissions
    if vc is not None:
        cfg["view_config"] = vc
    kw = {"parent_id": coll, "type": "application", "alias": aid.split("/", 1)[1], "manifest": manifest, "stage": True}
    if cfg:
        kw["config"] = cfg
    art = await artifact_manager.create(**kw)
    logger.info(f"Created new artifact '{art.get('id')}'")
    return art, True


async def upload_file_to_artifact(artifact_manager, artifact_id: str, file_name: str, file_content, file_type: str = "text"):
    url = await artifact_manager.put_file(artifact_id, file_path=file_name)
    if isinstance(file_content, bytes):
        data = file_content
    elif file_type == "base64":
        data = base64.b64decode(file_content)
    else:
        data = str(file_content).encode("utf-8")
    async with httpx.AsyncClient(timeout=120) as c:
        r = await c.put(url, content=data)
        if r.status_code >= 400:
            raise RuntimeError(f"Upload of '{file_name}' failed: HTTP {r.status_code} {r.text[:200]}")


async def remove_file_from_artifact(artifact_manager, artifact_id: str, file_name: str):
    await artifact_manager.remove_file(artifact_id, file_path=file_name)


async def commit_artifact(artifact_manager, artifact_id: str, version: str | None = None, logger=None):
    kw = {"artifact_id": artifact_id}
    if version is not None:
        kw["version"] = version
    await artifact_manager.commit(**kw)
    (logger or _log).info(f"Committed artifact '{artifact_id}' (version={version or 'latest'})")


def get_static_site_url(artifact_id: str, server_url: str) -> str:
    ws, alias = artifact_id.split("/", 1)
    return f"{server_url.rstrip('/')}/{ws}/view/{alias}/"


async def create_application_from_files(artifact_manager, files: list[dict], workspace: str, logger=None,
                                        permissions: dict | None = None) -> str:
    """Stage, upload, prune and commit an application artifact. Returns the artifact id."""
    logger = logger or _log
    manifest = load_manifest_from_files(files)
    await ensure_applications_collection(artifact_manager, workspace, logger)
    art, version_is_new = await stage_artifact(artifact_manager, workspace, manifest, logger, permissions)
    aid = art.get("id") or validate_artifact_id(manifest, workspace)
    try:
        existing = {f.get("name") for f in await artifact_manager.list_files(aid, version="stage")}
    except Exception:
        existing = set()
    new = set()
    for f in files:
        await upload_file_to_artifact(artifact_manager, aid, f["name"], f["content"], f.get("type", "text"))
        new.add(f["name"].split("/")[0])
    for name in existing - new:
        try:
            await remove_file_from_artifact(artifact_manager, aid, name)
        except Exception as e:  # noqa: BLE001
            logger.warning(f"could not prune '{name}': {e}")
    await commit_artifact(artifact_manager, aid, manifest.get("version") if version_is_new else None, logger)
    return aid
