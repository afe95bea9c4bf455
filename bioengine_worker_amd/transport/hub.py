"""BioEngine hub: a self-contained, Hypha-compatible RPC / artifact / storage server.

The reference talks to an external Hypha server for everything outside Ray:
service registry with ``require_context``, token minting/parsing, the artifact manager (app code
and manifests, with staging + versioning semantics relied on by
``bioengine/utils/artifact_utils.py:320-478``), S3 presigned URLs (model-runner uploads,
``apps/model-runner/entry_deployment.py:1821-1867``) and static site hosting of app frontends
(``artifact_utils.py:612-628``).  All of the reference's tests hit the production server.

This module implements those server-side semantics in-process so the worker, apps, CLI and tests
run offline.  The same :class:`Hub` is reachable

* in-process (``connect_to_server({"server_url": "local://<name>"})``), and
* over WebSocket (``python -m bioengine_worker_amd.transport.hub_server``), so clients and workers
  in different processes/hosts talk exactly as they would through Hypha.

Presigned upload/download URLs and static sites are served by an aiohttp HTTP endpoint owned by
the hub.
"""
from __future__ import annotations

import asyncio
import base64
import copy
import fnmatch
import hashlib
import hmac
import inspect
import json
import mimetypes
import os
import secrets
import shutil
import tempfile
import time
import uuid
from pathlib import Path
from typing import Any, Callable


class ObjDict(dict):
    """dict with attribute access (Hypha returns ObjectProxy-like values)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


def _obj(x):
    if isinstance(x, dict) and not isinstance(x, ObjDict):
        return ObjDict({k: _obj(v) for k, v in x.items()})
    if isinstance(x, list):
        return [_obj(v) for v in x]
    return x


# ====================================================================== tokens


class TokenAuthority:
    """HMAC-signed bearer tokens carrying {user id, email, workspace, scope, expiry}."""

    def __init__(self, secret: bytes | None = None):
        self.secret = secret or secrets.token_bytes(32)

    def mint(self, payload: dict) -> str:
        body = base64.urlsafe_b64encode(json.dumps(payload, sort_keys=True).encode()).decode().rstrip("=")
        sig = hmac.new(self.secret, body.encode(), hashlib.sha256).hexdigest()[:32]
        return f"be1.{body}.{sig}"

    def parse(self, token: str) -> dict:
        try:
            _, body, sig = token.split(".")
        except ValueError as e:
            raise PermissionError("malformed token") from e
        want = hmac.new(self.secret, body.encode(), hashlib.sha256).hexdigest()[:32]
        if not hmac.compare_digest(want, sig):
            raise PermissionError("invalid token signature")
        payload = json.loads(base64.urlsafe_b64decode(body + "=" * (-len(body) % 4)))
        if payload.get("expires_at") and payload["expires_at"] < time.time():
            raise PermissionError("token expired")
        return payload


# ====================================================================== artifact manager


class ArtifactManager:
    """Artifact collections with staged edits and version snapshots (Hypha artifact-manager subset)."""

    def __init__(self, hub: "Hub", root: Path):
        self.hub = hub
        self.root = root
        self.root.mkdir(parents=True, exist_ok=True)
        self.arts: dict[str, dict] = {}

    # -- helpers
    def _resolve(self, artifact_id: str, ws: str) -> str:
        return artifact_id if "/" in artifact_id else f"{ws}/{artifact_id}"

    def _get(self, aid: str) -> dict:
        if aid not in self.arts:
            raise KeyError(f"Artifact with ID '{aid}' does not exist.")
        return self.arts[aid]

    def _dir(self, aid: str, slot: str) -> Path:
        return self.root / aid.replace("/", "__") / slot

    def _version_index(self, a: dict, version) -> int:
        if not a["versions"]:
            raise KeyError(f"Artifact '{a['id']}' has no committed versions.")
        if version in (None, "latest"):
            return len(a["versions"]) - 1
        for i, v in enumerate(a["versions"]):
            if v["version"] == version:
                return i
        if isinstance(version, int) or (isinstance(version, str) and version.isdigit()):
            return int(version)
        raise KeyError(f"Version '{version}' of artifact '{a['id']}' does not exist.")

    def _files_dir(self, a: dict, version) -> Path:
        if version == "stage":
            if a["staging"] is None:
                raise ValueError(f"Artifact '{a['id']}' is not in staging mode.")
            return self._dir(a["id"], "stage")
        if not a["versions"] and a["staging"] is not None and version in (None, "latest"):
            return self._dir(a["id"], "stage")
        return self._dir(a["id"], f"v{self._version_index(a, version)}")

    def _check(self, ctx, a: dict, mode: str):
        perms = (a.get("config") or {}).get("permissions") or {}
        ws = a["id"].split("/")[0]
        user = (ctx or {}).get("user", {})
        if ctx is None or ctx.get("ws") == ws or user.get("id") == a.get("created_by"):
            return
        for who, p in perms.items():
            if who in ("*", user.get("id"), user.get("email")) and (mode == "r" and p in ("r", "r+", "rw", "*")):
                return
        if mode == "r" and a.get("parent_id"):
            parent = self.arts.get(a["parent_id"])
            if parent is not None:
                return self._check(ctx, parent, mode)
        raise PermissionError(f"Permission denied on artifact '{a['id']}'")

    def _view(self, a: dict, version=None) -> ObjDict:
        d = {k: copy.deepcopy(v) for k, v in a.items() if k not in ("staging",)}
        if version == "stage" or (not a["versions"] and a["staging"] is not None):
            st = a["staging"] or {}
            d["manifest"] = copy.deepcopy(st.get("manifest", a["manifest"]))
            d["staging"] = True
        elif a["versions"]:
            i = self._version_index(a, version)
            d["manifest"] = copy.deepcopy(a["versions"][i]["manifest"])
            d["version"] = a["versions"][i]["version"]
        d["versions"] = [{k: v for k, v in ver.items() if k != "manifest"} for ver in a["versions"]]
        return _obj(d)

    # -- API (methods take `context` like any require_context service)
    async def create(self, type: str = "generic", alias: str | None = None, manifest: dict | None = None,
                     parent_id: str | None = None, config: dict | None = None, stage: bool = False,
                     version: str | None = None, overwrite: bool = False, context=None, **_):
        ws = (context or {}).get("ws", "public")
        alias = alias or uuid.uuid4().hex[:12]
        aid = alias if "/" in alias else f"{ws}/{alias}"
        if parent_id is not None:
            parent_id = self._resolve(parent_id, ws)
            self._get(parent_id)
        if aid in self.arts and not overwrite:
            raise FileExistsError(f"Artifact with ID '{aid}' already exists.")
        now = time.time()
        a = {
            "id": aid, "alias": aid.split("/", 1)[1], "type": type, "parent_id": parent_id,
            "manifest": copy.deepcopy(manifest or {}), "config": copy.deepcopy(config or {}),
            "versions": [], "staging": None,
            "created_by": (context or {}).get("user", {}).get("id"), "created_at": now, "last_modified": now,
        }
        self.arts[aid] = a
        shutil.rmtree(self.root / aid.replace("/", "__"), ignore_errors=True)
        if stage or version == "stage":
            a["staging"] = {"manifest": copy.deepcopy(manifest or {}), "new_version": True}
            self._dir(aid, "stage").mkdir(parents=True, exist_ok=True)
        else:
            self._dir(aid, "v0").mkdir(parents=True, exist_ok=True)
            a["versions"].append({"version": version or "v0", "manifest": copy.deepcopy(a["manifest"]),
                                  "created_at": now, "comment": None})
        return self._view(a)

    async def edit(self, artifact_id: str, manifest: dict | None = None, type: str | None = None,
                   config: dict | None = None, stage: bool = False, version: str | None = None, context=None, **_):
        aid = self._resolve(artifact_id, (context or {}).get("ws", "public"))
        a = self._get(aid)
        self._check(context, a, "w")
        if config is not None:
            a["config"] = copy.deepcopy(config)
        if type is not None:
            a["type"] = type
        if stage or version == "stage":
            sd = self._dir(aid, "stage")
            if a["staging"] is None:
                shutil.rmtree(sd, ignore_errors=True)
                if a["versions"]:
                    shutil.copytree(self._files_dir(a, None), sd)
                else:
                    sd.mkdir(parents=True, exist_ok=True)
                a["staging"] = {"manifest": copy.deepcopy(manifest if manifest is not None else a["manifest"]),
                                "new_version": version == "new" or not a["versions"]}
            else:
                if manifest is not None:
                    a["staging"]["manifest"] = copy.deepcopy(manifest)
                if version == "new":
                    a["staging"]["new_version"] = True
        else:
            if manifest is not None:
                a["manifest"] = copy.deepcopy(manifest)
                if a["versions"]:
                    a["versions"][-1]["manifest"] = copy.deepcopy(manifest)
        a["last_modified"] = time.time()
        return self._view(a, "stage" if a["staging"] else None)

    async def commit(self, artifact_id: str, version: str | None = None, comment: str | None = None, context=None, **_):
        aid = self._resolve(artifact_id, (context or {}).get("ws", "public"))
        a = self._get(aid)
        self._check(context, a, "w")
        st = a["staging"]
        if st is None:
            raise ValueError(f"Artifact '{aid}' has no staged changes to commit.")
        sd = self._dir(aid, "stage")
        now = time.time()
        if st["new_version"] or not a["versions"]:
            idx = len(a["versions"])
            tag = version or f"v{idx}"
            if any(v["version"] == tag for v in a["versions"]):
                raise ValueError(f"Version '{tag}' already exists for artifact '{aid}'.")
            dst = self._dir(aid, f"v{idx}")
            shutil.rmtree(dst, ignore_errors=True)
            sd.rename(dst)
            a["versions"].append({"version": tag, "manifest": copy.deepcopy(st["manifest"]), "created_at": now,
                                  "comment": comment})
        else:
            idx = len(a["versions"]) - 1
            dst = self._dir(aid, f"v{idx}")
            shutil.rmtree(dst, ignore_errors=True)
            sd.rename(dst)
            a["versions"][idx]["manifest"] = copy.deepcopy(st["manifest"])
            a["versions"][idx]["created_at"] = now
            if version:
                a["versions"][idx]["version"] = version
        a["manifest"] = copy.deepcopy(st["manifest"])
        a["staging"] = None
        a["last_modified"] = now
        return self._view(a)

    async def discard(self, artifact_id: str, context=None, **_):
        aid = self._resolve(artifact_id, (context or {}).get("ws", "public"))
        a = self._get(aid)
        a["staging"] = None
        shutil.rmtree(self._dir(aid, "stage"), ignore_errors=True)
        return self._view(a)

    async def read(self, artifact_id: str, version: str | None = None, silent: bool = False, context=None, **_):
        aid = self._resolve(artifact_id, (context or {}).get("ws", "public"))
        a = self._get(aid)
        self._check(context, a, "r")
        return self._view(a, version)

    async def list(self, parent_id: str | None = None, keywords=None, filters=None, limit: int = 1000,
                   context=None, **_):
        ws = (context or {}).get("ws", "public")
        pid = self._resolve(parent_id, ws) if parent_id else None
        if pid:
            self._check(context, self._get(pid), "r")
        out = [self._view(a) for a in self.arts.values() if a["parent_id"] == pid]
        return out[:limit]

    async def delete(self, artifact_id: str, delete_files: bool = True, recursive: bool = False, context=None, **_):
        aid = self._resolve(artifact_id, (context or {}).get("ws", "public"))
        a = self._get(aid)
        self._check(context, a, "w")
        kids = [k for k, v in self.arts.items() if v["parent_id"] == aid]
        if kids and not recursive:
            for k in kids:
                self.arts[k]["parent_id"] = None
        for k in kids if recursive else []:
            await self.delete(k, delete_files, True, context)
        del self.arts[aid]
        if delete_files:
            shutil.rmtree(self.root / aid.replace("/", "__"), ignore_errors=True)

    async def put_file(self, artifact_id: str, file_path: str, download_weight: float = 0, context=None, **_):
        aid = self._resolve(artifact_id, (context or {}).get("ws", "public"))
        a = self._get(aid)
        self._check(context, a, "w")
        if a["staging"] is None:
            raise ValueError(f"Artifact '{aid}' must be in staging mode to upload files.")
        dst = self._dir(aid, "stage") / file_path
        return self.hub.presign(dst, "PUT")

    async def remove_file(self, artifact_id: str, file_path: str, context=None, **_):
        aid = self._resolve(artifact_id, (context or {}).get("ws", "public"))
        a = self._get(aid)
        if a["staging"] is None:
            raise ValueError(f"Artifact '{aid}' must be in staging mode to remove files.")
        p = self._dir(aid, "stage") / file_path
        if p.is_dir():
            shutil.rmtree(p)
        elif p.exists():
            p.unlink()

    async def get_file(self, artifact_id: str, file_path: str, version: str | None = None, use_proxy=None,
                       context=None, **_):
        aid = self._resolve(artifact_id, (context or {}).get("ws", "public"))
        a = self._get(aid)
        self._check(context, a, "r")
        p = self._files_dir(a, version) / file_path
        if not p.is_file():
            raise FileNotFoundError(f"File '{file_path}' not found in artifact '{aid}'.")
        return self.hub.presign(p, "GET")

    async def list_files(self, artifact_id: str, dir_path: str | None = None, version: str | None = None,
                         limit: int = 10000, context=None, **_):
        aid = self._resolve(artifact_id, (context or {}).get("ws", "public"))
        a = self._get(aid)
        self._check(context, a, "r")
        base = self._files_dir(a, version)
        d = base / dir_path if dir_path else base
        if not d.exists():
            return []
        out = []
        for p in sorted(d.iterdir()):
            out.append(ObjDict(name=p.name, type="directory" if p.is_dir() else "file",
                               size=p.stat().st_size if p.is_file() else 0, last_modified=p.stat().st_mtime))
        return out[:limit]

    def local_path(self, aid: str, file_path: str, version=None) -> Path:
        return self._files_dir(self._get(aid), version) / file_path

    def service(self) -> dict:
        return {
            "id": "artifact-manager", "name": "Artifact Manager", "type": "artifact-manager",
            "config": {"visibility": "public", "require_context": True},
            **{m: getattr(self, m) for m in ("create", "edit", "commit", "discard", "read", "list", "delete",
                                             "put_file", "remove_file", "get_file", "list_files")},
        }


class S3Storage:
    """Per-workspace object store with presigned URLs (Hypha ``s3-storage`` subset)."""

    def __init__(self, hub: "Hub", root: Path):
        self.hub = hub
        self.root = root
        root.mkdir(parents=True, exist_ok=True)

    def _p(self, ctx, file_path: str) -> Path:
        ws = (ctx or {}).get("ws", "public")
        p = (self.root / ws / file_path).resolve()
        if not str(p).startswith(str((self.root / ws).resolve())):
            raise PermissionError("path traversal")
        return p

    async def generate_presigned_url(self, file_path: str, client_method: str = "get_object", expiration: int = 3600,
                                     context=None, **_):
        method = "PUT" if client_method in ("put_object", "PUT") else "GET"
        return self.hub.presign(self._p(context, file_path), method, expiration)

    async def put_file(self, file_path: str, context=None, **_):
        return self.hub.presign(self._p(context, file_path), "PUT")

    async def get_file(self, file_path: str, context=None, **_):
        p = self._p(context, file_path)
        if not p.exists():
            raise FileNotFoundError(file_path)
        return self.hub.presign(p, "GET")

    async def list_files(self, path: str = "", context=None, **_):
        d = self._p(context, path)
        if not d.exists():
            return []
        return [ObjDict(name=p.name, type="directory" if p.is_dir() else "file", size=p.stat().st_size)
                for p in sorted(d.iterdir())]

    async def remove_file(self, file_path: str, context=None, **_):
        p = self._p(context, file_path)
        if p.exists():
            p.unlink()

    def service(self) -> dict:
        return {"id": "s3-storage", "name": "S3 Storage", "type": "s3-storage",
                "config": {"visibility": "public", "require_context": True},
                **{m: getattr(self, m) for m in ("generate_presigned_url", "put_file", "get_file", "list_files",
                                                 "remove_file")}}


# ====================================================================== service registry


class ServiceEntry:
    def __init__(self, full_id: str, owner: "Session", svc: dict):
        self.full_id = full_id
        self.owner = owner
        self.svc = svc
        self.config = dict(svc.get("config") or {})
        self.info = ObjDict(id=full_id, name=svc.get("name", svc.get("id")), type=svc.get("type", "generic"),
                            description=svc.get("description", ""), config=self.config,
                            app_id=svc.get("app_id"), service_schema=svc.get("service_schema"))

    def methods(self) -> dict[str, Any]:
        return {k: v for k, v in self.svc.items() if callable(v) or isinstance(v, dict) and k not in ("config",)}


class Session:
    """A connected client (in-process or a WebSocket connection)."""

    def __init__(self, hub: "Hub", workspace: str, client_id: str, user: dict, remote_caller=None):
        self.hub = hub
        self.workspace = workspace
        self.client_id = client_id
        self.user = user
        self.remote_caller = remote_caller  # for WS sessions: async fn(service_local_id, path, args, kwargs)
        self.services: dict[str, ServiceEntry] = {}
        self.closed = False

    @property
    def full_client(self) -> str:
        return f"{self.workspace}/{self.client_id}"


class Hub:
    def __init__(self, data_dir: str | Path | None = None, name: str = "local", public_base_url: str | None = None):
        self.name = name
        self.data_dir = Path(data_dir or tempfile.mkdtemp(prefix=f"behub-{name}-"))
        self.tokens = TokenAuthority()
        self.sessions: dict[str, Session] = {}
        self.services: dict[str, ServiceEntry] = {}
        self.artifacts = ArtifactManager(self, self.data_dir / "artifacts")
        self.s3 = S3Storage(self, self.data_dir / "s3")
        self._presigned: dict[str, tuple[Path, str, float]] = {}
        self._http_runner = None
        self.http_base: str | None = None
        self.public_base_url = public_base_url
        self._system = Session(self, "public", "hub", {"id": "hub", "email": "hub@local", "roles": ["admin"]})
        self._register(self._system, self.artifacts.service())
        self._register(self._system, self.s3.service())
        self._lock = asyncio.Lock()
        self.ws_server_url: str | None = None

    # ------------------------------------------------------------------ http
    async def start_http(self, host: str = "127.0.0.1", port: int = 0) -> str:
        if self.http_base:
            return self.http_base
        from aiohttp import web

        app = web.Application(client_max_size=1024 ** 4)
        app.router.add_route("PUT", "/presigned/{key}", self._http_put)
        app.router.add_route("POST", "/presigned/{key}", self._http_put)
        app.router.add_route("GET", "/presigned/{key}", self._http_get)
        app.router.add_route("GET", "/{ws}/view/{alias}/{path:.*}", self._http_view)
        async def health(_r):
            return web.json_response({"ok": True, "name": self.name})

        app.router.add_route("GET", "/health", health)
        self._extra_routes(app)
        runner = web.AppRunner(app)
        await runner.setup()
        site = web.TCPSite(runner, host, port)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        self._http_runner = runner
        self.http_base = f"http://{host}:{port}"
        if self.public_base_url is None:
            self.public_base_url = self.http_base
        return self.http_base

    def _extra_routes(self, app):  # hub_server adds the websocket route
        pass

    async def stop_http(self):
        if self._http_runner is not None:
            await self._http_runner.cleanup()
            self._http_runner = None
            self.http_base = None

    def presign(self, path: Path, method: str, expiration: int = 3600) -> str:
        if self.http_base is None:
            raise RuntimeError("hub HTTP endpoint not started (await hub.start_http())")
        key = secrets.token_urlsafe(24)
        self._presigned[key] = (Path(path), method, time.time() + expiration)
        return f"{self.http_base}/presigned/{key}"

    def _lookup(self, key: str, method: str) -> Path:
        ent = self._presigned.get(key)
        if ent is None or ent[2] < time.time() or ent[1] != method:
            raise KeyError(key)
        return ent[0]

    async def _http_put(self, request):
        from aiohttp import web

        try:
            p = self._lookup(request.match_info["key"], "PUT")
        except KeyError:
            return web.Response(status=403, text="invalid or expired upload URL")
        p.parent.mkdir(parents=True, exist_ok=True)
        tmp = p.with_name(p.name + f".{uuid.uuid4().hex}.part")
        with open(tmp, "wb") as f:
            async for chunk in request.content.iter_chunked(1 << 20):
                f.write(chunk)
        os.replace(tmp, p)
        return web.Response(status=200)

    async def _http_get(self, request):
        from aiohttp import web

        try:
            p = self._lookup(request.match_info["key"], "GET")
        except KeyError:
            return web.Response(status=403, text="invalid or expired download URL")
        if not p.exists():
            return web.Response(status=404)
        return web.FileResponse(p)

    async def _http_view(self, request):
        from aiohttp import web

        aid = f"{request.match_info['ws']}/{request.match_info['alias']}"
        try:
            a = self.artifacts._get(aid)
        except KeyError:
            return web.Response(status=404, text="not found")
        vc = (a.get("config") or {}).get("view_config") or {}
        root = vc.get("root_directory", "")
        rel = request.match_info["path"] or vc.get("index", "index.html")
        try:
            p = self.artifacts.local_path(aid, str(Path(root) / rel) if root else rel)
        except KeyError:
            return web.Response(status=404)
        if not p.is_file():
            return web.Response(status=404)
        ctype = mimetypes.guess_type(str(p))[0] or "application/octet-stream"
        return web.Response(body=p.read_bytes(), content_type=ctype)

    # ------------------------------------------------------------------ sessions / tokens
    def issue_token(self, user_id: str, email: str | None = None, workspace: str | None = None,
                    permission: str = "admin", expires_in: float = 3600 * 24, roles=None) -> str:
        return self.tokens.mint({"id": user_id, "email": email or f"{user_id}@local", "workspace": workspace or f"ws-user-{user_id}",
                                 "permission": permission, "expires_at": time.time() + expires_in, "roles": roles or []})

    def open_session(self, token: str | None, workspace: str | None = None, client_id: str | None = None,
                     remote_caller=None) -> Session:
        if token:
            info = self.tokens.parse(token)
            user = {"id": info["id"], "email": info.get("email"), "roles": info.get("roles", []),
                    "scope": {"workspaces": {info["workspace"]: info.get("permission", "read")}}}
            ws = workspace or info["workspace"]
            if workspace and workspace != info["workspace"] and "admin" not in info.get("roles", []):
                raise PermissionError(f"token is not valid for workspace {workspace}")
        else:
            anon = f"anonymouz-{uuid.uuid4().hex[:8]}"
            user = {"id": anon, "email": None, "is_anonymous": True, "roles": []}
            ws = f"ws-{anon}"
            # an anonymous client only ever gets its own fresh workspace (as on Hypha): joining a
            # named workspace would let it call that workspace's protected services
            if workspace and workspace != ws:
                raise PermissionError(f"anonymous clients cannot join workspace {workspace}")
        cid = client_id or uuid.uuid4().hex[:10]
        key = f"{ws}/{cid}"
        old = self.sessions.get(key)
        if old is not None and not old.closed:
            # reconnect of the same client replaces its stale session; anyone else is refused
            # (otherwise any client could evict e.g. the worker and take over its service ids)
            if old.user.get("id") != user["id"]:
                raise PermissionError(f"client id {cid} is already in use in workspace {ws}")
            self.close_session(old)
        s = Session(self, ws, cid, user, remote_caller)
        self.sessions[key] = s
        return s

    def close_session(self, s: Session):
        s.closed = True
        for fid in list(s.services):
            if self.services.get(fid) is not None and self.services[fid].owner is s:
                self.services.pop(fid, None)
        s.services.clear()
        # only drop the table entry if it is still THIS session (a reconnect may have replaced it)
        if self.sessions.get(s.full_client) is s:
            self.sessions.pop(s.full_client, None)

    # ------------------------------------------------------------------ services
    def _register(self, s: Session, svc: dict, overwrite: bool = True) -> ObjDict:
        sid = svc.get("id") or "default"
        full = f"{s.workspace}/{s.client_id}:{sid}"
        if full in self.services and not overwrite:
            raise FileExistsError(full)
        e = ServiceEntry(full, s, svc)
        self.services[full] = e
        s.services[full] = e
        return e.info

    async def register_service(self, s: Session, svc: dict, overwrite: bool = True) -> ObjDict:
        return self._register(s, svc, overwrite)

    async def unregister_service(self, s: Session, service_id: str):
        full = self._find(s, service_id).full_id
        e = self.services.pop(full, None)
        if e is not None:
            e.owner.services.pop(full, None)

    def _find(self, s: Session | None, sid: str) -> ServiceEntry:
        ws = s.workspace if s else "public"
        cands = []
        if sid in self.services:
            return self.services[sid]
        name = sid
        if "/" in sid:
            ws, name = sid.split("/", 1)
        if ":" in name:
            cid, svc = name.split(":", 1)
            full = f"{ws}/{cid}:{svc}"
            if full in self.services:
                return self.services[full]
            raise KeyError(f"Service not found: {sid}")
        svc = name.split("@")[0]
        for fid, e in self.services.items():
            fws, rest = fid.split("/", 1)
            if rest.split(":", 1)[1] == svc and (fws == ws or fws == "public"):
                cands.append(e)
        if not cands:
            raise KeyError(f"Service not found: {sid}")
        own = [e for e in cands if e.full_id.startswith(ws + "/")]
        return (own or cands)[-1]

    def list_service_infos(self, s: Session | None, query=None) -> list[ObjDict]:
        ws = s.workspace if s else "public"
        q = query or {}
        if isinstance(q, str):
            q = {"workspace": q} if "/" not in q else {"workspace": q.split("/")[0]}
        qws = q.get("workspace", ws)
        out = []
        for fid, e in self.services.items():
            fws = fid.split("/", 1)[0]
            if qws not in ("*", fws) and not (qws == "public" and e.config.get("visibility") == "public"):
                continue
            if q.get("type") and e.info.type != q["type"]:
                continue
            if q.get("id") and not fnmatch.fnmatch(fid.split(":", 1)[1], q["id"]):
                continue
            out.append(e.info)
        return out

    def context_for(self, caller: Session | None, entry: ServiceEntry) -> dict:
        if caller is None:
            caller = self._system
        return {"user": dict(caller.user), "ws": caller.workspace, "from": caller.full_client, "to": entry.full_id}

    async def call(self, caller: Session | None, service_id: str, method: str, args: list, kwargs: dict):
        entry = self._find(caller, service_id)
        vis = entry.config.get("visibility", "protected")
        if caller is not None and vis != "public" and caller.workspace != entry.full_id.split("/")[0]:
            if "admin" not in caller.user.get("roles", []):
                raise PermissionError(f"Permission denied for protected service {entry.full_id}")
        kwargs = dict(kwargs or {})
        if entry.config.get("require_context"):
            kwargs["context"] = self.context_for(caller, entry)
        owner = entry.owner
        if owner.remote_caller is not None:
            local_id = entry.full_id.split(":", 1)[1]
            return await owner.remote_caller(local_id, method, list(args), kwargs)
        fn = _resolve_method(entry.svc, method)
        args = [_awaitable_callbacks(a) for a in args]
        kwargs = {k: (v if k == "context" else _awaitable_callbacks(v)) for k, v in kwargs.items()}
        res = fn(*args, **kwargs)
        if inspect.isawaitable(res):
            res = await res
        return res


def _awaitable_callbacks(x):
    """In-process calls see callables exactly like remote ones: always awaitable."""
    if callable(x) and not isinstance(x, type):
        fn = x

        async def acall(*a, **k):
            r = fn(*a, **k)
            if inspect.isawaitable(r):
                r = await r
            return r

        return acall
    if isinstance(x, list):
        return [_awaitable_callbacks(v) for v in x]
    if isinstance(x, dict) and not isinstance(x, ObjDict):
        return {k: _awaitable_callbacks(v) for k, v in x.items()}
    return x


def _resolve_method(svc: dict, path: str) -> Callable:
    obj: Any = svc
    for part in path.split("."):
        if isinstance(obj, dict):
            if part not in obj:
                raise AttributeError(f"Method '{path}' not found in service {svc.get('id')}")
            obj = obj[part]
        else:
            obj = getattr(obj, part)
    if not callable(obj):
        raise AttributeError(f"'{path}' is not callable")
    return obj


_HUBS: dict[str, Hub] = {}


def get_local_hub(name: str = "default", data_dir: str | None = None) -> Hub:
    if name not in _HUBS:
        _HUBS[name] = Hub(data_dir=data_dir, name=name)
    return _HUBS[name]


def reset_local_hubs():
    _HUBS.clear()
