"""BioEngine datasets server (FastAPI): ``python -m bioengine_worker_amd.datasets --data-dir PATH``.

Same HTTP API as the reference (``bioengine/datasets/proxy_server.py:285-679``,
``docs/datasets-guide.md:171-304``):

``GET /health/liveness``, ``GET /ping``, ``GET /datasets``, ``GET /datasets/{id}/files?dir_path&token``,
``GET /data/{id}/{path}?token`` (HTTP Range -> 206), ``POST /save?filename&public&token``
(public: ``saved/public``, never overwritten; private: ``saved/<user>``), ``GET /saved?token``,
``GET /saved/{path}?token``.

Datasets are ``data_dir/<name>/manifest.yaml`` (``id``, ``authorized_users``); the catalog is
rescanned every 30 s.  Tokens are validated against the hub (``--authentication-server-url``:
``local://<name>``, ``ws://...`` or a Hypha URL) and cached (1 000 entries).  Path traversal is
rejected both syntactically (``..``) and after ``resolve()``.  On start the server writes its URL
to ``~/.bioengine/datasets/bioengine_current_server`` for client auto-discovery.
"""
from __future__ import annotations

import asyncio
import collections
import os
import re
from contextlib import asynccontextmanager
from pathlib import Path

import yaml
from fastapi import FastAPI, HTTPException, Request
from fastapi.responses import FileResponse, Response

from ..utils.permissions import check_permissions

DISCOVERY_FILE = Path.home() / ".bioengine" / "datasets" / "bioengine_current_server"
DEFAULT_PORT = 39527


def scan_datasets(data_dir: Path) -> dict[str, dict]:
    if not data_dir.is_dir():
        raise ValueError(f"data_dir does not exist or is not a directory: {data_dir}")
    out = {}
    for sub in sorted(data_dir.iterdir()):
        mf = sub / "manifest.yaml"
        if not sub.is_dir() or not mf.exists() or sub.name == "saved":
            continue
        try:
            m = yaml.safe_load(mf.read_text()) or {}
        except Exception:
            continue
        users = m.get("authorized_users", [])
        if isinstance(users, str):
            users = [users]
        out[m.get("id") or sub.name] = {"manifest": m, "path": sub, "authorized_users": users}
    return out


class TokenValidator:
    def __init__(self, auth_url: str | None, cache_size: int = 1000):
        self.auth_url = auth_url
        self.cache: collections.OrderedDict = collections.OrderedDict()
        self.cache_size = cache_size
        self._client = None

    async def parse(self, token: str | None) -> dict:
        if not token:
            return {"id": "anonymous", "email": "anonymous@example.com", "is_anonymous": True}
        if token in self.cache:
            self.cache.move_to_end(token)
            return self.cache[token]
        if self.auth_url is None:
            raise PermissionError("token validation is not configured")
        if self._client is None:
            from ..transport.client import connect_to_server

            self._client = await connect_to_server({"server_url": self.auth_url})
        try:
            info = await self._client.parse_token(token)
        except Exception as e:  # noqa: BLE001
            raise PermissionError(f"invalid token: {e}") from e
        u = {"id": info.get("id"), "email": info.get("email")}
        self.cache[token] = u
        while len(self.cache) > self.cache_size:
            self.cache.popitem(last=False)
        return u


def _safe_path(base: Path, rel: str) -> Path:
    if not rel:
        raise ValueError("path must not be empty")
    if any(part == ".." for part in Path(rel).parts):
        raise ValueError("path traversal is not allowed")
    full = (base / rel).resolve()
    full.relative_to(base.resolve())  # raises ValueError on escape
    return full


def build_app(data_dir: str | Path, auth_url: str | None = None, rescan_s: float = 30.0):
    data_dir = Path(data_dir).resolve()
    state = {"datasets": scan_datasets(data_dir)}
    tv = TokenValidator(auth_url)

    async def rescan():
        while True:
            await asyncio.sleep(rescan_s)
            try:
                state["datasets"] = scan_datasets(data_dir)
            except Exception:
                pass

    @asynccontextmanager
    async def lifespan(app):
        t = asyncio.create_task(rescan())
        yield
        t.cancel()

    app = FastAPI(title="BioEngine Datasets", lifespan=lifespan)

    async def user_for(token):
        try:
            return await tv.parse(token)
        except PermissionError as e:
            raise HTTPException(status_code=403, detail=str(e))

    def authorize(user, ds_id, what):
        ds = state["datasets"].get(ds_id)
        if ds is None:
            raise HTTPException(status_code=404, detail=f"Dataset '{ds_id}' not found")
        try:
            check_permissions({"user": user}, ds["authorized_users"], what)
        except PermissionError as e:
            raise HTTPException(status_code=403, detail=str(e))
        return ds

    @app.get("/health/liveness")
    async def liveness():
        return {"status": "ok"}

    @app.get("/ping")
    async def ping():
        return "pong"

    @app.get("/datasets")
    async def list_datasets():
        return {k: v["manifest"] for k, v in state["datasets"].items()}

    @app.get("/datasets/{dataset_id}/files")
    async def list_files(dataset_id: str, dir_path: str | None = None, token: str | None = None):
        if dataset_id not in state["datasets"]:
            raise HTTPException(status_code=400, detail=f"ValueError: Dataset '{dataset_id}' does not exist")
        ds = authorize(await user_for(token), dataset_id, f"list files in dataset '{dataset_id}'")
        base = ds["path"]
        try:
            scan = _safe_path(base, dir_path) if dir_path else base
        except ValueError as e:
            raise HTTPException(status_code=400, detail=str(e))
        if not scan.exists():
            raise HTTPException(status_code=400, detail=f"ValueError: Path '{dir_path}' does not exist in dataset '{dataset_id}'")
        files = []
        for root, dirs, names in os.walk(scan):
            dirs.sort()
            for n in sorted(names):
                files.append(str((Path(root) / n).relative_to(base)))
        return files

    @app.get("/data/{dataset_id}/{path:path}")
    async def serve_file(dataset_id: str, path: str, request: Request, token: str | None = None):
        ds = authorize(await user_for(token), dataset_id, f"access '{path}' in dataset '{dataset_id}'")
        try:
            full = _safe_path(ds["path"], path)
        except ValueError as e:
            raise HTTPException(status_code=400, detail=str(e))
        if not full.is_file():
            raise HTTPException(status_code=404, detail=f"'{path}' not found")
        rng = request.headers.get("range")
        if rng:
            m = re.match(r"bytes=(\d*)-(\d*)", rng)
            size = full.stat().st_size
            if m:
                a, b = m.group(1), m.group(2)
                if a == "" and b:
                    start, end = max(0, size - int(b)), size - 1
                else:
                    start = int(a or 0)
                    end = min(size - 1, int(b)) if b else size - 1
                if start >= size:
                    return Response(status_code=416, headers={"Content-Range": f"bytes */{size}"})

                def read():
                    with open(full, "rb") as f:
                        f.seek(start)
                        return f.read(end - start + 1)

                data = await asyncio.to_thread(read)
                return Response(content=data, status_code=206, media_type="application/octet-stream",
                                headers={"Content-Range": f"bytes {start}-{end}/{size}", "Accept-Ranges": "bytes"})
        return FileResponse(full)

    def _uid(user):
        uid = user.get("id") or "anonymous"
        return uid, re.sub(r"[^A-Za-z0-9_.-]", "_", uid)

    @app.post("/save")
    async def save(request: Request, filename: str, public: bool = False, token: str | None = None):
        if not filename or "/" in filename or "\\" in filename or filename in (".", ".."):
            raise HTTPException(status_code=400, detail="filename must not contain path separators")
        if not token:
            raise HTTPException(status_code=403, detail="a token is required to save files")
        user = await user_for(token)
        uid, safe = _uid(user)
        if public:
            ds_id, d, users, name = "saved-public", data_dir / "saved" / "public", ["*"], "Public Saved Files"
        else:
            ds_id, d, users, name = f"saved-{safe}", data_dir / "saved" / safe, [uid], f"Private files for {uid}"
        d.mkdir(parents=True, exist_ok=True)
        mf = d / "manifest.yaml"
        if not mf.exists():
            mf.write_text(yaml.safe_dump({"id": ds_id, "name": name, "authorized_users": users,
                                          "description": "Files saved via the BioEngine Datasets save API."}))
        fp = d / filename
        if public and fp.exists():
            raise HTTPException(status_code=409, detail=f"'{filename}' already exists in the public directory")
        body = await request.body()
        await asyncio.to_thread(fp.write_bytes, body)
        return {"dataset_id": ds_id, "filename": filename, "size": len(body), "public": public}

    def _saved_dirs(user):
        uid, safe = _uid(user)
        out = [("public", data_dir / "saved" / "public")]
        if not user.get("is_anonymous"):
            out.append(("private", data_dir / "saved" / safe))
        return out

    @app.get("/saved")
    async def list_saved(token: str | None = None):
        user = await user_for(token)
        res = {}
        for kind, d in _saved_dirs(user):
            if d.is_dir():
                res[kind] = sorted(p.name for p in d.iterdir() if p.is_file() and p.name != "manifest.yaml")
            else:
                res[kind] = []
        return res

    @app.get("/saved/{path:path}")
    async def get_saved(path: str, token: str | None = None, public: bool | None = None):
        user = await user_for(token)
        for kind, d in _saved_dirs(user):
            if public is True and kind != "public":
                continue
            if public is False and kind != "private":
                continue
            try:
                fp = _safe_path(d, path)
            except ValueError as e:
                raise HTTPException(status_code=400, detail=str(e))
            if fp.is_file():
                return FileResponse(fp)
        raise HTTPException(status_code=404, detail=f"'{path}' not found")

    app.state.datasets_state = state
    return app


def write_discovery_file(url: str, path: Path = DISCOVERY_FILE):
    path.parent.mkdir(parents=True, exist_ok=True)
    path.write_text(url)


def start_proxy_server(data_dir: str, server_ip: str | None = None, server_port: int | None = None,
                       authentication_server_url: str | None = None, log_file: str | None = None):
    import uvicorn

    from ..utils.network import acquire_free_port, get_internal_ip

    ip = server_ip or get_internal_ip()
    port = server_port or acquire_free_port(DEFAULT_PORT, ip=ip)
    app = build_app(data_dir, authentication_server_url)
    url = f"http://{ip}:{port}"
    write_discovery_file(url)
    print(f"BioEngine datasets server at {url}", flush=True)
    uvicorn.run(app, host=ip, port=port, log_level="info")
