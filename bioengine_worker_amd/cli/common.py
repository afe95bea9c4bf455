"""Shared helpers of the ``bioengine`` CLI (reference bioengine/cli/utils.py behaviour: env-var
resolution, service connection with multi-replica fallback, JSON/table output, image I/O)."""
from __future__ import annotations

import asyncio
import io
import json
import os
import sys
from functools import wraps
from pathlib import Path
from typing import Any

import click
import numpy as np

DEFAULT_SERVER = "https://hypha.aicell.io"


def server_url(v: str | None) -> str:
    return v or os.environ.get("BIOENGINE_SERVER_URL") or DEFAULT_SERVER


def token(v: str | None) -> str | None:
    return v or os.environ.get("HYPHA_TOKEN") or os.environ.get("BIOENGINE_TOKEN")


def worker_id(v: str | None) -> str | None:
    return v or os.environ.get("BIOENGINE_WORKER_SERVICE_ID")


def fail(msg: str, hint: str = "") -> None:
    click.secho(f"Error: {msg}", fg="red", err=True)
    if hint:
        click.echo(f"Hint: {hint}", err=True)
    sys.exit(1)


_OPEN: list = []


def run(coro):
    """Run a command coroutine and close every hub connection it opened in the same loop."""
    async def wrapped():
        try:
            return await coro
        finally:
            while _OPEN:
                srv = _OPEN.pop()
                try:
                    await srv.disconnect()
                except Exception:  # noqa: BLE001
                    pass
    return asyncio.run(wrapped())


def as_async(f):
    @wraps(f)
    def wrapper(*a, **k):
        return run(f(*a, **k))
    return wrapper


def parse_value(s: str) -> Any:
    """Auto-type a KEY=VALUE value: bool, int, float, JSON list/dict, else string."""
    low = s.lower()
    if low in ("true", "false"):
        return low == "true"
    if low in ("none", "null"):
        return None
    for cast in (int, float):
        try:
            return cast(s)
        except ValueError:
            pass
    if s[:1] in "[{":
        try:
            return json.loads(s)
        except json.JSONDecodeError:
            pass
    return s


async def connect(url: str, tok: str | None):
    from ..transport import connect_to_server

    cfg = {"server_url": url}
    if tok:
        cfg["token"] = tok
    srv = await connect_to_server(cfg)
    _OPEN.append(srv)
    return srv


async def get_service(url: str, service_id: str, tok: str | None):
    """Connect and resolve a service; when the id matches several replicas, take the first one
    (reference cli/utils.py:45-78 multi-replica fallback)."""
    srv = await connect(url, tok)
    try:
        return srv, await srv.get_service(service_id)
    except Exception as first:  # noqa: BLE001
        try:
            found = await srv.list_services({"id": f"*:{service_id.split(':')[-1]}"} if ":" in service_id else
                                            {"id": f"*{service_id.split('/')[-1]}*"})
        except Exception:  # noqa: BLE001
            found = []
        for s in found or []:
            sid = s["id"] if isinstance(s, dict) else str(s)
            try:
                return srv, await srv.get_service(sid)
            except Exception:  # noqa: BLE001
                continue
        raise first


def method_names(svc) -> list[str]:
    m = svc.__dict__.get("_methods") if hasattr(svc, "__dict__") else None
    if m:
        return sorted(m)
    return sorted(n for n in dir(svc) if not n.startswith("_") and callable(getattr(svc, n, None)))


def print_json(data: Any) -> None:
    click.echo(json.dumps(data, indent=2, default=_default))


def _default(o):
    if isinstance(o, np.ndarray):
        return {"__ndarray__": True, "shape": list(o.shape), "dtype": str(o.dtype)} if o.size > 64 else o.tolist()
    if isinstance(o, (np.integer, np.floating)):
        return o.item()
    return str(o)


def print_table(rows: list[list], headers: list[str]) -> None:
    cols = [[str(h)] + [str(r[i]) for r in rows] for i, h in enumerate(headers)]
    widths = [max(len(c) for c in col) for col in cols]
    click.echo("  ".join(h.ljust(w) for h, w in zip(headers, widths)))
    click.echo("  ".join("-" * w for w in widths))
    for r in rows:
        click.echo("  ".join(str(v).ljust(w) for v, w in zip(r, widths)))


def read_image(path: str) -> np.ndarray:
    p = Path(path)
    suf = p.suffix.lower()
    if suf == ".npy":
        return np.load(p)
    if suf == ".npz":
        z = np.load(p)
        return z[z.files[0]]
    from PIL import Image

    return np.asarray(Image.open(p))


def write_image(arr: np.ndarray, path: str) -> None:
    p = Path(path)
    suf = p.suffix.lower()
    if suf == ".npy":
        np.save(p, arr)
    elif suf == ".npz":
        np.savez_compressed(p, data=arr)
    else:
        from PIL import Image

        a = np.asarray(arr)
        if a.dtype != np.uint8:
            a = a.astype(np.int32) if a.dtype.kind in "iu" else (np.clip(a, 0, 1) * 255).astype(np.uint8)
        Image.fromarray(np.squeeze(a)).save(p)


async def upload_array(model_runner, arr: np.ndarray) -> str:
    import httpx

    up = await model_runner.get_upload_url(file_type=".npy")
    buf = io.BytesIO()
    np.save(buf, arr)
    async with httpx.AsyncClient(timeout=300) as c:
        (await c.put(up["upload_url"], content=buf.getvalue())).raise_for_status()
    return up["file_path"]


async def download_array(url: str) -> np.ndarray:
    import httpx

    async with httpx.AsyncClient(timeout=300) as c:
        r = await c.get(url)
        r.raise_for_status()
    return np.load(io.BytesIO(r.content))


def worker_options(f):
    f = click.option("--worker", "worker_service_id", default=None, metavar="SERVICE_ID",
                     help="Worker service id (env BIOENGINE_WORKER_SERVICE_ID).")(f)
    f = click.option("--token", default=None, help="Auth token (env HYPHA_TOKEN / BIOENGINE_TOKEN).")(f)
    f = click.option("--server-url", default=None, help="Hub URL (env BIOENGINE_SERVER_URL).")(f)
    return f


async def worker(worker_service_id, tok, url):
    wid = worker_id(worker_service_id)
    if not wid:
        fail("no worker service id", "pass --worker or set BIOENGINE_WORKER_SERVICE_ID")
    srv = await connect(server_url(url), token(tok))
    return srv, await srv.get_service(wid)
