"""Read-only HTTP zarr store + process-wide chunk cache.

Reference: ``bioengine/datasets/http_zarr_store.py:31-245`` (zarr v3 ``Store`` over HTTP Range,
50 concurrent requests / 100 pooled connections via env) and ``chunk_cache.py:18-103`` (size-bounded
LRU, 1 GB default via ``BIOENGINE_DATASETS_ZARR_STORE_CACHE_SIZE``).

``zarr`` is not a dependency: :class:`HttpZarrStore` implements the async store calls zarr uses
(``get``/``get_partial_values``/``exists``), and :func:`read_zarr_array` decodes zarr v3 arrays
(regular chunk grid, ``bytes`` codec with optional ``gzip``) straight into numpy, so apps can
stream dataset chunks without zarr installed.  When zarr is installed, the store is usable from
``zarr.open_array(store=...)`` as well.
"""
from __future__ import annotations

import asyncio
import collections
import gzip
import itertools
import json
import os

import httpx
import numpy as np


class ChunkCache:
    def __init__(self, max_bytes: float):
        self.max_bytes = int(max_bytes)
        self.data: collections.OrderedDict[str, bytes] = collections.OrderedDict()
        self.size = 0
        self.hits = 0
        self.misses = 0
        self.lock = asyncio.Lock()

    async def get(self, key: str):
        async with self.lock:
            v = self.data.get(key)
            if v is None:
                self.misses += 1
                return None
            self.data.move_to_end(key)
            self.hits += 1
            return v

    async def put(self, key: str, value: bytes):
        n = len(value)
        if n > self.max_bytes:
            return
        async with self.lock:
            old = self.data.pop(key, None)
            if old is not None:
                self.size -= len(old)
            self.data[key] = value
            self.size += n
            while self.size > self.max_bytes and self.data:
                _, v = self.data.popitem(last=False)
                self.size -= len(v)

    async def resize(self, max_size_gb: float):
        async with self.lock:
            self.max_bytes = int(max_size_gb * 1024 ** 3)
            while self.size > self.max_bytes and self.data:
                _, v = self.data.popitem(last=False)
                self.size -= len(v)

    def clear(self):
        self.data.clear()
        self.size = 0


_CACHE: ChunkCache | None = None


def get_chunk_cache() -> ChunkCache:
    global _CACHE
    if _CACHE is None:
        gb = float(os.environ.get("BIOENGINE_DATASETS_ZARR_STORE_CACHE_SIZE", "1"))
        _CACHE = ChunkCache(gb * 1024 ** 3)
    return _CACHE


class HttpZarrStore:
    supports_writes = False
    supports_deletes = False
    supports_partial_writes = False
    supports_listing = False

    def __init__(self, base_url: str, token: str | None = None, max_concurrent: int | None = None):
        self.base_url = base_url.rstrip("/")
        self.token = token
        self.sem = asyncio.Semaphore(int(max_concurrent or os.environ.get("BIOENGINE_DATASETS_ZARR_STORE_CONCURRENT_REQUESTS", 50)))
        nconn = int(os.environ.get("BIOENGINE_DATASETS_ZARR_STORE_CONNECTIONS", 100))
        self.client = httpx.AsyncClient(timeout=60, limits=httpx.Limits(max_connections=nconn))
        self.cache = get_chunk_cache()
        self.read_only = True

    def _url(self, key: str) -> str:
        return f"{self.base_url}/{key.lstrip('/')}"

    async def get(self, key: str, prototype=None, byte_range: tuple[int, int | None] | None = None):
        ck = f"{self.base_url}|{key}|{byte_range}"
        hit = await self.cache.get(ck)
        if hit is not None:
            return hit
        headers = {}
        if byte_range is not None:
            a, b = byte_range
            headers["Range"] = f"bytes={a}-{'' if b is None else b - 1}"
        params = {"token": self.token} if self.token else None
        async with self.sem:
            r = await self.client.get(self._url(key), headers=headers, params=params)
        if r.status_code == 404:
            return None
        if r.status_code == 403:
            raise PermissionError(r.text)
        r.raise_for_status()
        data = r.content
        await self.cache.put(ck, data)
        return data

    async def get_partial_values(self, prototype, key_ranges):
        return await asyncio.gather(*[self.get(k, prototype, br) for k, br in key_ranges])

    async def exists(self, key: str) -> bool:
        return (await self.get(key)) is not None

    async def close(self):
        await self.client.aclose()


class LocalZarrStore:
    """Read-only zarr v3 store over a local directory (the same ``get`` contract as
    :class:`HttpZarrStore`, so :func:`read_zarr_array` reads regions of local and served arrays)."""

    read_only = True

    def __init__(self, root: str):
        from pathlib import Path

        self.root = Path(root)

    async def get(self, key: str, prototype=None, byte_range=None):
        from pathlib import Path

        p = (self.root / key.lstrip("/")).resolve()
        if self.root.resolve() not in p.parents and p != self.root.resolve():
            raise PermissionError(f"zarr key escapes the store: {key}")
        if not p.is_file():
            return None
        data = p.read_bytes()
        if byte_range is not None:
            a, b = byte_range
            data = data[a:b]
        return data

    async def close(self):
        pass


def zarr_shape(meta_raw: bytes) -> tuple[int, ...]:
    return tuple(json.loads(meta_raw)["shape"])


def _decode_chunk(raw: bytes, meta: dict, chunk_shape) -> np.ndarray:
    dtype = np.dtype(meta["data_type"]) if meta["data_type"] not in ("bool",) else np.dtype(bool)
    endian = "<"
    for c in meta.get("codecs", []):
        name = c.get("name")
        if name == "gzip":
            raw = gzip.decompress(raw)
        elif name == "bytes":
            endian = "<" if c.get("configuration", {}).get("endian", "little") == "little" else ">"
        elif name in ("crc32c",):
            raw = raw[:-4]
        elif name == "transpose":
            pass
        else:
            raise NotImplementedError(f"zarr codec '{name}' is not supported without zarr installed")
    dt = dtype.newbyteorder(endian) if dtype.itemsize > 1 else dtype
    return np.frombuffer(raw, dtype=dt).reshape(chunk_shape).astype(dtype, copy=False)


async def read_zarr_array(store: HttpZarrStore, path: str = "", region: tuple[slice, ...] | None = None) -> np.ndarray:
    """Read (a region of) a zarr v3 array from an HttpZarrStore into numpy."""
    prefix = f"{path.strip('/')}/" if path else ""
    meta_raw = await store.get(prefix + "zarr.json")
    if meta_raw is None:
        raise FileNotFoundError(f"{prefix}zarr.json")
    meta = json.loads(meta_raw)
    shape = tuple(meta["shape"])
    chunks = tuple(meta["chunk_grid"]["configuration"]["chunk_shape"])
    fill = meta.get("fill_value", 0) or 0
    sep = meta.get("chunk_key_encoding", {}).get("configuration", {}).get("separator", "/")
    region = region or tuple(slice(0, s) for s in shape)
    region = tuple(slice(r.start or 0, s if r.stop is None else min(r.stop, s)) for r, s in zip(region, shape))
    out = np.full([r.stop - r.start for r in region], fill, dtype=np.dtype(meta["data_type"]))
    ranges = [range(r.start // c, (r.stop - 1) // c + 1) for r, c in zip(region, chunks)]
    idxs = list(itertools.product(*ranges))

    async def fetch(ci):
        key = prefix + "c" + sep + sep.join(map(str, ci))
        raw = await store.get(key)
        return ci, raw

    for ci, raw in await asyncio.gather(*[fetch(ci) for ci in idxs]):
        if raw is None:
            continue
        arr = _decode_chunk(raw, meta, chunks)
        src, dst = [], []
        for d, (i, c, r) in enumerate(zip(ci, chunks, region)):
            c0 = i * c
            a, b = max(r.start, c0), min(r.stop, c0 + c)
            src.append(slice(a - c0, b - c0))
            dst.append(slice(a - r.start, b - r.start))
        out[tuple(dst)] = arr[tuple(src)]
    return out


def write_zarr_array(path: str, arr: np.ndarray, chunks: tuple[int, ...], compress: bool = False) -> None:
    """Write a zarr v3 array (bytes codec [+ gzip]) to a local directory (dataset authoring/tests)."""
    from pathlib import Path

    root = Path(path)
    root.mkdir(parents=True, exist_ok=True)
    codecs = [{"name": "bytes", "configuration": {"endian": "little"}}]
    if compress:
        codecs.append({"name": "gzip", "configuration": {"level": 5}})
    meta = {"zarr_format": 3, "node_type": "array", "shape": list(arr.shape), "data_type": arr.dtype.name,
            "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": list(chunks)}},
            "chunk_key_encoding": {"name": "default", "configuration": {"separator": "/"}},
            "fill_value": 0, "codecs": codecs}
    (root / "zarr.json").write_text(json.dumps(meta))
    grid = [range((s + c - 1) // c) for s, c in zip(arr.shape, chunks)]
    for ci in itertools.product(*grid):
        sl = tuple(slice(i * c, min((i + 1) * c, s)) for i, c, s in zip(ci, chunks, arr.shape))
        block = np.zeros(chunks, arr.dtype)
        part = arr[sl]
        block[tuple(slice(0, n) for n in part.shape)] = part
        raw = block.astype(block.dtype.newbyteorder("<")).tobytes()
        if compress:
            raw = gzip.compress(raw)
        p = root / "c" / Path(*map(str, ci))
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_bytes(raw)
