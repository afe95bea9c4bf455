"""Datasets client injected into every app replica as ``self.bioengine_datasets``
(reference: ``bioengine/datasets/datasets.py:11-462``, injected at ``bioengine/apps/builder.py:656-661``).

``get_file`` returns an :class:`~.store.HttpZarrStore` for ``*.zarr`` paths (chunk-wise HTTP range
reads with an LRU chunk cache) and raw bytes otherwise.  Requests use exponential-backoff retry
(4 attempts; 4xx other than 429 is final — reference ``datasets/utils/network.py:8-73``).
"""
from __future__ import annotations

import asyncio
import logging
import os
from pathlib import Path

import httpx

from .server import DISCOVERY_FILE
from .store import HttpZarrStore, get_chunk_cache


async def get_url_with_retry(client: httpx.AsyncClient, url: str, params=None, headers=None, attempts: int = 4,
                             backoff: float = 0.25) -> httpx.Response:
    last = None
    for i in range(attempts):
        try:
            r = await client.get(url, params=params, headers=headers)
            if r.status_code < 400 or (400 <= r.status_code < 500 and r.status_code != 429):
                return r
            last = r
        except httpx.TransportError as e:
            last = e
        await asyncio.sleep(backoff * (2 ** i))
    if isinstance(last, httpx.Response):
        return last
    raise last  # type: ignore[misc]


class BioEngineDatasets:
    def __init__(self, data_server_url: str | None = "auto", hypha_token: str | None = None, logger=None,
                 timeout: float = 30.0):
        self.logger = logger or logging.getLogger("bioengine.datasets")
        if data_server_url == "auto":
            data_server_url = self.discover()
        self.data_server_url = data_server_url.rstrip("/") if data_server_url else None
        self.token = hypha_token
        self.timeout = timeout
        self._client: httpx.AsyncClient | None = None

    @staticmethod
    def discover() -> str | None:
        env = os.environ.get("BIOENGINE_DATA_SERVER_URL")
        if env:
            return env
        try:
            return Path(DISCOVERY_FILE).read_text().strip() or None
        except OSError:
            return None

    def _c(self) -> httpx.AsyncClient:
        if self._client is None or self._client.is_closed:
            self._client = httpx.AsyncClient(timeout=self.timeout)
        return self._client

    def _require(self):
        if not self.data_server_url:
            raise RuntimeError("No BioEngine datasets server is configured or discoverable")

    def _params(self, extra=None):
        p = dict(extra or {})
        if self.token:
            p["token"] = self.token
        return p

    async def set_chunk_cache_size_gb(self, gb: float) -> None:
        await get_chunk_cache().resize(gb)

    async def ping_data_server(self) -> bool:
        if not self.data_server_url:
            return False
        r = await get_url_with_retry(self._c(), f"{self.data_server_url}/ping", attempts=2)
        if r.status_code != 200:
            raise RuntimeError(f"datasets server unhealthy: HTTP {r.status_code}")
        return True

    async def list_datasets(self) -> dict:
        self._require()
        r = await get_url_with_retry(self._c(), f"{self.data_server_url}/datasets")
        r.raise_for_status()
        return r.json()

    async def list_files(self, dataset_id: str, dir_path: str | None = None) -> list[str]:
        self._require()
        p = self._params({"dir_path": dir_path} if dir_path else None)
        r = await get_url_with_retry(self._c(), f"{self.data_server_url}/datasets/{dataset_id}/files", params=p)
        if r.status_code == 403:
            raise PermissionError(r.json().get("detail"))
        if r.status_code >= 400:
            raise ValueError(r.json().get("detail", r.text))
        return r.json()

    async def get_file(self, dataset_id: str, file_path: str):
        self._require()
        if file_path.rstrip("/").endswith(".zarr") or ".zarr/" in file_path:
            root = file_path.split(".zarr")[0] + ".zarr"
            return HttpZarrStore(f"{self.data_server_url}/data/{dataset_id}/{root}", token=self.token)
        r = await get_url_with_retry(self._c(), f"{self.data_server_url}/data/{dataset_id}/{file_path}",
                                     params=self._params())
        if r.status_code == 403:
            raise PermissionError(r.json().get("detail"))
        if r.status_code == 404:
            raise FileNotFoundError(file_path)
        r.raise_for_status()
        return r.content

    async def save_file(self, filename: str, content: bytes | str, public: bool = False) -> dict:
        self._require()
        data = content.encode() if isinstance(content, str) else bytes(content)
        r = await self._c().post(f"{self.data_server_url}/save", params=self._params({"filename": filename,
                                                                                      "public": str(public).lower()}),
                                 content=data)
        if r.status_code >= 400:
            raise RuntimeError(f"save failed: HTTP {r.status_code} {r.text[:200]}")
        return r.json()

    async def list_saved_files(self) -> dict:
        self._require()
        r = await get_url_with_retry(self._c(), f"{self.data_server_url}/saved", params=self._params())
        r.raise_for_status()
        return r.json()

    async def get_saved_file(self, filename: str, public: bool | None = None) -> bytes:
        self._require()
        extra = {} if public is None else {"public": str(public).lower()}
        r = await get_url_with_retry(self._c(), f"{self.data_server_url}/saved/{filename}", params=self._params(extra))
        if r.status_code == 404:
            raise FileNotFoundError(filename)
        r.raise_for_status()
        return r.content

    async def close(self):
        if self._client is not None:
            await self._client.aclose()
