"""Python face of the C++ shared-memory SPSC ring (``csrc/runtime/shm_ring.cpp``).

The serving runtime pairs every process replica with two rings (router -> replica and
replica -> router).  Request/response *headers* (pickle protocol 5) still travel over the replica's
Unix socket, while the out-of-band buffers — the ndarrays / tensors of images, volumes and masks —
are published into the ring as one atomic multi-frame message, so a 64 MiB volume crosses the
process boundary as one memcpy in and one memcpy out instead of socket chunking through the
kernel.  Replaces the Ray object store between the reference's proxy, entry and runtime
deployments (reference ``bioengine/apps/proxy_deployment.py:522-554``,
``apps/model-runner/entry_deployment.py`` → ``runtime_deployment.py`` handle calls).
"""
from __future__ import annotations

import ctypes
import os
import uuid

import numpy as np

from ..ops import _native

EAGAIN_TIMEOUT, TOO_LARGE, CLOSED = -2, -3, -4


_MALLOC_TUNED = False


def tune_malloc(role: str = "replica") -> bool:
    """Keep freed payload-sized buffers in the process heap (``BE_REPLICA_MALLOC``, default on).

    ``role="router"``: the router is the main worker process that hosts every in-process app, so a
    process-wide 512 MiB trim threshold there could hold large amounts of freed memory across its
    many threads' arenas; it is applied there only when ``BE_ROUTER_MALLOC=1``.

    Every ring read allocates a fresh array for the payload; glibc serves multi-MiB requests from
    fresh mmaps, or trims the heap top after a free, so each request may page-fault its buffer in
    again (~1 ms per MiB on the VM hosts, see ``map_ring`` in shm_ring.cpp).  With the mmap
    threshold at 64 MiB and the trim threshold at 512 MiB, the freed buffers are reused instead.
    Applied once per replica process.  Measured on an MI355X box with the parallel ring
    copies (tools/replica_hop_bench.py, profiles/r04/serve/replica_hop_ab.jsonl): a 2 MiB request
    round trip 245 us -> 191 us (4 copy threads) -> 150 us (+ this)."""
    global _MALLOC_TUNED
    if _MALLOC_TUNED or os.environ.get("BE_REPLICA_MALLOC", "1") in ("0", "false", "no"):
        return _MALLOC_TUNED
    if role == "router" and os.environ.get("BE_ROUTER_MALLOC", "0") not in ("1", "true", "yes"):
        return False
    try:
        libc = ctypes.CDLL("libc.so.6")
        ok = libc.mallopt(-3, 64 << 20) == 1 and libc.mallopt(-1, 512 << 20) == 1  # M_MMAP_THRESHOLD, M_TRIM_THRESHOLD
    except OSError:
        ok = False
    _MALLOC_TUNED = ok
    return ok


class RingClosed(RuntimeError):
    pass


def _populate_default() -> int:
    """Pre-fault ring mappings (``BE_RING_POPULATE``, default on): see ``map_ring`` in shm_ring.cpp."""
    return 0 if os.environ.get("BE_RING_POPULATE", "1") in ("0", "false", "no") else 1


def _addr(buf) -> int:
    """Address of a (possibly read-only) contiguous buffer without copying it."""
    a = np.frombuffer(buf, dtype=np.uint8)
    return a.ctypes.data if a.size else 0


class ShmRing:
    """One direction of a bulk-data channel.  ``create`` on the owning side, ``open`` on the peer;
    exactly one thread writes and one thread reads."""

    def __init__(self, handle: int, name: str, owner: bool):
        self._h = ctypes.c_void_p(handle)
        self.name = name
        self.owner = owner
        self._rt = _native.runtime()

    @classmethod
    def create(cls, capacity: int = 256 << 20, name: str | None = None, populate: bool | None = None) -> "ShmRing":
        name = name or f"/be-ring-{os.getpid()}-{uuid.uuid4().hex[:10]}"
        h = ctypes.c_void_p()
        pop = _populate_default() if populate is None else int(bool(populate))
        rc = _native.runtime().be_rt_ring_create(name.encode(), int(capacity), ctypes.byref(h), pop)
        if rc != 0:
            raise OSError(-rc, f"shm ring create {name}: {os.strerror(-rc)}")
        return cls(h.value, name, True)

    @classmethod
    def open(cls, name: str, populate: bool | None = None) -> "ShmRing":
        h = ctypes.c_void_p()
        pop = _populate_default() if populate is None else int(bool(populate))
        rc = _native.runtime().be_rt_ring_open(name.encode(), ctypes.byref(h), pop)
        if rc != 0:
            raise OSError(-rc, f"shm ring open {name}: {os.strerror(-rc)}")
        return cls(h.value, name, False)

    # ------------------------------------------------------------------ producer
    @property
    def capacity(self) -> int:
        return self.stats()["capacity"]

    def fits(self, lens) -> bool:
        return sum(8 + ((int(n) + 7) & ~7) for n in lens) <= self.capacity

    def write(self, bufs, timeout_s: float | None = 60.0) -> None:
        """Publish ``bufs`` (bytes-like objects) as one message; blocks while the ring is full."""
        n = len(bufs)
        ptrs = (ctypes.c_void_p * max(1, n))(*[_addr(b) for b in bufs])
        lens = (ctypes.c_int64 * max(1, n))(*[memoryview(b).nbytes for b in bufs])
        rc = self._rt.be_rt_ring_write(self._h, ptrs, lens, n, -1 if timeout_s is None else int(timeout_s * 1e6))
        if rc == TOO_LARGE:
            raise ValueError(f"message of {sum(lens[:n])} bytes exceeds ring capacity {self.capacity}")
        if rc == EAGAIN_TIMEOUT:
            raise TimeoutError(f"shm ring {self.name} full for {timeout_s}s")
        if rc == CLOSED:
            raise RingClosed(self.name)
        if rc != 0:
            raise OSError(-rc, f"shm ring write: {os.strerror(-rc)}")

    # ------------------------------------------------------------------ consumer
    def read(self, timeout_s: float | None = 60.0) -> np.ndarray:
        """Next frame's payload as a fresh writable uint8 array (``np.empty``: no zero-fill pass before
        the copy, unlike ``bytearray(n)``)."""
        n = ctypes.c_int64()
        rc = self._rt.be_rt_ring_next_len(self._h, ctypes.byref(n), -1 if timeout_s is None else int(timeout_s * 1e6))
        if rc == EAGAIN_TIMEOUT:
            raise TimeoutError(f"shm ring {self.name} empty for {timeout_s}s")
        if rc == CLOSED:
            raise RingClosed(self.name)
        if rc != 0:
            raise OSError(-rc, f"shm ring wait: {os.strerror(-rc)}")
        out = np.empty(n.value, np.uint8)
        rc = self._rt.be_rt_ring_read(self._h, ctypes.c_void_p(out.ctypes.data if n.value else 0), n.value)
        if rc != 0:
            raise OSError(-rc, "shm ring read")
        return out

    # ------------------------------------------------------------------ lifecycle
    def stats(self) -> dict:
        o = (ctypes.c_int64 * 5)()
        self._rt.be_rt_ring_stats(self._h, o)
        return {"capacity": o[0], "queued_bytes": o[1], "frames": o[2], "bytes": o[3], "closed": bool(o[4])}

    def unlink(self) -> None:
        """Remove the name (mappings stay valid); call once both sides have opened it."""
        self._rt.be_rt_ring_unlink(self.name.encode())

    def shutdown(self) -> None:
        if self._h:
            self._rt.be_rt_ring_shutdown(self._h)

    def close(self) -> None:
        if self._h:
            self._rt.be_rt_ring_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self.close()
        except Exception:
            pass
