"""Wire encoding for the hub WebSocket protocol: msgpack with numpy/tensor and callback extensions.

* ndarray / torch tensor  -> ext 1: {dtype, shape} header + raw C-order bytes (zero-copy decode
  via ``np.frombuffer``), so image payloads cross process boundaries without pickling.
* callable                -> ``{"__rpc_cb__": id}``; the receiver gets a proxy that calls back
  through the hub (used for ``run_code`` stdout/stderr streaming).
* exceptions travel as ``{"type", "message", "traceback"}`` and are re-raised as
  :class:`RemoteError` (type name preserved in the message).
"""
from __future__ import annotations

import json
import traceback
from typing import Any, Callable

import msgpack
import numpy as np

EXT_NDARRAY = 1


class RemoteError(Exception):
    def __init__(self, type_name: str, message: str, tb: str = ""):
        super().__init__(f"{type_name}: {message}")
        self.type_name = type_name
        self.remote_traceback = tb


def _default(obj, cb_register: Callable | None):
    if isinstance(obj, np.ndarray):
        a = np.ascontiguousarray(obj)
        head = json.dumps({"dtype": a.dtype.str, "shape": list(a.shape)}).encode()
        return msgpack.ExtType(EXT_NDARRAY, len(head).to_bytes(4, "little") + head + a.tobytes())
    if isinstance(obj, np.generic):
        return obj.item()
    try:
        import torch

        if isinstance(obj, torch.Tensor):
            return _default(obj.detach().cpu().numpy(), cb_register)
    except ImportError:  # pragma: no cover
        pass
    if isinstance(obj, (set, frozenset, tuple)):
        return list(obj)
    if callable(obj) and cb_register is not None:
        return {"__rpc_cb__": cb_register(obj)}
    if hasattr(obj, "model_dump"):
        return obj.model_dump()
    if hasattr(obj, "__dict__") and not isinstance(obj, type):
        return {k: v for k, v in vars(obj).items() if not k.startswith("_")}
    return str(obj)


def _ext_hook(code, data):
    if code == EXT_NDARRAY:
        n = int.from_bytes(data[:4], "little")
        head = json.loads(data[4: 4 + n])
        arr = np.frombuffer(data, dtype=np.dtype(head["dtype"]), offset=4 + n)
        return arr.reshape(head["shape"]).copy()
    return msgpack.ExtType(code, data)


def pack(msg: Any, cb_register: Callable | None = None) -> bytes:
    return msgpack.packb(msg, default=lambda o: _default(o, cb_register), use_bin_type=True, strict_types=False)


def unpack(data: bytes, cb_factory: Callable | None = None) -> Any:
    obj = msgpack.unpackb(data, ext_hook=_ext_hook, raw=False, strict_map_key=False)
    if cb_factory is not None:
        obj = _revive(obj, cb_factory)
    return obj


def _revive(obj, cb_factory):
    if isinstance(obj, dict):
        if "__rpc_cb__" in obj and len(obj) == 1:
            return cb_factory(obj["__rpc_cb__"])
        return {k: _revive(v, cb_factory) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_revive(v, cb_factory) for v in obj]
    return obj


def error_payload(e: BaseException) -> dict:
    return {"type": type(e).__name__, "message": str(e), "traceback": "".join(traceback.format_exception(e))[-4000:]}


def raise_remote(err: dict):
    t = err.get("type", "Exception")
    builtin = {"PermissionError": PermissionError, "KeyError": KeyError, "ValueError": ValueError,
               "TimeoutError": TimeoutError, "FileNotFoundError": FileNotFoundError, "RuntimeError": RuntimeError}
    cls = builtin.get(t)
    if cls is not None:
        raise cls(f"{err.get('message')}") from RemoteError(t, err.get("message", ""), err.get("traceback", ""))
    raise RemoteError(t, err.get("message", ""), err.get("traceback", ""))
