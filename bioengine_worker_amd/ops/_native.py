"""Loader for the in-tree native libraries (``_native/libbe_hip.so``, ``_native/libbe_runtime.so``).

The HIP library is a plain C-ABI shared object built by ``tools/build_native.py`` with
``hipcc --offload-arch=gfx950``.  It is loaded with ``ctypes`` *after* ``import torch`` so that its
``libamdhip64.so.7`` dependency resolves to the HIP runtime PyTorch already mapped (one runtime per
process, shared streams).  Kernels are launched on PyTorch's current HIP stream, so they order
correctly with torch ops and are captured by ``torch.cuda.graphs`` / hipGraph capture.

Policy: on a GPU tensor the HIP kernel is the only path — if the library is missing or fails to
load, ops raise (``NativeUnavailable``) instead of silently falling back.  CPU tensors run the
PyTorch fp32 reference of the same op (the numerics oracle used by tests).
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

import torch

_HERE = Path(__file__).resolve().parent.parent / "_native"
_lock = threading.Lock()
_hip = None
_rt = None
_hip_err: str | None = None


class NativeUnavailable(RuntimeError):
    pass


c_int = ctypes.c_int
c_float = ctypes.c_float
c_void_p = ctypes.c_void_p
c_int64 = ctypes.c_int64

# name -> argtypes (restype int).  'p' = pointer, 'i' = int32, 'f' = float32, 'l' = int64,
# 's' = stream.  Generated at build time from the C prototypes (tools/build_native.py), so the
# Python side can never drift from the kernels' ABI.
_HIP_SIGS: dict[str, str] = {}


def _ctype(ch):
    return {"p": c_void_p, "i": c_int, "f": c_float, "l": c_int64, "s": c_void_p, "d": ctypes.c_double}[ch]


def _bind(lib, sigs):
    for name, sig in sigs.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = [_ctype(c) for c in sig]
        fn.restype = c_int


def register_hip_signatures(sigs: dict[str, str]) -> None:
    """Kept for op modules that want to document their entry points; the generated
    ``hip_signatures.json`` is authoritative when present."""
    for k, v in sigs.items():
        _HIP_SIGS.setdefault(k, v)


def hip_lib_path() -> Path:
    return Path(os.environ.get("BE_HIP_LIB", _HERE / "libbe_hip.so"))


def hip():
    """Return the loaded HIP kernel library, raising NativeUnavailable if it cannot be loaded."""
    global _hip, _hip_err
    if _hip is not None:
        return _hip
    with _lock:
        if _hip is not None:
            return _hip
        p = hip_lib_path()
        if not p.exists():
            _hip_err = f"{p} not built (run `python tools/build_native.py`)"
            raise NativeUnavailable(_hip_err)
        try:
            lib = ctypes.CDLL(str(p), mode=ctypes.RTLD_GLOBAL)
        except OSError as e:  # pragma: no cover - depends on box
            _hip_err = str(e)
            raise NativeUnavailable(f"failed to load {p}: {e}") from e
        sig_file = p.parent / "hip_signatures.json"
        if sig_file.exists():
            import json

            _HIP_SIGS.update(json.loads(sig_file.read_text()))
        _bind(lib, _HIP_SIGS)
        _hip = lib
        return _hip


def runtime():
    """Host runtime library (CPU only; always loadable where it was built)."""
    global _rt
    if _rt is not None:
        return _rt
    with _lock:
        if _rt is None:
            p = Path(os.environ.get("BE_RUNTIME_LIB", _HERE / "libbe_runtime.so"))
            if not p.exists():
                raise NativeUnavailable(f"{p} not built (run `python tools/build_native.py`)")
            lib = ctypes.CDLL(str(p))
            sig_file = p.parent / "runtime_signatures.json"
            if sig_file.exists():
                import json

                _bind(lib, json.loads(sig_file.read_text()))
            _rt = lib
    return _rt


def rt_call(name: str, *args) -> None:
    """Call a host-runtime (C++) entry point and raise on a non-zero status."""
    fn = getattr(runtime(), name)
    if fn.argtypes is not None and len(fn.argtypes) != len(args):
        raise TypeError(f"{name}: expected {len(fn.argtypes)} args, got {len(args)}")
    rc = fn(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with status {rc}")


def hip_available() -> bool:
    if not torch.cuda.is_available():
        return False
    try:
        hip()
        return True
    except NativeUnavailable:
        return False


def loaded_libraries() -> list[str]:
    out = []
    if _hip is not None:
        out.append(str(hip_lib_path()))
    if _rt is not None:
        out.append("libbe_runtime.so")
    return out


class _TensorPtr(c_void_p):
    """A tensor's device address that keeps the tensor alive.  Call sites often pass converted
    temporaries (``ptr(q.float().contiguous())``, ``ptr(probes.int())``): with a bare address the
    first temporary is freed while the argument list is still being built, the next conversion is
    allocated into the same caching-allocator block and overwrites it before the kernel is even
    launched (the IVF scan once read its query block as the probe-index integers).  Holding the
    tensor until ``call`` returns keeps every operand distinct; after the launch, stream order
    protects the memory."""

    __slots__ = ("_t",)


_KEEP = os.environ.get("BE_NATIVE_PTR_KEEP", "1") != "0"  # 0: bare addresses (A/B only)


def ptr(t: torch.Tensor | None):
    if t is None:
        return None
    if not _KEEP:
        return c_void_p(t.data_ptr())
    p = _TensorPtr(t.data_ptr())
    p._t = t
    return p


def stream(device: torch.device | int | None = None):
    """The current HIP stream of ``device`` as a ``c_void_p``.  Reads the raw handle straight from
    the C++ stream registry: ``torch.cuda.current_stream(dev)`` builds a Python Stream object and
    re-resolves the device on every call (~5 us; 60+ calls per batch-1 Cellpose request)."""
    if isinstance(device, torch.device):
        idx = device.index
    else:
        idx = device
    if idx is None:
        idx = torch.cuda.current_device()
    return c_void_p(torch._C._cuda_getCurrentRawStream(idx))


def call(name: str, *args) -> None:
    """Call a HIP entry point and raise on a non-zero status."""
    lib = hip()
    fn = getattr(lib, name)
    if fn.argtypes is not None and len(fn.argtypes) != len(args):
        raise TypeError(f"{name}: expected {len(fn.argtypes)} args, got {len(args)}")
    rc = fn(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with status {rc}")
