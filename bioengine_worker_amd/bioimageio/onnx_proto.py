"""ONNX model files without the ``onnx`` package: a protobuf wire-format reader and writer for the
subset of ``onnx.proto`` a model file uses (ModelProto / GraphProto / NodeProto / AttributeProto /
TensorProto / ValueInfoProto).

The reference runs ONNX weights through onnxruntime (``/root/reference/apps/model-runner/
runtime_deployment.py:22``, format choice at ``entry_deployment.py:1884-1887``).  Neither ``onnx`` nor
onnxruntime exists in this ROCm image, so :mod:`.onnx_runtime` executes the graph itself on PyTorch-
ROCm + the fused MFMA convs; this module only turns the file into plain Python objects.

Tensor payloads are never copied while parsing: ``raw_data`` stays a ``memoryview`` slice of the
file buffer until :func:`tensor_to_torch` materialises it (one ``frombuffer`` + copy per
initializer).  Field numbers follow the public ``onnx.proto3`` schema.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from pathlib import Path, PurePosixPath
from typing import Any

import numpy as np
import torch

# TensorProto.DataType
FLOAT, UINT8, INT8, UINT16, INT16, INT32, INT64, STRING, BOOL, FLOAT16, DOUBLE, UINT32, UINT64 = range(1, 14)
BFLOAT16 = 16
_NP = {FLOAT: np.float32, UINT8: np.uint8, INT8: np.int8, UINT16: np.uint16, INT16: np.int16, INT32: np.int32,
       INT64: np.int64, BOOL: np.bool_, FLOAT16: np.float16, DOUBLE: np.float64, UINT32: np.uint32,
       UINT64: np.uint64}
_TORCH = {FLOAT: torch.float32, UINT8: torch.uint8, INT8: torch.int8, INT16: torch.int16, INT32: torch.int32,
          INT64: torch.int64, BOOL: torch.bool, FLOAT16: torch.float16, DOUBLE: torch.float64,
          BFLOAT16: torch.bfloat16, UINT16: torch.int32, UINT32: torch.int64, UINT64: torch.int64}
_FROM_TORCH = {v: k for k, v in _TORCH.items() if k not in (UINT16, UINT32, UINT64)}

# AttributeProto.AttributeType
A_FLOAT, A_INT, A_STRING, A_TENSOR, A_GRAPH, A_FLOATS, A_INTS, A_STRINGS = 1, 2, 3, 4, 5, 6, 7, 8


# ----------------------------------------------------------------------------- wire format
def _varint(buf, i: int) -> tuple[int, int]:
    r = s = 0
    while True:
        b = buf[i]
        i += 1
        r |= (b & 0x7F) << s
        if b < 0x80:
            return r, i
        s += 7


def _fields(buf):
    """Yield (field_number, wire_type, value) over one message; length-delimited values are
    memoryview slices (no copy)."""
    i, n = 0, len(buf)
    while i < n:
        key, i = _varint(buf, i)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(buf, i)
        elif wt == 2:
            ln, i = _varint(buf, i)
            v = buf[i:i + ln]
            i += ln
        elif wt == 5:
            v = buf[i:i + 4]
            i += 4
        elif wt == 1:
            v = buf[i:i + 8]
            i += 8
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield fn, wt, v


def _sint64(v: int) -> int:
    return v - (1 << 64) if v >= (1 << 63) else v


def _packed_varints(v, wt) -> list[int]:
    if wt == 0:
        return [_sint64(v)]
    out, i = [], 0
    while i < len(v):
        x, i = _varint(v, i)
        out.append(_sint64(x))
    return out


def _packed_floats(v, wt) -> list[float]:
    if wt == 5:
        return [struct.unpack("<f", v)[0]]
    return list(np.frombuffer(v, dtype="<f4").tolist())


def _str(v) -> str:
    return bytes(v).decode("utf-8")


# ----------------------------------------------------------------------------- messages
@dataclass
class Tensor:
    name: str = ""
    dims: list = field(default_factory=list)
    data_type: int = FLOAT
    raw: Any = None                      # memoryview of raw_data
    values: list = field(default_factory=list)  # typed *_data fields
    external: dict = field(default_factory=dict)


@dataclass
class Attribute:
    name: str
    value: Any


@dataclass
class Node:
    op_type: str
    inputs: list
    outputs: list
    name: str = ""
    domain: str = ""
    attrs: dict = field(default_factory=dict)


@dataclass
class ValueInfo:
    name: str
    elem_type: int = 0
    shape: list = field(default_factory=list)  # int | str (dim_param) | None


@dataclass
class Graph:
    name: str = ""
    nodes: list = field(default_factory=list)
    initializers: list = field(default_factory=list)
    inputs: list = field(default_factory=list)
    outputs: list = field(default_factory=list)


@dataclass
class Model:
    ir_version: int = 0
    opset: dict = field(default_factory=dict)   # domain -> version
    producer: str = ""
    graph: Graph = field(default_factory=Graph)


def _tensor(buf) -> Tensor:
    t = Tensor()
    for fn, wt, v in _fields(buf):
        if fn == 1:
            t.dims += _packed_varints(v, wt)
        elif fn == 2:
            t.data_type = v
        elif fn == 8:
            t.name = _str(v)
        elif fn == 9:
            t.raw = v
        elif fn == 4:
            t.values += _packed_floats(v, wt)
        elif fn in (5, 7, 11):
            t.values += _packed_varints(v, wt)
        elif fn == 10:
            t.values += (np.frombuffer(v, dtype="<f8").tolist() if wt == 2 else [struct.unpack("<d", v)[0]])
        elif fn == 13:  # external_data: StringStringEntryProto
            kv = {}
            for f2, _, v2 in _fields(v):
                kv[f2] = _str(v2)
            t.external[kv.get(1, "")] = kv.get(2, "")
    return t


def _value_info(buf) -> ValueInfo:
    vi = ValueInfo("")
    for fn, _, v in _fields(buf):
        if fn == 1:
            vi.name = _str(v)
        elif fn == 2:  # TypeProto
            for f2, _, v2 in _fields(v):
                if f2 != 1:  # tensor_type only
                    continue
                for f3, _, v3 in _fields(v2):
                    if f3 == 1:
                        vi.elem_type = v3
                    elif f3 == 2:  # TensorShapeProto
                        for f4, _, v4 in _fields(v3):
                            if f4 != 1:
                                continue
                            d = None
                            for f5, _, v5 in _fields(v4):
                                d = v5 if f5 == 1 else _str(v5) if f5 == 2 else d
                            vi.shape.append(d)
    return vi


def _attribute(buf) -> Attribute:
    name, typ = "", 0
    f = i = s = t = g = None
    floats, ints, strings = [], [], []
    for fn, wt, v in _fields(buf):
        if fn == 1:
            name = _str(v)
        elif fn == 20:
            typ = v
        elif fn == 2:
            f = struct.unpack("<f", v)[0]
        elif fn == 3:
            i = _sint64(v)
        elif fn == 4:
            s = bytes(v)
        elif fn == 5:
            t = _tensor(v)
        elif fn == 6:
            g = _graph(v)
        elif fn == 7:
            floats += _packed_floats(v, wt)
        elif fn == 8:
            ints += _packed_varints(v, wt)
        elif fn == 9:
            strings.append(bytes(v))
    by_type = {A_FLOAT: f, A_INT: i, A_STRING: s, A_TENSOR: t, A_GRAPH: g, A_FLOATS: floats, A_INTS: ints,
               A_STRINGS: strings}
    if typ in by_type:
        val = by_type[typ]
    else:  # pre-IR-3 files omit ``type``: take whichever field is set
        val = next((x for x in (f, i, s, t, g) if x is not None), floats or ints or strings)
    if isinstance(val, bytes):
        val = val.decode("utf-8", "replace")
    return Attribute(name, val)


def _node(buf) -> Node:
    n = Node("", [], [])
    for fn, _, v in _fields(buf):
        if fn == 1:
            n.inputs.append(_str(v))
        elif fn == 2:
            n.outputs.append(_str(v))
        elif fn == 3:
            n.name = _str(v)
        elif fn == 4:
            n.op_type = _str(v)
        elif fn == 7:
            n.domain = _str(v)
        elif fn == 5:
            a = _attribute(v)
            n.attrs[a.name] = a.value
    return n


def _graph(buf) -> Graph:
    g = Graph()
    for fn, _, v in _fields(buf):
        if fn == 1:
            g.nodes.append(_node(v))
        elif fn == 2:
            g.name = _str(v)
        elif fn == 5:
            g.initializers.append(_tensor(v))
        elif fn == 11:
            g.inputs.append(_value_info(v))
        elif fn == 12:
            g.outputs.append(_value_info(v))
    return g


def parse_model(data) -> Model:
    buf = memoryview(data)
    m = Model()
    for fn, _, v in _fields(buf):
        if fn == 1:
            m.ir_version = v
        elif fn == 2:
            m.producer = _str(v)
        elif fn == 7:
            m.graph = _graph(v)
        elif fn == 8:
            dom, ver = "", 1
            for f2, _, v2 in _fields(v):
                dom = _str(v2) if f2 == 1 else dom
                ver = v2 if f2 == 2 else ver
            m.opset[dom] = ver
    if not m.opset:
        m.opset[""] = 1
    return m


def load_model(path) -> Model:
    with open(path, "rb") as f:
        data = f.read()
    m = parse_model(data)
    m._base = str(path)  # external-data tensors resolve against the model's directory
    return m


def external_data_path(base_dir, location: str) -> Path:
    """Resolve an initializer's ``external_data`` location inside the model directory.

    Model packages are untrusted input: an absolute location or one with a ``..`` part could make
    the loader read any file the worker can read (and echo it back through an Identity output), so
    both are rejected, as is anything that resolves (symlinks included) outside ``base_dir``."""
    if not isinstance(location, str) or not location or "\x00" in location:
        raise ValueError("external data location must be a non-empty relative path")
    norm = location.replace("\\", "/")
    if norm.startswith("/") or PurePosixPath(norm).is_absolute() or (len(norm) > 1 and norm[1] == ":"):
        raise ValueError(f"external data location '{location}' is absolute")
    if any(part == ".." for part in PurePosixPath(norm).parts):
        raise ValueError(f"external data location '{location}' leaves the model directory")
    base = Path(base_dir or ".").resolve()
    path = (base / norm).resolve()
    if path != base and base not in path.parents:
        raise ValueError(f"external data location '{location}' resolves outside the model directory")
    if not path.is_file():
        raise FileNotFoundError(f"external data file '{location}' not found next to the model")
    return path


def tensor_to_torch(t: Tensor, base_dir=None) -> torch.Tensor:
    """Materialise a TensorProto as a CPU torch tensor (copies out of the file buffer)."""
    dt = t.data_type
    shape = [int(d) for d in t.dims]
    n = int(np.prod(shape)) if shape else 1
    if t.external:
        loc = external_data_path(base_dir, t.external.get("location", ""))
        size = loc.stat().st_size
        off, ln = int(t.external.get("offset", 0) or 0), t.external.get("length")
        ln = None if ln in (None, "") else int(ln)
        if off < 0 or off > size or (ln is not None and (ln < 0 or off + ln > size)):
            raise ValueError(f"external data of '{t.name}' (offset {off}, length {ln}) exceeds {loc.name} ({size} B)")
        with open(loc, "rb") as f:
            f.seek(off)
            raw = f.read(ln if ln is not None else -1)
        t = Tensor(t.name, t.dims, dt, memoryview(raw))
    if t.raw is not None and len(t.raw):
        if dt == BFLOAT16:
            a = np.frombuffer(t.raw, dtype="<u2").astype(np.int32) << 16
            return torch.from_numpy(a.view(np.float32).copy()).to(torch.bfloat16).reshape(shape)
        a = np.frombuffer(t.raw, dtype=np.dtype(_NP[dt]).newbyteorder("<"), count=n).copy()
    elif dt == FLOAT16:  # int32_data holds the fp16 bit patterns
        a = np.asarray(t.values, dtype=np.uint16).view(np.float16)
    elif dt == BFLOAT16:
        a = (np.asarray(t.values, dtype=np.int32) << 16).view(np.float32)
        return torch.from_numpy(a.copy()).to(torch.bfloat16).reshape(shape)
    else:
        a = np.asarray(t.values, dtype=_NP[dt]) if t.values else np.zeros(n, dtype=_NP[dt])
    if dt in (UINT16, UINT32, UINT64):
        a = a.astype(np.int64 if dt != UINT16 else np.int32)
    return torch.from_numpy(np.ascontiguousarray(a)).reshape(shape)


# ----------------------------------------------------------------------------- writer
def _enc_varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(fn: int, wt: int) -> bytes:
    return _enc_varint((fn << 3) | wt)


def _ld(fn: int, payload: bytes) -> bytes:
    return _key(fn, 2) + _enc_varint(len(payload)) + payload


def _vint(fn: int, v: int) -> bytes:
    return _key(fn, 0) + _enc_varint(v)


def encode_tensor(name: str, value) -> bytes:
    t = value if torch.is_tensor(value) else torch.as_tensor(np.asarray(value))
    t = t.detach().cpu().contiguous()
    dt = _FROM_TORCH[t.dtype]
    out = b"".join(_vint(1, d) for d in t.shape) + _vint(2, dt) + _ld(8, name.encode())
    if t.dtype == torch.bfloat16:
        raw = t.view(torch.int16).numpy().tobytes()
    else:
        raw = t.numpy().astype(np.dtype(_NP[dt]).newbyteorder("<"), copy=False).tobytes()
    return out + _ld(9, raw)


def _encode_attr(name: str, v) -> bytes:
    out = _ld(1, name.encode())
    if isinstance(v, bool) or isinstance(v, int):
        return out + _key(3, 0) + _enc_varint(int(v)) + _vint(20, A_INT)
    if isinstance(v, float):
        return out + _key(2, 5) + struct.pack("<f", v) + _vint(20, A_FLOAT)
    if isinstance(v, str):
        return out + _ld(4, v.encode()) + _vint(20, A_STRING)
    if torch.is_tensor(v) or isinstance(v, np.ndarray):
        return out + _ld(5, encode_tensor("", v)) + _vint(20, A_TENSOR)
    if isinstance(v, (list, tuple)):
        if all(isinstance(x, int) for x in v):
            return out + _ld(8, b"".join(_enc_varint(int(x)) for x in v)) + _vint(20, A_INTS)
        if all(isinstance(x, (int, float)) for x in v):
            return out + _ld(7, struct.pack(f"<{len(v)}f", *v)) + _vint(20, A_FLOATS)
        return out + b"".join(_ld(9, str(x).encode()) for x in v) + _vint(20, A_STRINGS)
    raise TypeError(f"attribute {name}: unsupported value {type(v)}")


def _encode_value_info(name: str, elem_type: int = FLOAT, shape=None) -> bytes:
    dims = b""
    for d in shape or []:
        dims += _ld(1, _vint(1, d) if isinstance(d, int) else _ld(2, str(d).encode()))
    tt = _vint(1, elem_type) + (_ld(2, dims) if shape is not None else b"")
    return _ld(1, name.encode()) + _ld(2, _ld(1, tt))


class GraphBuilder:
    """Writes ONNX model files (test fixtures and exports): ``node(op, inputs, outputs, **attrs)``,
    ``init(name, tensor)``, ``input``/``output`` declarations, then ``to_bytes()`` / ``save(path)``."""

    def __init__(self, name: str = "graph", opset: int = 17):
        self.name, self.opset = name, opset
        self._nodes, self._inits, self._ins, self._outs = [], [], [], []
        self._n = 0

    def input(self, name, shape=None, elem_type=FLOAT):
        self._ins.append(_encode_value_info(name, elem_type, shape))
        return name

    def output(self, name, shape=None, elem_type=FLOAT):
        self._outs.append(_encode_value_info(name, elem_type, shape))
        return name

    def init(self, name, value):
        self._inits.append(encode_tensor(name, value))
        return name

    def node(self, op, inputs, outputs=None, domain: str = "", **attrs):
        if outputs is None:
            self._n += 1
            outputs = [f"{op.lower()}_{self._n}"]
        elif isinstance(outputs, str):
            outputs = [outputs]
        body = b"".join(_ld(1, x.encode()) for x in inputs) + b"".join(_ld(2, x.encode()) for x in outputs)
        body += _ld(3, f"{op}_{len(self._nodes)}".encode()) + _ld(4, op.encode())
        if domain:
            body += _ld(7, domain.encode())
        body += b"".join(_ld(5, _encode_attr(k, v)) for k, v in attrs.items())
        self._nodes.append(body)
        return outputs[0] if len(outputs) == 1 else outputs

    def to_bytes(self) -> bytes:
        g = b"".join(_ld(1, n) for n in self._nodes) + _ld(2, self.name.encode())
        g += b"".join(_ld(5, t) for t in self._inits) + b"".join(_ld(11, x) for x in self._ins)
        g += b"".join(_ld(12, x) for x in self._outs)
        opset = _ld(1, b"") + _vint(2, self.opset)
        return _vint(1, 8) + _ld(2, b"bioengine_worker_amd") + _ld(7, g) + _ld(8, opset)

    def save(self, path) -> None:
        with open(path, "wb") as f:
            f.write(self.to_bytes())
