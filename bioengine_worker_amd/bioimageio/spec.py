"""BioImage.IO resource description (RDF) handling: load, validate, axes and sizes.

Covers model RDF format 0.4.x (axes strings such as ``"bcyx"``, ``shape: {min, step}``) and
0.5.x (axis lists with ``type``/``id``/``size``/``halo``), normalised into :class:`TensorSpec`.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any

import yaml

REQUIRED_MODEL_FIELDS = ("format_version", "type", "name", "inputs", "outputs", "weights")
WEIGHT_FORMATS = ("pytorch_state_dict", "torchscript", "onnx", "tensorflow_saved_model", "keras_hdf5")


@dataclass
class AxisSpec:
    id: str            # b, c, z, y, x, t, i
    type: str          # batch | channel | space | time | index
    size: Any = None   # int | {"min","step"} | {"tensor_id","axis_id"} | None
    halo: int = 0
    scale: float = 1.0
    offset: int = 0
    channel_names: list | None = None


@dataclass
class TensorSpec:
    id: str
    axes: list[AxisSpec]
    data_type: str = "float32"
    preprocessing: list = field(default_factory=list)
    postprocessing: list = field(default_factory=list)
    test_tensor: str | None = None
    sample_tensor: str | None = None

    @property
    def axis_ids(self) -> list[str]:
        return [a.id for a in self.axes]

    def axis(self, aid: str) -> AxisSpec | None:
        for a in self.axes:
            if a.id == aid:
                return a
        return None


_TYPE_OF = {"b": "batch", "c": "channel", "z": "space", "y": "space", "x": "space", "t": "time", "i": "index"}


def _src(v):
    if isinstance(v, dict):
        return v.get("source") or v.get("uri")
    if isinstance(v, list):
        return _src(v[0]) if v else None
    return v


def _axes_04(t: dict, is_output: bool) -> list[AxisSpec]:
    ax = list(t["axes"])
    shape = t.get("shape")
    halo = t.get("halo") or [0] * len(ax)
    out = []
    for i, a in enumerate(ax):
        size = None
        if isinstance(shape, list):
            size = shape[i]
        elif isinstance(shape, dict):
            if "min" in shape:
                size = {"min": shape["min"][i], "step": shape["step"][i]}
            elif "reference_tensor" in shape:
                size = {"tensor_id": shape["reference_tensor"], "axis_id": a,
                        "scale": shape["scale"][i], "offset": shape["offset"][i]}
        out.append(AxisSpec(id=a, type=_TYPE_OF.get(a, "space"), size=size, halo=int(halo[i]) if is_output else 0))
    return out


def _axes_05(t: dict) -> list[AxisSpec]:
    out = []
    for a in t["axes"]:
        typ = a.get("type")
        aid = a.get("id") or {"batch": "b", "channel": "c", "index": "i", "time": "t"}.get(typ, typ)
        size = a.get("size")
        if typ == "channel":
            names = a.get("channel_names")
            size = len(names) if names else size
        if typ == "batch":
            size = a.get("size")
        out.append(AxisSpec(id=str(aid)[0] if typ in ("batch", "channel", "index", "time") else str(aid), type=typ,
                            size=size, halo=int(a.get("halo", 0) or 0), scale=float(a.get("scale", 1.0) or 1.0),
                            channel_names=a.get("channel_names")))
    return out


def tensors(rdf: dict, which: str) -> list[TensorSpec]:
    v05 = str(rdf.get("format_version", "0.4")).startswith("0.5")
    specs = []
    for i, t in enumerate(rdf.get(which, [])):
        tid = t.get("id") or t.get("name") or f"{which[:-1]}{i}"
        axes = _axes_05(t) if v05 else _axes_04(t, which == "outputs")
        pre = t.get("preprocessing") or []
        post = t.get("postprocessing") or []
        test = _src(t.get("test_tensor"))
        if test is None and rdf.get("test_inputs" if which == "inputs" else "test_outputs"):
            lst = rdf["test_inputs" if which == "inputs" else "test_outputs"]
            test = _src(lst[i]) if i < len(lst) else None
        dt = t.get("data_type") or (t.get("data", {}) or {}).get("type", "float32")
        specs.append(TensorSpec(id=str(tid), axes=axes, data_type=dt, preprocessing=pre, postprocessing=post,
                                test_tensor=test, sample_tensor=_src(t.get("sample_tensor"))))
    return specs


def load_rdf(source) -> tuple[dict, Path | None]:
    """source: path to rdf.yaml / a package directory / a dict -> (rdf, package_root)."""
    if isinstance(source, dict):
        return source, None
    p = Path(source)
    if p.is_dir():
        for name in ("rdf.yaml", "bioimageio.yaml"):
            if (p / name).exists():
                p = p / name
                break
    rdf = yaml.safe_load(p.read_text())
    return rdf, p.parent


def weights_entries(rdf: dict) -> dict:
    w = rdf.get("weights") or {}
    return {k: v for k, v in w.items() if v}


def sha256_file(path: Path) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def validate_format(rdf: dict, known_files: dict | None = None, root: Path | None = None) -> dict:
    """Format validation (no I/O beyond ``root`` files when given).  Returns
    ``{"status": "valid-format" | "invalid", "errors": [...], "warnings": [...]}``."""
    errors, warnings = [], []
    if not isinstance(rdf, dict):
        return {"status": "invalid", "errors": ["RDF must be a mapping"], "warnings": []}
    typ = rdf.get("type")
    fv = str(rdf.get("format_version", ""))
    if not fv:
        errors.append("format_version: missing")
    elif not (fv.startswith("0.4") or fv.startswith("0.5") or fv.startswith("0.2") or fv.startswith("0.3")):
        errors.append(f"format_version: unsupported {fv}")
    if typ == "model":
        for f in REQUIRED_MODEL_FIELDS:
            if f not in rdf or rdf[f] in (None, [], {}):
                errors.append(f"{f}: field required")
        w = weights_entries(rdf)
        for k, v in w.items():
            if k not in WEIGHT_FORMATS:
                errors.append(f"weights.{k}: unknown weights format")
            elif not _src(v):
                errors.append(f"weights.{k}.source: field required")
            if k == "pytorch_state_dict" and isinstance(v, dict) and not v.get("architecture"):
                errors.append("weights.pytorch_state_dict.architecture: field required")
        try:
            ins, outs = tensors(rdf, "inputs"), tensors(rdf, "outputs")
            for t in ins + outs:
                if not t.axes:
                    errors.append(f"{t.id}.axes: empty")
                ids = t.axis_ids
                if len(set(ids)) != len(ids):
                    errors.append(f"{t.id}.axes: duplicate axis ids {ids}")
            names = [t.id for t in ins + outs]
            if len(set(names)) != len(names):
                errors.append(f"tensor ids not unique: {names}")
        except Exception as e:  # noqa: BLE001
            errors.append(f"inputs/outputs: {type(e).__name__}: {e}")
        if not (rdf.get("test_inputs") or any(t.get("test_tensor") for t in rdf.get("inputs", []) if isinstance(t, dict))):
            warnings.append("no test tensors declared")
    elif typ is None:
        errors.append("type: field required")
    for k in ("name", "description"):
        if not rdf.get(k):
            (errors if k == "name" else warnings).append(f"{k}: missing")
    kf = known_files or {}
    if root is not None or kf:
        for k, v in weights_entries(rdf).items():
            s = _src(v)
            if not s or "://" in str(s):
                continue
            if kf:
                if s not in kf:
                    errors.append(f"weights.{k}.source: file {s} not in known_files")
                elif isinstance(v, dict) and v.get("sha256") and kf[s] not in (None, v["sha256"]):
                    errors.append(f"weights.{k}.sha256 mismatch")
            elif root is not None and not (root / s).exists():
                errors.append(f"weights.{k}.source: {s} not found")
    return {"status": "valid-format" if not errors else "invalid", "errors": errors, "warnings": warnings}


def format_summary(summary: dict) -> str:
    lines = [f"status: {summary['status']}"]
    lines += [f"error: {e}" for e in summary.get("errors", [])]
    lines += [f"warning: {w}" for w in summary.get("warnings", [])]
    return "\n".join(lines)
