"""``test_model``: reproduce a package's test outputs from its test inputs (bioimageio.core
``test_model`` semantics as used by the reference model-runner ``test``, runtime_deployment.py:101-156).

The reproducibility check runs the unmodified fp32 network (the package's own numerics); the
MI355X-optimised bf16 path is run as well and its deviation is reported as a separate check, so a
report says both "the package is correct" and "what the fast path costs in accuracy"."""
from __future__ import annotations

import platform
import time
from pathlib import Path

import numpy as np
import torch

from .report import env_rows
from .runner import PredictionPipeline
from .spec import format_summary, load_rdf, tensors, validate_format


def _tol(rdf: dict) -> tuple[float, float, float]:
    t = (((rdf.get("config") or {}).get("bioimageio") or {}).get("reproducibility_tolerance") or [{}])
    t = t[0] if isinstance(t, list) and t else {}
    return float(t.get("relative_tolerance", 1e-3)), float(t.get("absolute_tolerance", 1e-4)), \
        float(t.get("mismatched_elements_per_million", 100))


def _compare(got: np.ndarray, exp: np.ndarray, rtol: float, atol: float, mepm: float) -> tuple[bool, str]:
    if got.shape != exp.shape:
        return False, f"shape {got.shape} != expected {exp.shape}"
    bad = np.abs(got.astype(np.float64) - exp) > atol + rtol * np.abs(exp)
    n_bad = int(bad.sum())
    allowed = mepm * exp.size / 1e6
    ok = n_bad <= allowed
    return ok, f"{n_bad} mismatched elements (allowed {allowed:.1f}), max abs diff {float(np.abs(got - exp).max()):.3g}"


def test_model(source, device=None, weights_format: str | None = None) -> dict:
    rdf, root = load_rdf(source)
    t0 = time.time()
    details = []
    v = validate_format(rdf, root=root)
    details.append({"name": "bioimageio.spec format validation", "status": "passed" if v["status"] == "valid-format" else "failed",
                    "errors": v["errors"], "warnings": v["warnings"]})
    ins, outs = tensors(rdf, "inputs"), tensors(rdf, "outputs")
    if root is None or any(t.test_tensor is None for t in ins + outs):
        details.append({"name": "Reproduce test outputs from test inputs", "status": "failed",
                        "errors": ["package has no test tensors"]})
    else:
        inputs = {t.id: np.load(root / t.test_tensor) for t in ins}
        expected = {t.id: np.load(root / t.test_tensor) for t in outs}
        rtol, atol, mepm = _tol(rdf)
        for label, optimize in (("Reproduce test outputs from test inputs", False),
                                ("MI355X bf16 fused path vs test outputs", True)):
            try:
                pipe = PredictionPipeline(root, device=device, weights_format=weights_format, optimize=optimize)
                got = pipe.predict(inputs)
                errs, infos = [], []
                for t in outs:
                    if optimize:  # bf16 activations: report, judge against a bf16-appropriate tolerance
                        ok, msg = _compare(got[t.id], expected[t.id], 5e-2, 2e-2, 5e3)
                    else:
                        ok, msg = _compare(got[t.id], expected[t.id], rtol, atol, mepm)
                    (infos if ok else errs).append(f"{t.id}: {msg}")
                details.append({"name": label, "status": "passed" if not errs else "failed", "errors": errs,
                                "info": infos, "weights_format": pipe.weights_format, "optimized": pipe.optimized,
                                "convert_stats": pipe.convert_stats})
            except Exception as e:  # noqa: BLE001
                details.append({"name": label, "status": "failed", "errors": [f"{type(e).__name__}: {e}"]})
            if not torch.cuda.is_available():
                break  # the optimised path is the GPU path
    status = "passed" if all(d["status"] == "passed" for d in details) else "failed"
    return {"name": "bioimageio format validation and model test", "status": status, "type": rdf.get("type"),
            "id": rdf.get("id"), "format_version": rdf.get("format_version"), "details": details,
            "summary": format_summary(v), "duration_s": round(time.time() - t0, 3),
            "env": env_rows({"torch": torch.__version__, "python": platform.python_version(),
                             "device": torch.cuda.get_device_name(0) if torch.cuda.is_available() else "cpu"})}
