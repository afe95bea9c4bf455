"""Regression tests for the round-3 advisor findings.

* ``batchable()`` refuses a fixed batch size, and ``predict_many`` falls back to per-request
  forwards when a batched forward fails (a graph with a static batch dim);
* a requirement that the worker already has at a different version is reported as shadowed, so
  the app never runs in-process on the worker's copy;
* the resume state is written atomically;
* fibsem ``tiled3d`` only resolves installed 3-D models (no path built from the caller's id, no
  random-weights package written).
"""
from __future__ import annotations

import importlib.util
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

from bioengine_worker_amd.bioimageio.runner import PredictionPipeline
from bioengine_worker_amd.bioimageio.spec import AxisSpec, TensorSpec

ROOT = Path(__file__).resolve().parents[1]


def _pipe(batch_size, forward):
    p = PredictionPipeline.__new__(PredictionPipeline)
    p.blocksize = None
    axes = [AxisSpec("b", "batch", batch_size), AxisSpec("c", "channel", 1), AxisSpec("y", "space", None),
            AxisSpec("x", "space", None)]
    p.inputs = [TensorSpec("input", axes)]
    p.outputs = [TensorSpec("output", [AxisSpec(a.id, a.type, None) for a in axes])]
    p.device = torch.device("cpu")
    p._forward = forward
    p._valid_len = lambda L, size: L
    return p


def test_batchable_refuses_fixed_batch():
    assert _pipe(None, None).batchable()
    assert not _pipe(1, None).batchable()
    assert not _pipe({"min": 1, "step": 0}, None).batchable()
    assert _pipe({"min": 1, "step": 1}, None).batchable()


def test_predict_many_falls_back_on_static_batch_graph():
    calls = []

    def forward(xs):
        calls.append(xs[0].shape[0])
        if xs[0].shape[0] != 1:
            raise RuntimeError("static batch dim 1")
        return [xs[0] * 2]

    p = _pipe(None, forward)
    samples = [np.full((1, 1, 8, 8), float(i), np.float32) for i in range(3)]
    out = p.predict_many(samples)
    assert calls[0] == 3 and calls[1:] == [1, 1, 1]
    for i, o in enumerate(out):
        np.testing.assert_allclose(o["output"], np.full((1, 1, 8, 8), 2.0 * i))


def test_shadowed_requirement_detected():
    from bioengine_worker_amd.apps.requirements import shadowed

    np_ver = np.__version__
    assert shadowed([f"numpy=={np_ver}"]) == []
    bad = shadowed(["numpy==1.0.0"])
    assert bad and bad[0][0] == "numpy==1.0.0"
    assert shadowed(["surely-not-a-package==1.0"]) == []


def test_trainer_state_saved_atomically(tmp_path, monkeypatch):
    from bioengine_worker_amd.train import session

    target = tmp_path / "trainer_state.pt"
    target.write_bytes(b"old")
    real_save = torch.save

    def dying_save(obj, f):
        Path(f).write_bytes(b"trunc")
        raise KeyboardInterrupt  # the writer dies mid-save

    monkeypatch.setattr(session.torch, "save", dying_save)
    with pytest.raises(KeyboardInterrupt):
        session._save_atomic({"a": 1}, target)
    assert target.read_bytes() == b"old"  # never replaced by a partial file
    monkeypatch.setattr(session.torch, "save", real_save)
    session._save_atomic({"a": torch.ones(2)}, target)
    assert torch.load(target, weights_only=True)["a"].sum() == 2


def test_fibsem_model3d_requires_installed_model(tmp_path, monkeypatch):
    from bioengine_worker_amd import compat

    compat.install()
    monkeypatch.setenv("HOME", str(tmp_path))
    path = ROOT / "apps" / "fibsem-mito-analysis" / "analysis_deployment.py"
    sys.path.insert(0, str(path.parent))
    try:
        spec = importlib.util.spec_from_file_location("fibsem_analysis_advice", path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        sys.path.remove(str(path.parent))
    inner = mod.MitoAnalysisDeployment.func_or_class
    obj = inner.__new__(inner)
    for mid in ("mito-unet3d", "../../escape"):
        with pytest.raises(FileNotFoundError):
            obj._model3d_root(mid)
    assert not (tmp_path / "model_zoo").exists()
    assert not (tmp_path.parent / "escape").exists()
