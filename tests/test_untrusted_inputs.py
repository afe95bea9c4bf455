"""Untrusted-input hardening: ONNX external-data locations, metadata record paths, pip requirement
strings (ADVICE r02 findings)."""
from pathlib import Path

import numpy as np
import pytest

from bioengine_worker_amd.apps import requirements as rq
from bioengine_worker_amd.bioimageio import onnx_proto as P
from bioengine_worker_amd.cellpose import datasets as ds


def _ext_tensor(location, offset=0, length=None):
    ext = {"location": location, "offset": str(offset)}
    if length is not None:
        ext["length"] = str(length)
    return P.Tensor(name="w", dims=[4], data_type=P.FLOAT, external=ext)


def test_onnx_external_data_inside_model_dir(tmp_path):
    (tmp_path / "weights.bin").write_bytes(np.arange(8, dtype="<f4").tobytes())
    t = P.tensor_to_torch(_ext_tensor("weights.bin", offset=16, length=16), str(tmp_path))
    assert t.tolist() == [4.0, 5.0, 6.0, 7.0]
    (tmp_path / "sub").mkdir()
    (tmp_path / "sub" / "w.bin").write_bytes(np.ones(4, dtype="<f4").tobytes())
    assert P.tensor_to_torch(_ext_tensor("sub/w.bin"), str(tmp_path)).tolist() == [1.0] * 4


@pytest.mark.parametrize("loc", ["/etc/passwd", "../secret.bin", "sub/../../secret.bin", "..", "", "C:/x.bin"])
def test_onnx_external_data_traversal_rejected(tmp_path, loc):
    model_dir = tmp_path / "model"
    model_dir.mkdir()
    (tmp_path / "secret.bin").write_bytes(b"\x00" * 16)
    with pytest.raises(ValueError):
        P.tensor_to_torch(_ext_tensor(loc), str(model_dir))


def test_onnx_external_data_symlink_escape_and_bounds(tmp_path):
    model_dir = tmp_path / "model"
    model_dir.mkdir()
    (tmp_path / "secret.bin").write_bytes(b"\x00" * 16)
    (model_dir / "link.bin").symlink_to(tmp_path / "secret.bin")
    with pytest.raises(ValueError):
        P.tensor_to_torch(_ext_tensor("link.bin"), str(model_dir))
    (model_dir / "w.bin").write_bytes(b"\x00" * 16)
    with pytest.raises(ValueError):
        P.tensor_to_torch(_ext_tensor("w.bin", offset=8, length=16), str(model_dir))
    with pytest.raises(ValueError):
        P.tensor_to_torch(_ext_tensor("w.bin", offset=32), str(model_dir))


def test_metadata_record_paths_cannot_escape(tmp_path):
    parent = Path("data/meta")
    assert ds._record_path("img/a.tif", parent) == Path("img/a.tif")
    assert ds._record_path("a.tif", parent) == Path("data/meta/a.tif")
    assert ds._record_path("/img/./b.tif", parent) == Path("img/b.tif")
    assert ds._record_path("../../sessions/other/data/x.tif", parent) is None
    assert ds._record_path("img/../../../x.tif", parent) is None
    with pytest.raises(ValueError):
        ds.local_path(tmp_path, "../outside.tif")
    (tmp_path / "cache").mkdir()
    (tmp_path / "cache" / "lnk").symlink_to(tmp_path)
    with pytest.raises(ValueError):
        ds.local_path(tmp_path / "cache", "lnk/escape.tif")
    assert ds.local_path(tmp_path, "a/b.tif") == tmp_path / "a" / "b.tif"


@pytest.mark.parametrize("bad", ["--target=/tmp/x", "-e /some/path", "--find-links=http://x", "pkg @ https://h/x.whl",
                                 "pkg @ file:///tmp/pkg-1.0.tar.gz", "not a requirement!!"])
def test_invalid_requirements_never_reach_pip(tmp_path, monkeypatch, bad):
    calls = []
    monkeypatch.setattr(rq.subprocess, "run", lambda *a, **k: calls.append(a) or None)
    wh = tmp_path / "wheels"
    wh.mkdir()
    with pytest.raises(rq.MissingRequirementsError):
        rq.ensure([bad], tmp_path / "site", wheel_dirs=[str(wh)])
    assert calls == []


def test_valid_requirements_passed_after_separator(tmp_path, monkeypatch):
    seen = {}

    class R:
        returncode = 1
        stderr = "boom"
        stdout = ""

    def fake_run(cmd, **kw):
        seen["cmd"] = cmd
        return R()

    monkeypatch.setattr(rq.subprocess, "run", fake_run)
    wh = tmp_path / "wheels"
    wh.mkdir()
    with pytest.raises(rq.MissingRequirementsError):
        rq.ensure(["definitely-not-installed-pkg==1.0"], tmp_path / "site", wheel_dirs=[str(wh)])
    cmd = seen["cmd"]
    i = cmd.index("--")
    assert cmd[i + 1:] == ["definitely-not-installed-pkg==1.0"]
