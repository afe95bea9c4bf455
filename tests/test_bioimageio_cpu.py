"""bioimage.io support on CPU: package writer, RDF validation, prediction pipeline (whole + blocked),
pre/post-processing, graph pass structure, model cache, test_model."""
import asyncio

import numpy as np
import pytest
import torch

from bioengine_worker_amd.bioimageio import processing
from bioengine_worker_amd.bioimageio.convert import HipConv2d, optimize_for_mi355x
from bioengine_worker_amd.bioimageio.package import load_module, write_unet2d_package
from bioengine_worker_amd.bioimageio.runner import PredictionPipeline
from bioengine_worker_amd.bioimageio.spec import load_rdf, tensors, validate_format
from bioengine_worker_amd.bioimageio.testing import test_model as run_model_test
from bioengine_worker_amd.bioimageio.zoo import ModelCache, search_local


@pytest.fixture(scope="module")
def pkg(tmp_path_factory):
    return write_unet2d_package(tmp_path_factory.mktemp("zoo") / "demo-unet2d", features=(8, 16, 32),
                                test_shape=(1, 1, 96, 128))


def test_rdf_validates_and_parses(pkg):
    rdf, root = load_rdf(pkg)
    assert validate_format(rdf, root=root)["status"] == "valid-format"
    bad = dict(rdf)
    bad.pop("weights")
    assert validate_format(bad)["status"] == "invalid"
    ins = tensors(rdf, "inputs")
    assert ins[0].axis_ids == ["b", "c", "y", "x"] and ins[0].axes[2].size == {"min": 64, "step": 16}
    outs = tensors(rdf, "outputs")
    assert outs[0].axes[2].halo == 16


def test_rdf_04_axes():
    rdf = {"format_version": "0.4.10", "type": "model", "name": "m", "inputs": [
        {"name": "in", "axes": "bcyx", "shape": {"min": [1, 1, 32, 32], "step": [0, 0, 16, 16]}, "data_type": "float32"}],
        "outputs": [{"name": "out", "axes": "bcyx", "halo": [0, 0, 8, 8],
                     "shape": {"reference_tensor": "in", "scale": [1, 1, 1, 1], "offset": [0, 0, 0, 0]}}],
        "weights": {"torchscript": {"source": "w.pt"}}, "test_inputs": ["a.npy"], "test_outputs": ["b.npy"]}
    i, o = tensors(rdf, "inputs")[0], tensors(rdf, "outputs")[0]
    assert i.axis_ids == list("bcyx") and i.axes[3].size == {"min": 32, "step": 16} and o.axes[2].halo == 8
    assert validate_format(rdf)["status"] == "valid-format"


def test_pipeline_reproduces_test_output_cpu(pkg):
    pipe = PredictionPipeline(pkg, device="cpu", optimize=False)
    x = np.load(pkg / "test_input.npy")
    y = pipe.predict(x)["probabilities"]
    ref = np.load(pkg / "test_output.npy")
    assert y.shape == ref.shape and np.abs(y - ref).max() < 1e-4
    # odd sizes are padded to min + k*step and cropped back
    y2 = pipe.predict(x[:, :, :90, :101])["probabilities"]
    assert y2.shape == (1, 2, 90, 101)
    # blocked (tiled) inference with halo: close to whole-image inference
    yb = pipe.predict(x, blocksize=0)["probabilities"]
    assert yb.shape == ref.shape and np.corrcoef(yb.ravel(), ref.ravel())[0, 1] > 0.98


def test_torchscript_weights(pkg):
    pipe = PredictionPipeline(pkg, device="cpu", weights_format="torchscript")
    y = pipe.predict(np.load(pkg / "test_input.npy"))["probabilities"]
    assert np.abs(y - np.load(pkg / "test_output.npy")).max() < 1e-4


def test_processing_ops():
    x = torch.arange(24.0).reshape(1, 2, 3, 4)
    ids = ["b", "c", "y", "x"]
    y = processing.apply_op(x, {"id": "scale_range", "kwargs": {"axes": ["y", "x"], "min_percentile": 0,
                                                                 "max_percentile": 100}}, ids)
    assert torch.allclose(y.amin(dim=(2, 3)), torch.zeros(1, 2)) and torch.allclose(y.amax(dim=(2, 3)), torch.ones(1, 2), atol=1e-5)
    z = processing.apply_op(x, {"name": "zero_mean_unit_variance", "kwargs": {"axes": "xy"}}, ids)
    assert torch.allclose(z.mean(dim=(2, 3)), torch.zeros(1, 2), atol=1e-5)
    f = processing.apply_op(x, {"id": "fixed_zero_mean_unit_variance", "kwargs": {"mean": [1.0, 2.0], "std": [2.0, 4.0], "axis": "c"}}, ids)
    assert torch.allclose(f[0, 1], (x[0, 1] - 2) / (4 + 1e-6))
    b = processing.apply_op(torch.rand(1, 1, 4, 4), {"id": "binarize", "kwargs": {"threshold": 0.5}}, ids)
    assert set(b.unique().tolist()) <= {0.0, 1.0}
    s = processing.apply_op(x, {"id": "scale_linear", "kwargs": {"gain": 2.0, "offset": 1.0}}, ids)
    assert torch.allclose(s, 2 * x + 1)


def test_graph_pass_structure(pkg):
    mod = load_module(pkg / "model.py", "t_graphpass")
    net = mod.UNet2d(in_channels=1, out_channels=2, features=[8, 16, 32]).eval()
    net.load_state_dict(torch.load(pkg / "weights.pt", weights_only=True))
    x = torch.randn(1, 1, 64, 64)
    with torch.no_grad():
        ref = net(x)
    net2, stats = optimize_for_mi355x(net)
    assert stats["convs"] == 11 and stats["bn_folded"] == 10 and stats["relu_fused"] == 10
    assert sum(isinstance(m, HipConv2d) for m in net2.modules()) == 11
    with torch.no_grad():
        y = net2(x.bfloat16()).float()
    assert (y - ref).abs().max() < 0.05


def test_model_cache_and_search(pkg, tmp_path, monkeypatch):
    monkeypatch.setenv("BIOENGINE_MODEL_ZOO", str(pkg.parent))
    assert search_local(["unet"])[0]["model_id"] == "demo-unet2d"
    assert search_local(["nonexistent-keyword"]) == []
    cache = ModelCache(tmp_path / "cache", cache_size_in_gb=1.0)

    async def go():
        lease = await cache.get_model_package("demo-unet2d")
        async with lease:
            assert (lease.source / "rdf.yaml").exists() and cache.cached_models()[0]["in_use"]
        assert not cache.cached_models()[0]["in_use"]
        with pytest.raises(ValueError):
            await cache.get_model_package("does-not-exist")
    asyncio.run(go())


def test_test_model_report(pkg):
    rep = run_model_test(pkg, device="cpu")
    assert rep["status"] == "passed", rep
    assert rep["details"][1]["name"].startswith("Reproduce")


def _hang_downloader(cache_dir, ready_path):
    """Child process: claims the download of 'remote-model', then hangs inside the fetch."""
    import asyncio as aio
    from pathlib import Path as P

    from bioengine_worker_amd.bioimageio.zoo import ModelCache as MC

    async def fetch(model_id, dest, stage):
        P(ready_path).write_text("claimed")
        await aio.sleep(3600)

    aio.run(MC(cache_dir, replica_id="dead", fetch_remote=fetch).get_model_package("remote-model"))


def test_model_cache_recovers_from_dead_downloader_and_stale_leases(tmp_path, monkeypatch):
    """A replica killed mid-download leaves its marker behind: the next request reclaims it at once
    instead of waiting out the timeout; a dead process's in-use lease no longer blocks eviction
    (reference entry_deployment.py:384-411, 833-837)."""
    import asyncio
    import json
    import multiprocessing as mp
    import os
    import signal
    import time

    from bioengine_worker_amd.bioimageio import zoo

    monkeypatch.delenv("BIOENGINE_MODEL_ZOO", raising=False)
    cache_dir = tmp_path / "cache"
    ready = tmp_path / "ready"
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_hang_downloader, args=(str(cache_dir), str(ready)))
    p.start()
    try:
        for _ in range(600):
            if ready.exists():
                break
            time.sleep(0.1)
        assert ready.exists(), "child never claimed the download"
        assert (cache_dir / ".remote-model.downloading").is_dir()
    finally:
        os.kill(p.pid, signal.SIGKILL)
        p.join(10)

    async def fetch(model_id, dest, stage):
        (dest / "rdf.yaml").write_text("id: remote-model\n")
        (dest / "weights.bin").write_bytes(b"\0" * 1024)
        return 123.0

    cache = zoo.ModelCache(cache_dir, cache_size_in_gb=1.0, replica_id="live", fetch_remote=fetch)
    t0 = time.time()
    lease = asyncio.run(cache.get_model_package("remote-model"))
    assert time.time() - t0 < 5.0
    assert lease.rdf_path.exists() and not (cache_dir / ".remote-model.downloading").exists()

    # a lease from a dead pid on this host, and one older than the max age: neither pins the package
    d = lease.source
    (d / ".in_use.999999999.x").write_text(json.dumps({"host": zoo._HOST, "pid": 999999999, "t": time.time()}))
    old = d / ".in_use.1.y"
    old.write_text(json.dumps({"host": "elsewhere", "pid": 1, "t": time.time() - 2 * zoo.LEASE_MAX_AGE_S}))
    assert not any(m["in_use"] for m in cache.cached_models())

    async def held():
        async with lease:
            return [m["in_use"] for m in cache.cached_models()]
    assert any(asyncio.run(held()))
    cache.cache_size_bytes = 10  # force eviction of everything not in use
    asyncio.run(cache.ensure_space(0))
    assert not d.exists()


def test_chunked_mean_std_matches_direct():
    """processing._mean_std: chunk moments combined exactly (the EM line's per-tile normalisation)."""
    import torch

    from bioengine_worker_amd.bioimageio.processing import _mean_std

    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, 2, 256, 384, generator=g) * 7 + 3
    for dims in ([2, 3], [1, 2, 3], [3]):
        m, s = _mean_std(x, dims)
        assert torch.allclose(m, x.mean(dim=dims, keepdim=True), atol=1e-5)
        assert torch.allclose(s, x.std(dim=dims, keepdim=True, unbiased=False), rtol=1e-5)
