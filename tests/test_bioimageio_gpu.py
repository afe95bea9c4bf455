"""Model runner on the GPU: graph-pass numerics (fused NHWC MFMA convs, bf16 channels-last) vs the
fp32 PyTorch model, package test, tiled inference, post-ReLU conv epilogue."""
import numpy as np
import pytest
import torch

from bioengine_worker_amd.bioimageio.package import load_module, write_unet2d_package


@pytest.fixture(scope="module")
def pkg(tmp_path_factory):
    return write_unet2d_package(tmp_path_factory.mktemp("zoo") / "gpu-unet", "gpu-unet", test_shape=(1, 1, 256, 256),
                                torchscript=False)


@pytest.mark.gpu
def test_post_relu_epilogue(gpu):
    from bioengine_worker_amd.ops.conv import PackedConv, fused_conv2d, fused_conv2d_ref

    x = torch.randn(2, 40, 72, 32).bfloat16()
    pc = PackedConv.from_weight(torch.randn(64, 32, 3, 3) / 17, torch.randn(64) * 0.1)
    res = torch.randn(2, 40, 72, 64).bfloat16()
    ref = fused_conv2d_ref(x, pc, residual=res, post_relu=True).float()
    out = fused_conv2d(x.to(gpu), pc.to(gpu), residual=res.to(gpu), post_relu=True).float().cpu()
    assert (out - ref).abs().max() < 3e-2 and (out >= 0).all()


@pytest.mark.gpu
def test_graph_pass_unet_matches_fp32(gpu, pkg):
    from bioengine_worker_amd.bioimageio.convert import optimize_for_mi355x

    mod = load_module(pkg / "model.py", "gpu_unet_src")
    net = mod.UNet2d(in_channels=1, out_channels=2, features=[32, 64, 128, 256]).eval()
    net.load_state_dict(torch.load(pkg / "weights.pt", weights_only=True))
    x = torch.randn(2, 1, 256, 256)
    with torch.no_grad():
        ref = net.to(gpu)(x.to(gpu)).float().cpu()
    net2, stats = optimize_for_mi355x(net, gpu)
    assert stats["convs"] == 15 and stats["relu_fused"] == 14
    with torch.no_grad():
        y = net2(x.to(gpu).bfloat16().contiguous(memory_format=torch.channels_last)).float().cpu()
    assert (y - ref).abs().max() < 0.05, (y - ref).abs().max()


@pytest.mark.gpu
def test_package_test_on_gpu(gpu, pkg):
    from bioengine_worker_amd.bioimageio.testing import test_model

    rep = test_model(pkg)
    assert rep["status"] == "passed", rep
    assert rep["details"][2]["optimized"] is True


@pytest.mark.gpu
def test_blocked_inference_gpu(gpu, pkg):
    from bioengine_worker_amd.bioimageio.runner import PredictionPipeline

    pipe = PredictionPipeline(pkg, device=gpu)
    x = np.random.default_rng(0).normal(300, 50, (1, 1, 700, 530)).astype(np.float32)
    whole = pipe.predict(x)["probabilities"]
    tiled = pipe.predict(x, blocksize=8)["probabilities"]
    assert whole.shape == tiled.shape == (1, 2, 700, 530)
    assert np.corrcoef(whole.ravel(), tiled.ravel())[0, 1] > 0.98


@pytest.mark.gpu
@pytest.mark.parametrize("norm,down", [("group", "conv"), ("instance", "pool")])
def test_graph_pass_norm_and_strided_unets(gpu, tmp_path, norm, down):
    """GroupNorm / InstanceNorm run in the next conv's prologue, 2x2 stride-2 convs as
    space-to-depth + 1x1, transposed convs as 1x1 + depth-to-space: fp32-oracle numerics and the
    package test through the optimised pipeline."""
    import yaml

    from bioengine_worker_amd.bioimageio.convert import optimize_for_mi355x
    from bioengine_worker_amd.bioimageio.testing import test_model

    p = write_unet2d_package(tmp_path / norm, f"gpu-{norm}", test_shape=(1, 1, 128, 128), torchscript=False,
                             norm=norm, down=down, features=(32, 64, 128, 256))
    mod = load_module(p / "model.py", f"gpu_{norm}_src")
    kw = yaml.safe_load((p / "rdf.yaml").read_text())["weights"]["pytorch_state_dict"]["architecture"]["kwargs"]
    net = mod.UNet2d(**kw).eval()
    net.load_state_dict(torch.load(p / "weights.pt", weights_only=True))
    x = torch.randn(2, 1, 128, 160)
    with torch.no_grad():
        ref = net.to(gpu)(x.to(gpu)).float().cpu()
    net2, stats = optimize_for_mi355x(net, gpu)
    assert stats["norm_fused"] == 7 and stats["conv_transpose"] == 3
    assert stats["strided"] == (3 if down == "conv" else 0)
    with torch.no_grad():
        y = net2(x.to(gpu).bfloat16().contiguous(memory_format=torch.channels_last)).float().cpu()
    assert (y - ref).abs().max() < 0.05, (y - ref).abs().max()
    rep = test_model(p)
    assert rep["status"] == "passed", rep
    assert rep["details"][2]["optimized"] is True


@pytest.mark.gpu
def test_torchscript_only_package_is_optimized(gpu, tmp_path):
    from bioengine_worker_amd.bioimageio import ts_convert
    from bioengine_worker_amd.bioimageio.runner import PredictionPipeline
    from bioengine_worker_amd.bioimageio.testing import test_model

    p = write_unet2d_package(tmp_path / "ts", "gpu-ts-only", test_shape=(1, 1, 128, 128), state_dict=False)
    pipe = PredictionPipeline(p, device=gpu)
    assert pipe.weights_format == "torchscript" and pipe.optimized
    assert pipe.convert_stats["convs"] == 15 and pipe.convert_stats["relu_fused"] == 14
    before = ts_convert.COUNTS["hip"]
    x = np.load(p / "test_input.npy")
    y = pipe.predict(x)["probabilities"]
    assert ts_convert.COUNTS["hip"] - before >= 15  # the convs ran on the HIP kernel
    assert np.abs(y - np.load(p / "test_output.npy")).max() < 0.05
    rep = test_model(p)
    assert rep["status"] == "passed", rep
    assert rep["details"][2]["optimized"] is True
