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
