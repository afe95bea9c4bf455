"""3-D convolution path: depth-tap decomposition onto the fused NHWC MFMA conv kernel (ops/conv3d.py),
the 3-D graph pass (Conv3d + BatchNorm3d + ReLU -> HipConv3d), and a 3-D BioImage.IO U-Net package
through the model runner (whole-volume and tiled) — GPU results against plain PyTorch fp32."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from bioengine_worker_amd.bioimageio.package import load_module, write_unet3d_package
from bioengine_worker_amd.ops.conv3d import PackedConv3d, conv3d_ref, fused_conv3d


@pytest.fixture(scope="module")
def pkg3d(tmp_path_factory):
    return write_unet3d_package(tmp_path_factory.mktemp("zoo3d") / "unet3d", "unet3d", test_shape=(1, 1, 24, 48, 48))


def _net(pkg):
    mod = load_module(pkg / "model.py", "unet3d_src_test")
    net = mod.UNet3d(in_channels=1, out_channels=1, features=[16, 32, 64, 128]).eval()
    net.load_state_dict(torch.load(pkg / "weights.pt", weights_only=True))
    return net


def test_conv3d_ref_matches_torch():
    x = torch.randn(2, 5, 9, 11, 8)  # NDHWC
    w, b = torch.randn(12, 8, 3, 3, 3), torch.randn(12)
    pc = PackedConv3d(w, b)
    y = conv3d_ref(x, pc, post_relu=True)
    ref = torch.relu(F.conv3d(x.permute(0, 4, 1, 2, 3), w, b, padding=1)).permute(0, 2, 3, 4, 1)
    torch.testing.assert_close(y, ref, rtol=1e-4, atol=1e-4)
    assert len(pc.taps) == 3 and pc.taps[1].bias is not None and pc.taps[0].bias is None


def test_graph_pass_3d_structure_and_cpu_numerics(pkg3d):
    from bioengine_worker_amd.bioimageio.convert import HipConv3d, optimize_for_mi355x

    net = _net(pkg3d)
    x = torch.randn(1, 1, 16, 32, 32)
    with torch.no_grad():
        ref = net(x)
    net2, stats = optimize_for_mi355x(net)
    # 7 conv blocks x 2 Conv3d(3x3x3) with BN + ReLU, the 1-channel 1x1x1 head (fp32 NCDHW epilogue),
    # 3 ConvTranspose3d(2, 2) and the MaxPool3d(2): no library convolution or pooling is left
    assert stats["convs"] == 15 and stats["bn_folded"] == 14 and stats["relu_fused"] == 14
    assert stats["skipped"] == 0 and stats["conv_transpose"] == 3 and stats["pool3d"] == 1
    assert sum(isinstance(m, HipConv3d) for m in net2.modules()) == 15
    lib = (torch.nn.Conv3d, torch.nn.ConvTranspose3d, torch.nn.MaxPool3d)
    assert not [m for m in net2.modules() if type(m) in lib]
    with torch.no_grad():
        y = net2(x.bfloat16()).float()
    assert (y - ref).abs().max() < 0.05


def test_unet3d_package_cpu(pkg3d):
    from bioengine_worker_amd.bioimageio.testing import test_model

    rep = test_model(pkg3d, device="cpu")
    assert rep["status"] == "passed", rep


@pytest.mark.gpu
@pytest.mark.parametrize("N,D,H,W,Cin,Cout,ks", [(1, 8, 40, 72, 32, 64, 3), (2, 5, 33, 20, 16, 32, 3),
                                                 (1, 1, 16, 16, 64, 64, 3), (1, 6, 24, 24, 32, 16, 1),
                                                 (1, 7, 20, 36, 1, 16, 3)])
@pytest.mark.parametrize("post_relu", [False, True])
def test_fused_conv3d_matches_fp32(gpu, N, D, H, W, Cin, Cout, ks, post_relu):
    g = torch.Generator().manual_seed(N * D + Cin)
    x = torch.randn(N, D, H, W, Cin, generator=g).bfloat16()
    w = torch.randn(Cout, Cin, ks, ks, ks, generator=g) / (Cin * ks ** 3) ** 0.5
    b = torch.randn(Cout, generator=g) * 0.1
    pc = PackedConv3d(w, b)
    ref = conv3d_ref(x.float(), pc, post_relu)  # fp32 oracle on bf16-valued input
    xp = F.pad(x, (0, pc.cin_pad - Cin)).contiguous().to(gpu)
    y = fused_conv3d(xp, pc.to(gpu), post_relu).float().cpu()
    assert y.shape == (N, D, H, W, Cout)
    err = (y - ref).abs().max().item()
    assert err < 3e-2 * max(1.0, ref.abs().max().item()), err
    if post_relu:
        assert (y >= 0).all()


@pytest.mark.gpu
def test_graph_pass_unet3d_matches_fp32(gpu, pkg3d):
    from bioengine_worker_amd.bioimageio.convert import optimize_for_mi355x

    net = _net(pkg3d)
    x = torch.randn(1, 1, 24, 64, 64)
    with torch.no_grad():
        ref = net.to(gpu)(x.to(gpu)).float().cpu()
    net2, stats = optimize_for_mi355x(net, gpu)
    assert stats["convs"] == 15 and stats["conv_transpose"] == 3 and stats["pool3d"] == 1
    with torch.no_grad():
        y = net2(x.to(gpu).bfloat16().contiguous(memory_format=torch.channels_last_3d)).float().cpu()
    assert (y - ref).abs().max() < 0.05, (y - ref).abs().max()


@pytest.mark.gpu
def test_unet3d_package_and_tiled_volume_gpu(gpu, pkg3d):
    from bioengine_worker_amd.bioimageio.runner import PredictionPipeline
    from bioengine_worker_amd.bioimageio.testing import test_model

    rep = test_model(pkg3d)
    assert rep["status"] == "passed", rep
    pipe = PredictionPipeline(pkg3d, device=gpu)
    vol = np.random.default_rng(0).normal(300, 50, (1, 1, 40, 96, 80)).astype(np.float32)
    whole = pipe.predict(vol)["probabilities"]
    tiled = pipe.predict(vol, blocksize=2)["probabilities"]
    assert whole.shape == tiled.shape == (1, 1, 40, 96, 80)
    # tiles see reflect-padded context instead of the neighbouring voxels: compare the interiors
    assert np.abs(whole - tiled)[:, :, 4:-4, 4:-4, 4:-4].mean() < 0.02


@pytest.mark.gpu
@pytest.mark.parametrize("N,D,H,W,Cin,Cout", [(1, 8, 40, 72, 32, 64), (2, 5, 33, 20, 16, 32), (1, 7, 20, 36, 1, 16),
                                             (1, 12, 24, 24, 64, 128), (2, 9, 17, 23, 48, 96)])
def test_conv3d_igemm_single_rounding(gpu, N, D, H, W, Cin, Cout, monkeypatch):
    """The implicit-GEMM 3x3x3 kernel (one launch, K = 27 x Cin, fp32 accumulation over all taps)
    against fp32 F.conv3d of the same bf16 operands with ONE bf16 rounding of the output."""
    monkeypatch.setenv("BE_CONV3D", "igemm")
    g = torch.Generator().manual_seed(D * H + Cout)
    x = torch.randn(N, D, H, W, Cin, generator=g).bfloat16()
    w = torch.randn(Cout, Cin, 3, 3, 3, generator=g) / (Cin * 27) ** 0.5
    b = torch.randn(Cout, generator=g) * 0.1
    pc = PackedConv3d(w, b)
    wb = w.bfloat16().float()
    ref = torch.relu(F.conv3d(x.float().permute(0, 4, 1, 2, 3), wb, b, padding=1)).permute(0, 2, 3, 4, 1)
    xp = F.pad(x, (0, pc.cin_pad - Cin)).contiguous().to(gpu)
    y = fused_conv3d(xp, pc.to(gpu), post_relu=True).float().cpu()
    err = (y - ref).abs()
    # one bf16 rounding of the output (2^-8 relative) plus fp32 summation-order noise
    assert (err <= ref.abs() * 2 ** -8 + 1e-4 * ref.abs().max()).all(), err.max()


@pytest.mark.gpu
@pytest.mark.parametrize("N,D,H,W,Cin,Cout", [(1, 6, 10, 12, 64, 32), (2, 3, 5, 7, 128, 64), (1, 4, 8, 8, 32, 16)])
def test_conv_transpose3d_matches_fp32(gpu, N, D, H, W, Cin, Cout):
    """ConvTranspose3d(k=2, s=2) = 1x1x1 MFMA conv to 8*Cout + vol3d.hip depth-to-space, against the
    fp32 torch op on the same bf16-rounded operands."""
    from bioengine_worker_amd.bioimageio.convert import HipConvTranspose3x2

    g = torch.Generator().manual_seed(N * 100 + D + Cin)
    ct = torch.nn.ConvTranspose3d(Cin, Cout, 2, stride=2)
    with torch.no_grad():
        ct.weight.copy_(torch.randn(ct.weight.shape, generator=g) * 0.1)
        ct.bias.copy_(torch.randn(Cout, generator=g))
    x = torch.randn(N, Cin, D, H, W, generator=g)
    xb = x.bfloat16().float()
    with torch.no_grad():
        ref = F.conv_transpose3d(xb, ct.weight.bfloat16().float(), ct.bias, stride=2)
        mod = HipConvTranspose3x2(ct)
        y = mod(x.to(gpu).bfloat16().contiguous(memory_format=torch.channels_last_3d)).float().cpu()
    assert y.shape == ref.shape
    err = ((y - ref).abs().max() / ref.abs().max()).item()
    assert err < 1e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(1, 6, 10, 12, 16), (2, 7, 9, 5, 64), (1, 4, 64, 64, 32)])
def test_maxpool3d_and_depth2space_exact(gpu, shape):
    from bioengine_worker_amd.ops.conv3d import depth2space3d, maxpool3d_ndhwc

    N, D, H, W, C = shape
    x = torch.randn(shape).bfloat16()
    y = maxpool3d_ndhwc(x.to(gpu)).cpu()
    ref = F.max_pool3d(x.float().permute(0, 4, 1, 2, 3), 2).permute(0, 2, 3, 4, 1).bfloat16()
    assert torch.equal(y, ref)  # max of bf16 values is exact
    z = torch.randn(N, D, H, W, 8 * C).bfloat16()
    d = depth2space3d(z.to(gpu), C).cpu()
    assert torch.equal(d, depth2space3d(z, C))  # CPU path: reshape / permute
    assert torch.equal(d[0, 1, 0, 1], z[0, 0, 0, 0, 5 * C: 6 * C])  # sub-voxel (dz, dy, dx) = (1, 0, 1)


@pytest.mark.gpu
def test_head_1x1x1_small_cout(gpu):
    from bioengine_worker_amd.bioimageio.convert import HipConv3d

    conv = torch.nn.Conv3d(16, 3, 1)
    x = torch.randn(2, 16, 5, 12, 20)
    with torch.no_grad():
        ref = conv(x.bfloat16().float())
        mod = HipConv3d(conv)
        y = mod(x.to(gpu).bfloat16().contiguous(memory_format=torch.channels_last_3d)).float().cpu()
    assert y.shape == ref.shape
    assert (y - ref).abs().max().item() < 2e-2 * ref.abs().max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("ck16", ["0", "1"])
@pytest.mark.parametrize("N,D,H,W,Cin,Cout", [(1, 8, 40, 72, 32, 64), (2, 5, 33, 20, 16, 32), (1, 6, 20, 36, 16, 16),
                                              (1, 4, 24, 40, 128, 64), (1, 5, 18, 34, 1, 16)])
def test_conv3d_ztaps_single_rounding(gpu, N, D, H, W, Cin, Cout, ck16, monkeypatch):
    """BE_CONV3D=ztaps: the 3x3x3 conv as ONE launch of the LDS-staged 2-D kernel with the depth taps
    stacked on K, fp32 accumulation over all 27 taps, one bf16 rounding (same bound as the igemm);
    16- and 1-channel inputs unpadded (8-channel chunks, or 16 with BE_CONV3D_CK16=1)."""
    monkeypatch.setenv("BE_CONV3D", "ztaps")
    monkeypatch.setenv("BE_CONV3D_CK16", ck16)
    g = torch.Generator().manual_seed(N * 1000 + D * 10 + Cin)
    w = torch.randn(Cout, Cin, 3, 3, 3, generator=g) / (27 * Cin) ** 0.5
    b = torch.randn(Cout, generator=g) * 0.1
    pc = PackedConv3d(w, b).to(gpu)
    x = torch.randn(N, D, H, W, pc.cin_pad, generator=g)
    x[..., Cin:] = 0
    xb = x.to(gpu).bfloat16().contiguous()
    for relu in (False, True):
        y = fused_conv3d(xb, pc, post_relu=relu).float().cpu()
        ref = F.conv3d(x.bfloat16().float()[..., :Cin].permute(0, 4, 1, 2, 3), w.bfloat16().float(), b, padding=1)
        ref = (torch.relu(ref) if relu else ref).permute(0, 2, 3, 4, 1)
        err = (y - ref).abs().max().item()
        assert err <= 2 ** -7 * ref.abs().max().item() + 1e-3, err
