"""Deferred cat / max-pool fusion of the 2-D graph pass (bioimageio/convert.py, DeferredFusion).

CPU: the scope defers ``torch.cat`` / ``MaxPool2d`` into placeholders that the consuming HipConv2d
reads from their sources, fills a placeholder before any other consumer touches it, and leaves
results unchanged.  GPU: the U-Net of the EM line runs its decoder convs on ``be_conv2d_concat``
and its encoder convs on the pooling loader with bit-identical output to the unfused graph.
"""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from bioengine_worker_amd.bioimageio import convert as cv


class TinyUNet(nn.Module):
    def __init__(self, leak_cat: bool = False):
        super().__init__()
        self.enc = nn.Sequential(nn.Conv2d(8, 32, 3, padding=1), nn.BatchNorm2d(32), nn.ReLU())
        self.down = nn.MaxPool2d(2)
        self.mid = nn.Sequential(nn.Conv2d(32, 32, 3, padding=1), nn.ReLU())
        self.dec = nn.Sequential(nn.Conv2d(64, 32, 3, padding=1), nn.ReLU())
        self.head = nn.Conv2d(32, 8, 1)
        self.leak_cat = leak_cat

    def forward(self, x):
        s = self.enc(x)
        m = self.mid(self.down(s))
        u = F.interpolate(m, scale_factor=2, mode="nearest")
        c = torch.cat([s, u], dim=1)
        y = self.head(self.dec(c))
        if self.leak_cat:  # a second, non-conv consumer of the concatenation: it must see real data
            y = y + c.float().mean()
        return y


def _pair(leak_cat):
    torch.manual_seed(0)
    net = TinyUNet(leak_cat).eval()
    with torch.no_grad():
        net.enc[1].running_mean.uniform_(-0.1, 0.1)
        net.enc[1].running_var.uniform_(0.5, 1.5)
    a, st = cv.optimize_for_mi355x(copy.deepcopy(net))
    assert st["pool2d"] == 1 and st["convs"] == 4
    return a


@pytest.mark.parametrize("leak_cat", [False, True])
def test_deferred_fusion_cpu_matches_eager(monkeypatch, leak_cat):
    model = _pair(leak_cat)
    x = torch.randn(2, 8, 32, 32).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        ref = model(x).float()  # scope off on CPU: plain cat / max-pool
        monkeypatch.setattr(cv.DeferredFusion, "ALLOW_CPU", True)
        out = model(x).float()
    deferred, filled = model._be_fusion_stats
    assert deferred == 2
    assert filled == (1 if leak_cat else 0)
    # the fused consumers run the kernel's reference math (bf16 weights / activations), the unfused
    # CPU convs fp32 weights: equal up to bf16 rounding
    err = (out - ref).abs().max().item()
    assert err <= 0.05 * ref.abs().max().item() + 1e-2, err


class TinyUp(nn.Module):
    """up-conv -> cat -> conv (the decoder step), plus an optional second use of the up-conv output."""

    def __init__(self, leak_up: bool = False):
        super().__init__()
        self.up = nn.ConvTranspose2d(32, 16, 2, stride=2)
        self.dec = nn.Sequential(nn.Conv2d(32, 16, 3, padding=1), nn.ReLU())
        self.leak_up = leak_up

    def forward(self, x, s):
        u = self.up(x)
        y = self.dec(torch.cat([s, u], dim=1)).float()
        return y + u.float().mean() if self.leak_up else y


@pytest.mark.parametrize("leak_up", [False, True])
def test_deferred_depth_to_space_cpu(monkeypatch, leak_up):
    torch.manual_seed(1)
    model, st = cv.optimize_for_mi355x(TinyUp(leak_up).eval())
    assert st["conv_transpose"] == 1
    x = torch.randn(2, 32, 8, 12).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    s = torch.randn(2, 16, 16, 24).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        ref = model(x, s)
        monkeypatch.setattr(cv.DeferredFusion, "ALLOW_CPU", True)
        out = model(x, s)
    assert model._be_fusion_stats == (2, 1 if leak_up else 0)
    err = (out - ref).abs().max().item()
    assert err <= 0.05 * ref.abs().max().item() + 1e-2, err


def test_scope_fills_on_any_other_use(monkeypatch):
    monkeypatch.setattr(cv.DeferredFusion, "ALLOW_CPU", True)
    a = torch.randn(1, 8, 4, 4).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    b = torch.randn(1, 16, 4, 4).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    scope = cv.DeferredFusion()
    with scope:
        c = torch.cat([a, b], dim=1)
        assert len(scope.pending) == 1
        s = c.sum()  # any torch call on the placeholder fills it first
        assert not scope.pending and scope.filled == 1
        p = scope.defer_pool(a)
        scope.flush()
    assert torch.equal(c, torch.cat([a, b], dim=1))
    assert torch.equal(s, torch.cat([a, b], dim=1).sum())
    assert torch.equal(p, F.max_pool2d(a, 2))


@pytest.mark.gpu
def test_unet2d_deferred_fusion_bit_identical(tmp_path, monkeypatch):
    from bioengine_worker_amd.bioimageio.package import write_unet2d_package
    from bioengine_worker_amd.bioimageio.runner import PredictionPipeline

    dev = torch.device("cuda", 0)
    root = tmp_path / "unet"
    write_unet2d_package(root, "unet", in_channels=1, out_channels=1, features=(32, 64, 128, 256),
                         test_shape=(1, 1, 128, 128), torchscript=False)
    pipe = PredictionPipeline(root, device=dev)
    x = torch.rand(4, 1, 256, 256, device=dev)
    fused = next(iter(pipe.predict_tensors(x).values())).float()
    assert pipe.convert_stats["pool2d"] == 3
    # 3 pools, 3 up-conv shuffles, 3 concatenations; none filled
    assert pipe.model._be_fusion_stats == (9, 0), pipe.model._be_fusion_filled
    monkeypatch.setattr(cv, "LAZY", False)
    plain = next(iter(pipe.predict_tensors(x).values())).float()
    assert torch.equal(fused, plain), (fused - plain).abs().max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("ca,cb,cout", [(32, 32, 32), (64, 64, 64), (128, 128, 128), (8, 24, 16)])
def test_conv2d_concat_matches_fp32(ca, cb, cout):
    """be_conv2d_concat against the fp32 conv of the materialised concatenation (one bf16 rounding)
    and bit-identical to the per-layer kernel on torch.cat."""
    from bioengine_worker_amd.ops.conv import PackedConv, fused_conv2d, fused_conv2d_concat

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    N, H, W = 3, 45, 70  # ragged tiles in both directions
    a = torch.randn(N, H, W, ca, device=dev, generator=g).to(torch.bfloat16)
    b = torch.randn(N, H, W, cb, device=dev, generator=g).to(torch.bfloat16)
    w = torch.randn(cout, ca + cb, 3, 3, device=dev, generator=g) / (3 * (ca + cb) ** 0.5)
    bias = torch.randn(cout, device=dev, generator=g)
    pc = PackedConv.from_weight(w, bias)
    y = fused_conv2d_concat(a, b, pc, post_relu=True)
    ycat = fused_conv2d(torch.cat([a, b], -1).contiguous(), pc, post_relu=True)
    assert torch.equal(y, ycat)
    x32 = torch.cat([a, b], -1).float().permute(0, 3, 1, 2)
    ref = torch.relu(F.conv2d(x32, w.to(torch.bfloat16).float(), bias, padding=1)).permute(0, 2, 3, 1)
    err = (y.float() - ref).abs().max().item()
    assert err <= 0.02 * ref.abs().max().item() + 1e-2, err


class TinyUNet3d(nn.Module):
    def __init__(self):
        super().__init__()
        self.enc = nn.Sequential(nn.Conv3d(8, 16, 3, padding=1), nn.ReLU())
        self.mid = nn.Sequential(nn.Conv3d(16, 16, 3, padding=1), nn.ReLU())
        self.dec = nn.Sequential(nn.Conv3d(32, 16, 3, padding=1), nn.ReLU())

    def forward(self, x):
        s = self.enc(x)
        return self.dec(torch.cat([s, self.mid(s)], dim=1))


def test_deferred_fusion_3d_cpu(monkeypatch):
    torch.manual_seed(0)
    model, st = cv.optimize_for_mi355x(TinyUNet3d().eval())
    assert st["convs"] == 3
    x = torch.randn(1, 8, 6, 16, 16).to(torch.bfloat16).contiguous(memory_format=torch.channels_last_3d)
    with torch.no_grad():
        ref = model(x).float()
        monkeypatch.setattr(cv.DeferredFusion, "ALLOW_CPU", True)
        out = model(x).float()
    assert model._be_fusion_stats == (1, 0)
    err = (out - ref).abs().max().item()
    assert err <= 0.05 * ref.abs().max().item() + 1e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize("ca,cb,cout", [(16, 16, 16), (32, 32, 32), (64, 64, 64)])
def test_conv3d_concat_matches_fp32(ca, cb, cout):
    from bioengine_worker_amd.ops.conv3d import PackedConv3d, fused_conv3d, fused_conv3d_concat

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    N, D, H, W = 2, 9, 21, 40
    a = torch.randn(N, D, H, W, ca, device=dev, generator=g).to(torch.bfloat16)
    b = torch.randn(N, D, H, W, cb, device=dev, generator=g).to(torch.bfloat16)
    w = torch.randn(cout, ca + cb, 3, 3, 3, device=dev, generator=g) / (5 * (ca + cb) ** 0.5)
    bias = torch.randn(cout, device=dev, generator=g)
    pc = PackedConv3d(w, bias)
    pc.to(dev)
    y = fused_conv3d_concat(a, b, pc, post_relu=True)
    ycat = fused_conv3d(torch.cat([a, b], -1).contiguous(), pc, post_relu=True)
    assert torch.equal(y, ycat)
    x32 = torch.cat([a, b], -1).float().permute(0, 4, 1, 2, 3)
    ref = torch.relu(F.conv3d(x32, w.to(torch.bfloat16).float(), bias, padding=1)).permute(0, 2, 3, 4, 1)
    err = (y.float() - ref).abs().max().item()
    assert err <= 0.02 * ref.abs().max().item() + 1e-2, err


@pytest.mark.gpu
def test_unet3d_deferred_fusion_bit_identical(tmp_path, monkeypatch):
    from bioengine_worker_amd.bioimageio.package import write_unet3d_package
    from bioengine_worker_amd.bioimageio.runner import PredictionPipeline

    dev = torch.device("cuda", 0)
    root = tmp_path / "unet3d"
    write_unet3d_package(root, "unet3d", in_channels=1, out_channels=1, features=(16, 32, 64, 128),
                         test_shape=(1, 1, 16, 32, 32))
    pipe = PredictionPipeline(root, device=dev)
    x = torch.rand(2, 1, 32, 64, 64, device=dev)
    fused = next(iter(pipe.predict_tensors(x).values())).float()
    assert pipe.model._be_fusion_stats == (3, 0)  # the three decoder concatenations, none filled
    monkeypatch.setattr(cv, "LAZY", False)
    plain = next(iter(pipe.predict_tensors(x).values())).float()
    assert torch.equal(fused, plain), (fused - plain).abs().max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("ca,cb", [(32, 32), (64, 64), (16, 16)])
def test_conv2d_concat_subpixel_source_identical(ca, cb):
    """INMODE 6 (the second source read in the 2x2 transposed conv's sub-pixel layout) is bit-identical
    to INMODE 4 on the shuffled tensor."""
    from bioengine_worker_amd.ops.conv import PackedConv, depth_to_space2, fused_conv2d_concat

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(2)
    N, H, W = 2, 38, 70
    a = torch.randn(N, H, W, ca, device=dev, generator=g).to(torch.bfloat16)
    y4 = torch.randn(N, H // 2, W // 2, 4 * cb, device=dev, generator=g).to(torch.bfloat16)
    w = torch.randn(32, ca + cb, 3, 3, device=dev, generator=g) / (3 * (ca + cb) ** 0.5)
    pc = PackedConv.from_weight(w, torch.randn(32, device=dev, generator=g))
    y = fused_conv2d_concat(a, y4, pc, post_relu=True, xb_d2s=True)
    ref = fused_conv2d_concat(a, depth_to_space2(y4, cb).contiguous(), pc, post_relu=True)
    assert torch.equal(y, ref)
