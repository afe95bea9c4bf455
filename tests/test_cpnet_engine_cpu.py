"""The hand-written CPnet training engine (forward + manual backward, BN in train mode, style path,
max-pool / upsample adjoints, residual and skip grads) against PyTorch autograd, on CPU in fp32.

On CPU every engine op runs its PyTorch reference, so agreement here validates the backward math the
HIP kernels implement (tests/test_cpnet_engine_gpu.py checks the kernels against the same oracle)."""
import copy

import pytest
import torch

from bioengine_worker_amd.models.cpnet import CPnet
from bioengine_worker_amd.ops import conv_train as ct
from bioengine_worker_amd.ops import train_ops
from bioengine_worker_amd.parallel.ddp import FlatParams
from bioengine_worker_amd.train.cpnet_engine import CPnetTrainEngine


def _setup(style_on=True, nbase=(2, 8, 16, 16, 32), B=2, S=32, seed=0):
    torch.manual_seed(seed)
    net = CPnet(nbase=nbase, style_on=style_on).randomize_(seed).train()
    ref = copy.deepcopy(net)
    x = torch.randn(B, 2, S, S)
    lbl = torch.zeros(B, 3, S, S)
    lbl[:, 0] = (torch.rand(B, S, S) > 0.6).float()
    lbl[:, 1:] = torch.randn(B, 2, S, S) * 0.3
    return net, ref, x, lbl


@pytest.mark.parametrize("style_on", [True, False])
def test_engine_grads_match_autograd(style_on):
    net, ref, x, lbl = _setup(style_on)
    # autograd oracle
    y_ref = ref(x)[0]
    loss_ref = train_ops.seg_loss_ref(y_ref, lbl)
    loss_ref.backward()
    # engine
    fp = FlatParams(net, "cpu")
    eng = CPnetTrainEngine(net, fp, B=x.shape[0], S=x.shape[2], device="cpu")
    loss = eng.loss_and_backward(x, lbl)
    assert abs(float(loss) - float(loss_ref.detach())) < 1e-5 * max(1.0, abs(float(loss_ref.detach())))
    named_ref = dict(ref.named_parameters())
    gmax = max(p.grad.abs().max().item() for p in ref.parameters() if p.grad is not None)
    for name, p in net.named_parameters():
        if not p.requires_grad:
            continue
        g_ref = named_ref[name].grad
        assert p.grad is not None, name
        # conv biases feeding a train-mode BN have a mathematically zero gradient (the batch mean
        # removes them): compare those on the global scale, everything else relative to itself
        err = (p.grad - g_ref).abs().max().item()
        tol = 2e-4 * g_ref.abs().max().item() + 2e-6 * gmax
        assert err < tol, f"{name}: err {err:.2e} > tol {tol:.2e}"
    # running statistics follow the same momentum update as nn.BatchNorm2d
    rb = dict(ref.named_buffers())
    for name, b in net.named_buffers():
        if "running" in name:
            torch.testing.assert_close(b, rb[name], rtol=1e-5, atol=1e-6)


def test_engine_forward_matches_module():
    net, ref, x, lbl = _setup()
    fp = FlatParams(net, "cpu")
    eng = CPnetTrainEngine(net, fp, B=x.shape[0], S=x.shape[2], device="cpu")
    y = eng.forward(x)
    torch.testing.assert_close(y, ref(x)[0], rtol=1e-4, atol=1e-4)


def test_bn_site_pool_and_upsample_adjoints():
    """bwd_apply routes du through the transform adjoints (autograd through the same transform)."""
    torch.manual_seed(1)
    N, H, C = 2, 8, 16
    for inmode in ("pool2", "up2"):
        Hs = H * 2 if inmode == "pool2" else H // 2
        x = torch.randn(N, Hs, Hs, C, requires_grad=True)
        v = ct._t_ref(x, inmode)
        du = torch.randn_like(v)
        (v * du).sum().backward()
        got = ct._tT_ref(du, x.detach(), inmode)
        torch.testing.assert_close(got, x.grad)


def test_pack_ref_matches_packed_conv():
    from bioengine_worker_amd.ops.conv import PackedConv

    w = torch.randn(32, 8, 3, 3)
    pc = PackedConv.from_weight(w)
    got = ct.pack_ref(w, pc.cout_pad, pc.cin_pad, pc.ck, pc.kp, False)
    torch.testing.assert_close(got.to(torch.bfloat16), pc.wp)
    # dgrad layout = packing the flipped / transposed weight
    wt = w.flip(2, 3).transpose(0, 1).contiguous()
    pct = PackedConv.from_weight(wt, cin_pad=32)
    got_t = ct.pack_ref(w, pct.cout_pad, pct.cin_pad, pct.ck, pct.kp, True)
    torch.testing.assert_close(got_t.to(torch.bfloat16), pct.wp)


@pytest.mark.parametrize("style_on", [True, False])
def test_groupnorm_engine_grads_match_autograd(style_on):
    """GroupNorm CPnet (per-image, per-group statistics; the data-parallel training default) through
    the same engine: forward and every gradient against autograd."""
    torch.manual_seed(3)
    net = CPnet(nbase=(2, 8, 16, 16, 32), style_on=style_on, norm="group").randomize_(3).train()
    with torch.no_grad():
        for n, p in net.named_parameters():
            if p.requires_grad and p.dim() == 1 and "full" not in n:
                p.add_(0.2 * torch.randn_like(p))  # non-trivial GN affine
    ref = copy.deepcopy(net)
    x = torch.randn(3, 2, 32, 32)
    lbl = torch.zeros(3, 3, 32, 32)
    lbl[:, 0] = (torch.rand(3, 32, 32) > 0.6).float()
    lbl[:, 1:] = torch.randn(3, 2, 32, 32) * 0.3
    loss_ref = train_ops.seg_loss_ref(ref(x)[0], lbl)
    loss_ref.backward()
    fp = FlatParams(net, "cpu")
    eng = CPnetTrainEngine(net, fp, B=3, S=32, device="cpu")
    loss = eng.loss_and_backward(x, lbl)
    assert abs(float(loss) - float(loss_ref.detach())) < 1e-5 * max(1.0, abs(float(loss_ref.detach())))
    named_ref = dict(ref.named_parameters())
    gmax = max(p.grad.abs().max().item() for p in ref.parameters() if p.grad is not None)
    for name, p in net.named_parameters():
        if not p.requires_grad:
            continue
        g_ref = named_ref[name].grad
        err = (p.grad - g_ref).abs().max().item()
        tol = 2e-4 * g_ref.abs().max().item() + 2e-6 * gmax
        assert err < tol, f"{name}: err {err:.2e} > tol {tol:.2e}"
