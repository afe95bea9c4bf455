"""Numerics of the fused NHWC conv HIP kernel vs the PyTorch fp32 reference of the same op."""
import pytest
import torch

from bioengine_worker_amd.ops.conv import PackedConv, fused_conv2d, fused_conv2d_ref

CASES = [
    # ks, cin, cout, inmode, H, W, with_x2, with_res, relu, shift2d
    (3, 8, 32, "none", 40, 72, False, False, True, False),
    (3, 32, 32, "none", 64, 64, False, True, True, False),
    (3, 64, 64, "pool2", 64, 96, False, False, True, False),
    (3, 128, 64, "up2", 16, 32, False, False, True, False),
    (1, 64, 128, "none", 32, 32, False, False, False, False),
    (3, 256, 256, "none", 16, 16, True, True, True, True),
    (1, 32, 16, "none", 24, 40, False, False, True, False),
    (3, 32, 64, "none", 13, 45, True, False, True, True),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_fused_conv_matches_reference(gpu, case):
    ks, cin, cout, inmode, H, W, with_x2, with_res, relu, shift2d = case
    torch.manual_seed(0)
    N = 2
    Hs, Ws = {"none": (H, W), "pool2": (H * 2, W * 2), "up2": (H // 2, W // 2)}[inmode]
    x = torch.randn(N, Hs, Ws, cin).bfloat16()
    w = torch.randn(cout, cin, ks, ks) / (cin * ks * ks) ** 0.5
    b = torch.randn(cout) * 0.1
    pc = PackedConv.from_weight(w, b)
    scale = (1 + 0.1 * torch.randn(cin)).float()
    shift = (0.1 * torch.randn(N, cin) if shift2d else 0.1 * torch.randn(cin)).float()
    x2 = torch.randn(N, H, W, cin).bfloat16() if with_x2 else None
    res = torch.randn(N, H, W, cout).bfloat16() if with_res else None
    ref = fused_conv2d_ref(x, pc, x2=x2, scale=scale, shift=shift, relu=relu, residual=res, inmode=inmode).float()
    dev = lambda t: None if t is None else t.to(gpu)
    out = fused_conv2d(dev(x), pc.to(gpu), x2=dev(x2), scale=dev(scale), shift=dev(shift), relu=relu,
                       residual=dev(res), inmode=inmode).float().cpu()
    err = (out - ref).abs().max().item()
    tol = 2e-2 * max(1.0, ref.abs().max().item())
    assert err < tol, f"max err {err} (tol {tol})"


@pytest.mark.gpu
def test_fused_conv_nchw_f32_head(gpu):
    torch.manual_seed(1)
    x = torch.randn(3, 48, 64, 32).bfloat16()
    w = torch.randn(3, 32, 1, 1) / 32 ** 0.5
    b = torch.randn(3)
    pc = PackedConv.from_weight(w, b, cout_pad_to=16)
    scale = torch.rand(32) + 0.5
    shift = torch.randn(32) * 0.1
    ref = fused_conv2d_ref(x, pc, scale=scale, shift=shift, relu=True, out_nchw_f32=True, cout_valid=3)
    out = fused_conv2d(x.to(gpu), pc.to(gpu), scale=scale.to(gpu), shift=shift.to(gpu), relu=True,
                       out_nchw_f32=True, cout_valid=3).cpu()
    assert out.shape == (3, 3, 48, 64)
    assert (out - ref).abs().max().item() < 2e-2 * max(1, ref.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("nw", [4, 8])
@pytest.mark.parametrize("cin,cout,inmode,persist", [(32, 32, "none", 7), (8, 32, "none", 0), (64, 32, "up2", 13),
                                                     (32, 16, "none", 3), (64, 64, "pool2", 0)])
def test_fused_conv_persistent_many_tiles(gpu, nw, cin, cout, inmode, persist):
    """Many more pixel tiles than persistent workgroups: every tile must be produced exactly once."""
    from bioengine_worker_amd.ops import _native

    torch.manual_seed(2)
    N, H, W = 6, 96, 160
    Hs, Ws = {"none": (H, W), "pool2": (H * 2, W * 2), "up2": (H // 2, W // 2)}[inmode]
    x = torch.randn(N, Hs, Ws, cin).bfloat16()
    w = torch.randn(cout, cin, 3, 3) / (cin * 9) ** 0.5
    pc = PackedConv.from_weight(w, torch.randn(cout) * 0.1)
    shift = (0.1 * torch.randn(N, cin)).float()
    ref = fused_conv2d_ref(x, pc, shift=shift, relu=True, inmode=inmode).float()
    _native.call("be_conv2d_set_persist", persist)
    try:
        out = fused_conv2d(x.to(gpu), pc.to(gpu), shift=shift.to(gpu), relu=True, inmode=inmode, nw=nw).float().cpu()
    finally:
        _native.call("be_conv2d_set_persist", 0)
    err = (out - ref).abs().max().item()
    assert err < 2e-2 * max(1.0, ref.abs().max().item()), err
