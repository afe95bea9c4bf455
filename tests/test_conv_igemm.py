"""Linear-tile implicit-GEMM 3x3 conv (csrc/kernels/conv_igemm.hip) against a plain fp32 PyTorch
oracle: conv2d of the same bf16 operands, fp32 accumulation, then bias / residual / the producer-side
activation of the next conv.  The shapes cover tiles that cross image boundaries (28x28, 13x17),
both block shapes (bn 128: 256 pixels x 128 channels; bn 64: 512 x 64), per-image activation shifts
read through a row-strided view, and a ragged last tile."""
import pytest
import torch
import torch.nn.functional as F

from bioengine_worker_amd.ops import conv_igemm as ig

CASES = [
    # N, H, W, Cin, Cout, bn, residual, act (None | "shared" | "image"), post_relu
    (3, 28, 28, 64, 128, 128, True, "image", False),
    (2, 28, 28, 256, 256, 128, True, None, False),
    (4, 56, 56, 128, 128, 128, False, "shared", False),
    (2, 13, 17, 32, 128, 128, True, "image", True),
    (2, 112, 112, 64, 64, 64, True, "image", False),
    (2, 28, 28, 128, 128, 65, True, "image", False),
    (3, 28, 28, 256, 256, 1128, True, "image", False),
    (2, 56, 56, 128, 128, 1065, True, "shared", True),
    (3, 13, 17, 64, 64, 1065, False, "image", False),
    (3, 56, 56, 128, 128, 64, True, "shared", False),
    (5, 7, 9, 16, 64, 64, False, "shared", False),
]


def _oracle(x, w, b, res, s, t, post_relu):
    y = F.conv2d(x.float().permute(0, 3, 1, 2), w.to(torch.bfloat16).float(), None, padding=1).permute(0, 2, 3, 1)
    y = y + b
    if res is not None:
        y = y + res.float()
    if post_relu:
        y = torch.relu(y)
    a = None
    if s is not None:
        yb = y.to(torch.bfloat16).float()
        tt = t[:, None, None, :] if t.dim() == 2 else t
        a = torch.relu(yb * s + tt)
    return y, a


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}x{c[1]}x{c[2]}_{c[3]}-{c[4]}_bn{c[5]}" for c in CASES])
def test_conv3_igemm_matches_fp32(case):
    N, H, W, cin, cout, bn, use_res, act, post_relu = case
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, H, W, cin, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(cout, cin, 3, 3, generator=g) / (9 * cin) ** 0.5).to(dev)
    b = (0.1 * torch.randn(cout, generator=g)).to(dev)
    res = torch.randn(N, H, W, cout, generator=g).to(torch.bfloat16).to(dev) if use_res else None
    s = t = None
    if act:
        s = (1 + 0.1 * torch.randn(cout, generator=g)).to(dev)
        if act == "image":
            big = 0.1 * torch.randn(N, cout + 64, generator=g)  # row-strided view, like the style shifts
            t = big.to(dev)[:, 32: 32 + cout]
        else:
            t = (0.1 * torch.randn(cout, generator=g)).to(dev)
    pk = ig.IgemmConv.from_weight(w, b, bn=bn).to(dev)
    assert ig.supported(N, H, W, cout, bn)
    out, aout = ig.conv3_igemm(x, pk, residual=res, ascale=s, ashift=t, post_relu=post_relu)
    torch.cuda.synchronize()
    y, a = _oracle(x, w, b, res, s, t, post_relu)
    tol = 0.02 * y.abs().max().item() + 1e-2
    err = (out.float() - y).abs().max().item()
    assert err < tol, (err, tol)
    if act:
        erra = (aout.float() - a).abs().max().item()
        assert erra < tol, (erra, tol)
        assert (aout.float() >= 0).all()
    else:
        assert aout is None


@pytest.mark.gpu
def test_conv3_igemm_activated_only():
    """want_out=False: only the consumer's activated copy is written."""
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(2)
    x = torch.randn(2, 28, 28, 128, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(128, 128, 3, 3, generator=g) / (9 * 128) ** 0.5).to(dev)
    pk = ig.IgemmConv.from_weight(w, None).to(dev)
    s = torch.ones(128, device=dev)
    t = torch.zeros(128, device=dev)
    out, aout = ig.conv3_igemm(x, pk, want_out=False, ascale=s, ashift=t)
    y, a = _oracle(x, w, torch.zeros(128, device=dev), None, s, t, False)
    assert out is None
    assert (aout.float() - a).abs().max().item() < 0.03 * a.abs().max().item() + 1e-2


def test_conv3_igemm_cpu_reference_path():
    """CPU fallback = the oracle itself (shapes and packing only)."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(1, 9, 11, 32, generator=g).to(torch.bfloat16)
    w = torch.randn(64, 32, 3, 3, generator=g) / 17
    pk = ig.IgemmConv.from_weight(w, torch.zeros(64))
    assert pk.wp.numel() == 64 * 32 * 9 and pk.bnc == 64
    # packing: block (c16=0, tap 4, f=0), slot h*32+co, element j == W[co][h*8+j][1][1]
    blk = pk.wp.view(1, 2, 9, 2, 2, 32, 8)[0, 0, 4, 0]
    assert torch.equal(blk[1, 5, 3], w[5, 11, 1, 1].to(torch.bfloat16))
    out, aout = ig.conv3_igemm(x, pk, ascale=torch.ones(64), ashift=torch.zeros(64))
    assert out.shape == (1, 9, 11, 64) and aout.shape == out.shape


@pytest.mark.gpu
@pytest.mark.parametrize("inmode,shift2d", [("pool2", False), ("up2", True), ("none", True)])
def test_fused_conv_post_activation(inmode, shift2d):
    """Per-layer kernel with the producer-side activation of its consumer in the epilogue."""
    from bioengine_worker_amd.ops.conv import PackedConv, fused_conv2d

    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(4)
    N, H, W, cin, cout = 2, 28, 36, 64, 128
    Hs, Ws = {"none": (H, W), "pool2": (2 * H, 2 * W), "up2": (H // 2, W // 2)}[inmode]
    x = torch.randn(N, Hs, Ws, cin, generator=g).bfloat16().to(dev)
    pc = PackedConv.from_weight(torch.randn(cout, cin, 3, 3, generator=g) / (9 * cin) ** 0.5,
                                0.1 * torch.randn(cout, generator=g)).to(dev)
    sc, sh = (1 + 0.1 * torch.randn(cin, generator=g)).to(dev), (0.1 * torch.randn(cin, generator=g)).to(dev)
    res = torch.randn(N, H, W, cout, generator=g).bfloat16().to(dev)
    qs = (1 + 0.2 * torch.randn(cout, generator=g)).to(dev)
    qt = (0.2 * torch.randn(N, cout, generator=g) if shift2d else 0.2 * torch.randn(cout, generator=g)).to(dev)
    base = fused_conv2d(x, pc, scale=sc, shift=sh, relu=True, inmode=inmode, residual=res)
    got = fused_conv2d(x, pc, scale=sc, shift=sh, relu=True, inmode=inmode, residual=res, post_scale=qs,
                       post_shift=qt, post_relu=True)
    want = torch.relu(base.float() * qs + (qt[:, None, None, :] if shift2d else qt))
    assert (got.float() - want).abs().max().item() < 0.02 * want.abs().max().item() + 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["1", "pp"])
def test_cpnet_engine_igemm_path_matches_module(monkeypatch, kind):
    """The whole inference network with the deep levels on an implicit-GEMM path (producer-side
    activations; kind 1 = conv_igemm.hip, pp = gemm_pp.hip) against the fp32 cellpose-style
    module; no worse than the per-layer path."""
    from bioengine_worker_amd.models.cpnet import CPnet, CPnetEngine, to_nhwc_input

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = CPnet().randomize_(3).eval()
    x = torch.randn(3, 2, 224, 224)
    with torch.no_grad():
        ref, style_ref = net(x)[:2]
    xin = to_nhwc_input(x, 8).to(dev)
    monkeypatch.setenv("BE_CPNET_IGEMM", kind)
    monkeypatch.setenv("BE_CPNET_IGEMM_LEVELS", "2,3")
    eng = CPnetEngine(net, dev)
    assert ("down", 3, 1) in eng.ig and ("up", 3, 0) in eng.ig and ("up", 2, 1) in eng.ig
    y, st = eng(xin)
    monkeypatch.setenv("BE_CPNET_IGEMM", "0")
    eng0 = CPnetEngine(net, dev)
    assert not eng0.ig
    y0, _ = eng0(xin)
    y, y0 = y.cpu(), y0.cpu()
    rel = lambda a, b: ((a - b).pow(2).mean().sqrt() / b.pow(2).mean().sqrt()).item()
    e_ig, e_layer = rel(y, ref), rel(y0, ref)
    assert e_ig < 4e-2 and e_ig < 1.25 * e_layer + 1e-3, (e_ig, e_layer)
    assert (st.cpu() - style_ref).abs().max().item() < 2e-2
