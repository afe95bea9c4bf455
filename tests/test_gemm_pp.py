"""Ping-pong bf16 GEMM / implicit-GEMM 3x3 conv (csrc/kernels/gemm_pp.hip) against plain fp32
PyTorch of the same op: every tile configuration, ragged M / N, short K (the prologue and drain
edges of the 4-slot ring: 1-6 K-halves), and the CPnet conv epilogue (bias, residual, post-ReLU,
the consumer's BN + ReLU with a per-image style shift)."""
import pytest
import torch
import torch.nn.functional as F

from bioengine_worker_amd.ops import gemm_pp as pp

GEMM_SHAPES = [(8192, 3072, 1024), (1000, 1024, 4096), (300, 260, 32), (512, 384, 64), (777, 512, 96),
               (1024, 256, 160), (256, 128, 192)]


def _rand(*shape, dev, scale=1.0, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    return (scale * torch.randn(*shape, device=dev, generator=g)).to(torch.bfloat16)


def _close(got, want, rtol=2e-2):
    err = (got.float() - want.float()).abs().max().item()
    assert err <= rtol * want.float().abs().max().item() + 1e-3, err


def test_conv3_ref_matches_conv2d_cpu():
    torch.manual_seed(0)
    x = torch.randn(2, 9, 7, 32).to(torch.bfloat16)
    w = torch.randn(64, 32, 3, 3) * 0.1
    b = torch.randn(64)
    out, aout = pp.conv3(x, pp.pack_conv3(w), b, ascale=torch.rand(64), ashift=torch.randn(2, 64))
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.to(torch.bfloat16).float(), b, padding=1).permute(0, 2, 3, 1)
    _close(out, ref)
    assert aout.shape == out.shape and (aout.float() >= 0).all()


def test_linear_cpu_fallback():
    x, w, b = torch.randn(64, 96).to(torch.bfloat16), torch.randn(32, 96).to(torch.bfloat16), torch.randn(32)
    _close(pp.linear(x, w, b), F.linear(x.float(), w.float(), b))
    g, f = pp.linear_gelu(x, w, b)
    _close(g, F.gelu(f.float()))


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", GEMM_SHAPES)
@pytest.mark.parametrize("cfg", [0, 1, 2])
def test_linear_gelu_gpu(M, N, K, cfg):
    dev = torch.device("cuda", 0)
    x, w = _rand(M, K, dev=dev, seed=1), _rand(N, K, dev=dev, scale=K ** -0.5, seed=2)
    b = torch.randn(N, device=dev)
    ref = F.linear(x.float(), w.float(), b)
    _close(pp.linear(x, w, b, cfg=cfg), ref)
    _close(pp.linear(x, w, None, cfg=cfg), ref - b)
    g, f = pp.linear_gelu(x, w, b, cfg=cfg)
    _close(f, ref)
    _close(g, F.gelu(f.float()))


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(8192, 1024, 3072), (1000, 256, 4096), (300, 512, 96), (777, 1024, 32)])
@pytest.mark.parametrize("cfg", [0, 1, 2])
def test_dgrad_and_dgelu_gpu(M, N, K, cfg):
    dev = torch.device("cuda", 0)
    dm, w2 = _rand(M, K, dev=dev, seed=5), _rand(K, N, dev=dev, scale=K ** -0.5, seed=6)
    if N % pp.TILES[cfg][1]:
        pytest.skip("N not a whole number of tiles")
    ref = dm.float() @ w2.float()
    _close(pp.mm(dm, w2, cfg=cfg), ref)
    f = _rand(M, N, dev=dev, seed=7)
    db = torch.empty(N, device=dev)
    df = pp.mm_dgelu(dm, w2, f, out_db=db, cfg=cfg)
    x = f.float()
    gp = 0.5 * (1.0 + torch.erf(x * 0.7071067811865476)) + x * torch.exp(-0.5 * x * x) * 0.3989422804014327
    want = gp * ref
    _close(df, want)
    _close(db, df.float().sum(0), rtol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k", [(8192, 3072, 1024), (1024, 1024, 4096), (2048, 256, 512), (96, 512, 256)])
@pytest.mark.parametrize("cfg", [0, 1, 2])
def test_wgrad_gpu(m, n, k, cfg):
    dev = torch.device("cuda", 0)
    bm, bn = pp.TILES[cfg]
    if n % bm or k % bn:
        pytest.skip("weight shape not a whole number of tiles")
    dy, x = _rand(m, n, dev=dev, seed=8), _rand(m, k, dev=dev, seed=9)
    ref = dy.float().t() @ x.float()
    for split in (None, 1):
        out = torch.full((n, k), float("nan"), device=dev)
        pp.wgrad(dy, x, out, cfg=cfg, split=split)
        _close(out, ref, rtol=5e-3)


CONV_SHAPES = [(2, 28, 28, 256, 256), (3, 56, 56, 128, 128), (2, 17, 23, 64, 128), (1, 5, 300, 32, 64),
               (4, 28, 28, 128, 256)]


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,W,Cin,Cout", CONV_SHAPES)
@pytest.mark.parametrize("cfg", [0, 1, 2])
def test_conv3_gpu(N, H, W, Cin, Cout, cfg):
    dev = torch.device("cuda", 0)
    x = _rand(N, H, W, Cin, dev=dev, seed=3)
    w = (torch.randn(Cout, Cin, 3, 3, device=dev) * (9 * Cin) ** -0.5)
    wp = pp.pack_conv3(w)
    b = torch.randn(Cout, device=dev)
    res = _rand(N, H, W, Cout, dev=dev, seed=4)
    s = torch.rand(Cout, device=dev) + 0.5
    sh = torch.randn(N, Cout, device=dev)
    out, aout = pp.conv3(x, wp, b, residual=res, ascale=s, ashift=sh, cfg=cfg)
    ro, ra = pp.conv3_ref(x, wp, b, residual=res, ascale=s, ashift=sh)
    _close(out, ro)
    _close(aout, ra)
    # activation only (no out), post-ReLU plain out
    o2, a2 = pp.conv3(x, wp, None, want_out=False, ascale=s, ashift=sh[0].contiguous(), cfg=cfg)
    assert o2 is None
    _close(a2, pp.conv3_ref(x, wp, None, ascale=s, ashift=sh[0])[1])
    o3, _ = pp.conv3(x, wp, b, post_relu=True, cfg=cfg)
    _close(o3, pp.conv3_ref(x, wp, b, post_relu=True)[0])
