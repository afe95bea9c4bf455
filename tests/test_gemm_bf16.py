"""In-house bf16 GEMM (csrc/kernels/gemm_bf16.hip) against plain fp32 PyTorch of the same op, for
every layout / epilogue the CPSAM engine uses, at ViT-L shapes (batch 1: M = 1,024 tokens) and
ragged ones."""
import pytest
import torch
import torch.nn.functional as F

from bioengine_worker_amd.ops import gemm_bf16 as gb

SHAPES = [(1024, 3072, 1024), (1024, 1024, 4096), (1536, 4096, 1024), (200, 384, 256)]


def _rand(*shape, dev, scale=1.0, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    return (scale * torch.randn(*shape, device=dev, generator=g)).to(torch.bfloat16)


def _close(got, want, rtol=2e-2):
    err = (got.float() - want.float()).abs().max().item()
    assert err <= rtol * want.float().abs().max().item() + 1e-3, err


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("cfg", [0, 1, 2, 3])
def test_linear_and_gelu(M, N, K, cfg):
    dev = torch.device("cuda", 0)
    x, w = _rand(M, K, dev=dev, seed=1), _rand(N, K, dev=dev, scale=K ** -0.5, seed=2)
    b = torch.randn(N, device=dev)
    ref = F.linear(x.float(), w.float(), b)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    gb._call(x, w, out, M, N, K, K, K, N, 0, 0, gb.E_BIAS, bias=b, cfg=cfg)
    _close(out, ref)
    out0 = torch.empty_like(out)
    gb._call(x, w, out0, M, N, K, K, K, N, 0, 0, gb.E_NONE, cfg=cfg)
    _close(out0, ref - b)
    f = torch.empty_like(out)
    g = torch.empty_like(out)
    gb._call(x, w, f, M, N, K, K, K, N, 0, 0, gb.E_BIAS_GELU, C2=g, bias=b, cfg=cfg)
    _close(f, ref)
    _close(g, F.gelu(f.float()))


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [s for s in SHAPES if s[1] % 128 == 0])
@pytest.mark.parametrize("cfg", [0, 1, 2])
def test_dgrad_and_dgelu(M, N, K, cfg):
    dev = torch.device("cuda", 0)
    dm, w2 = _rand(M, K, dev=dev, seed=3), _rand(K, N, dev=dev, scale=K ** -0.5, seed=4)
    ref = dm.float() @ w2.float()
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    gb._call(dm, w2, out, M, N, K, K, N, N, 0, 1, gb.E_NONE, cfg=cfg)
    _close(out, ref)
    f = _rand(M, N, dev=dev, seed=5)
    db = torch.zeros(N, device=dev)
    df = torch.empty_like(out)
    gb._call(dm, w2, df, M, N, K, K, N, N, 0, 1, gb.E_DGELU, aux=f, dbias=db, cfg=cfg)
    want = gb._gelu_grad(f) * ref
    _close(df, want)
    _close(db, df.float().sum(0), rtol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k", [(1024, 1024, 1024), (8192, 1024, 4096), (2048, 3072, 1024), (1024, 384, 256)])
def test_wgrad_fp32_split(m, n, k):
    dev = torch.device("cuda", 0)
    dy, x = _rand(m, n, dev=dev, seed=6), _rand(m, k, dev=dev, seed=7)
    out = torch.full((n, k), float("nan"), device=dev)
    gb.wgrad(dy, x, out)
    ref = dy.float().t() @ x.float()
    err = (out - ref).abs().max().item()
    assert err <= 1e-3 * ref.abs().max().item() + 1e-3, (err, gb.wgrad_split(n, k, m))


def test_cpu_reference_path():
    x, w, b = torch.randn(8, 64), torch.randn(32, 64), torch.randn(32)
    g, f = gb.linear_gelu(x, w, b)
    assert torch.allclose(f, F.linear(x, w, b)) and torch.allclose(g, F.gelu(f))
    out = torch.empty(32, 64)
    gb.wgrad(torch.randn(8, 32), x, out)
    assert gb.wgrad_split(1024, 1024, 8192) >= 2 and gb.wgrad_split(4096, 1024, 1024) == 1
