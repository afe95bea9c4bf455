"""Two-group ping-pong 256x256 GEMM (csrc/kernels/gemm_8p.hip via ops/gemm_8p.py) against fp32 PyTorch:
every epilogue, ragged M / N (partial tiles), K of 1-16+ tiles (the prologue / tail re-read path)."""
import pytest
import torch
import torch.nn.functional as F

from bioengine_worker_amd.ops import gemm_8p

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _close(got, want, tol=1.5e-2):
    err = ((got.float() - want).abs().max() / want.abs().max().clamp_min(1e-6)).item()
    assert err < tol, err


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 128), (300, 200, 192), (1000, 1028, 1024),
                                   (8192, 1024, 4096), (2048, 3072, 1024)])
def test_linear_bias(M, N, K):
    g = torch.Generator().manual_seed(M * 7 + N + K)
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV)
    ref = x.float() @ w.float().t()
    _close(gemm_8p.linear(x, w), ref)
    _close(gemm_8p.linear(x, w, b), ref + b)
    _close(gemm_8p.linear(x, w, b.to(torch.bfloat16)), ref + b.to(torch.bfloat16).float())


def test_epilogues():
    g = torch.Generator().manual_seed(3)
    M, N, K = 520, 1024, 512
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV)
    r = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    ref = x.float() @ w.float().t() + b
    _close(gemm_8p.linear_res(x, w, b, r), ref + r.float())
    gg, f = gemm_8p.linear_gelu(x, w, b)
    _close(f, ref)
    assert (gg.float() - F.gelu(f.float())).abs().max().item() < 2e-2
    g2 = gemm_8p.linear_gelu_only(x, w, b)
    assert torch.equal(g2, gg)


def test_matches_gemm_mt_bitwise_order_free():
    """Same bf16 rounding point as the macro-tile kernel: outputs agree to bf16 rounding."""
    from bioengine_worker_amd.ops import gemm_mt

    g = torch.Generator().manual_seed(5)
    x = torch.randn(1024, 1024, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(3072, 1024, generator=g) * 0.03).to(DEV, torch.bfloat16)
    a, b = gemm_8p.linear(x, w).float(), gemm_mt.linear(x, w).float()
    assert ((a - b).abs() / b.abs().clamp_min(1e-2)).max().item() < 2e-2
