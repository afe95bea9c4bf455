"""Macro-tile bf16 GEMM family (csrc/kernels/gemm_mt.hip via ops/gemm_mt.py) against fp32 PyTorch
references computed from the same bf16 operands: every tile configuration, every layout (forward x W^T,
data gradient x W, weight gradient dy^T x with in-launch split-K), every fused epilogue (bias fp32 /
bf16, bias + GELU, bias + residual, GELU backward with the bias gradient), partial edge tiles."""
import pytest
import torch
import torch.nn.functional as F

from bioengine_worker_amd.ops import gemm_mt

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _r(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(DEV, torch.bfloat16)


def _close(got, want, tol=2e-2):
    err = (got.float() - want.float()).abs().max().item()
    ref = want.float().abs().max().item() + 1e-6
    assert err <= tol * ref, (err, ref)


@pytest.fixture
def force_cfg(monkeypatch):
    def f(cfg, split=1):
        monkeypatch.setenv("BE_GEMM_MT_CFG", f"{cfg},{split}")
    return f


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("M,N,K", [(512, 384, 256), (300, 196, 128), (1024, 1024, 1024)])
def test_linear_bias_matches_fp32(cfg, M, N, K, force_cfg):
    force_cfg(cfg)
    x, w = _r(M, K, seed=1), _r(N, K, scale=0.05, seed=2)
    b = torch.randn(N, device=DEV)
    for bias in (b, b.to(torch.bfloat16), None):
        got = gemm_mt.linear(x, w, bias)
        want = F.linear(x.float(), w.float(), None if bias is None else bias.float())
        _close(got, want)


@pytest.mark.parametrize("cfg", [0, 1, 2, 4])
def test_linear_gelu_and_residual(cfg, force_cfg):
    force_cfg(cfg)
    M, N, K = 768, 512, 320
    x, w, b = _r(M, K, seed=3), _r(N, K, scale=0.05, seed=4), torch.randn(N, device=DEV)
    g, f = gemm_mt.linear_gelu(x, w, b)
    fref = F.linear(x.float(), w.float(), b)
    _close(f, fref)
    # g is the GELU of the bf16-rounded f the kernel stored
    _close(g, F.gelu(f.float()), tol=1e-2)
    r = _r(M, N, seed=5)
    y = gemm_mt.linear_res(x, w, b.to(torch.bfloat16), r)
    _close(y, fref + r.float())


@pytest.mark.parametrize("cfg", [0, 2, 3, 4])
def test_dgrad_and_dgelu(cfg, force_cfg):
    force_cfg(cfg)
    M, K, N = 640, 384, 512
    dy, w = _r(M, K, seed=6), _r(K, N, scale=0.05, seed=7)
    _close(gemm_mt.mm(dy, w), dy.float() @ w.float())
    f = _r(M, N, seed=8)
    db = torch.full((N,), 7.0, device=DEV)  # overwritten, not accumulated into
    df = gemm_mt.mm_dgelu(dy, w, f, db)
    want = gemm_mt._gelu_grad(f) * (dy.float() @ w.float())
    _close(df, want)
    _close(db, df.float().sum(0), tol=1e-3)


@pytest.mark.parametrize("cfg,split", [(0, 1), (0, 3), (2, 2), (3, 4), (4, 1), (4, 5)])
def test_wgrad_split_k_in_launch(cfg, split, force_cfg):
    force_cfg(cfg, split)
    m, n, k = 1024, 512, 256  # tokens, out features, in features
    dy, x = _r(m, n, seed=9), _r(m, k, seed=10)
    out = torch.full((n, k), float("nan"), device=DEV)
    for _ in range(3):  # repeated calls: the arrival counters reset themselves
        gemm_mt.wgrad(dy, x, out)
        torch.cuda.synchronize()
        _close(out, dy.float().t() @ x.float(), tol=1e-2)


def test_default_table_on_cpsam_shapes():
    """The shapes of the Cellpose-SAM ViT-L step (dim 1024, MLP 4096, 1024 tokens per image) at batch 1
    and 8, through the default (static) configuration choice."""
    for B in (1, 8):
        M = 1024 * B
        x = _r(M, 1024, seed=11)
        for N in (3072, 1024, 4096):
            w = _r(N, 1024, scale=0.03, seed=N)
            _close(gemm_mt.linear(x, w), x.float() @ w.float().t())
            dy = _r(M, N, seed=N + 1)
            _close(gemm_mt.mm(dy, w), dy.float() @ w.float())
            out = torch.empty(N, 1024, device=DEV)
            gemm_mt.wgrad(dy, x, out)
            _close(out, dy.float().t() @ x.float(), tol=1e-2)


@pytest.mark.parametrize("cfg", [0, 2, 3, 4])
def test_partial_tiles_of_transposed_operands(cfg, force_cfg):
    """The CPSAM head shapes: 192-wide outputs / inputs through the k-row-tile (transposed) staging,
    whose chunks past M / N re-read valid memory and are never stored."""
    force_cfg(cfg, 2)
    m = 512
    dy, x = _r(m, 192, seed=12), _r(m, 200, seed=13)
    out = torch.empty(192, 200, device=DEV)
    gemm_mt.wgrad(dy, x, out)
    _close(out, dy.float().t() @ x.float(), tol=1e-2)
    force_cfg(cfg, 1)
    w = _r(256, 184, scale=0.05, seed=14)
    a = _r(320, 256, seed=15)
    _close(gemm_mt.mm(a, w), a.float() @ w.float())
