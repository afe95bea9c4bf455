"""Epilogue-fused autotuned hipBLASLt GEMMs (``ops/gemm.py``, ``csrc/kernels/gemm_lt.hip``) against
fp32 PyTorch references of the same ops, at ViT block shapes and at ragged ones; plus graph capture
after tuning (the training engine's usage)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _lt_on(monkeypatch):
    monkeypatch.setenv("BE_LT", "1")  # the tuned-hipBLASLt path is opt-in (ops/gemm.py enabled())


def _rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def _bf(*shape, s=1.0, dev="cuda"):
    return (torch.randn(*shape, device=dev) * s).bfloat16()


@pytest.mark.parametrize("M,K,N", [(2048, 1024, 3072), (1000, 192, 1024), (1024, 4096, 1024)])
def test_linear_mm_wgrad(gpu, M, K, N):
    from bioengine_worker_amd.ops import gemm

    torch.manual_seed(0)
    x, w, b = _bf(M, K), _bf(N, K, s=K ** -0.5), _bf(N, s=0.1)
    ref = F.linear(x.float(), w.float(), b.float())
    assert _rel(gemm.linear(x, w, b), ref) < 1e-2
    assert _rel(gemm.linear(x, w), x.float() @ w.float().t()) < 1e-2
    w2 = _bf(K, N, s=K ** -0.5)
    assert _rel(gemm.mm(x, w2), x.float() @ w2.float()) < 1e-2
    dy = _bf(M, N)
    out = torch.full((N, K), 7.0, device=gpu)
    gemm.wgrad(dy, x, out)
    assert _rel(out, dy.float().t() @ x.float()) < 1e-3  # fp32 output: only the bf16 inputs round


def test_linear_gelu_aux_and_dgelu_bgrad(gpu):
    from bioengine_worker_amd.ops import gemm

    torch.manual_seed(1)
    M, D, F4 = 2048, 1024, 4096
    x, w1, b1 = _bf(M, D), _bf(F4, D, s=D ** -0.5), _bf(F4, s=0.5)
    g, f = gemm.linear_gelu(x, w1, b1)
    f_ref = F.linear(x.float(), w1.float(), b1.float())
    assert _rel(f, f_ref) < 1e-2  # aux = pre-activation including the bias
    assert _rel(g, F.gelu(f_ref)) < 1.2e-2  # tanh-form epilogue GELU vs the erf reference
    dm, w2 = _bf(M, D), _bf(D, F4, s=F4 ** -0.5)
    db = torch.full((F4,), 5.0, device=gpu)
    df = gemm.mm_dgelu(dm, w2, f, out_db=db)
    ff = f.float().requires_grad_(True)
    (gp,) = torch.autograd.grad(F.gelu(ff), ff, grad_outputs=dm.float() @ w2.float())
    assert _rel(df, gp) < 2e-2
    assert _rel(db, gp.sum(0)) < 2e-2


def test_tuned_gemm_replays_in_graph(gpu):
    from bioengine_worker_amd.ops import gemm

    torch.manual_seed(2)
    x, w, b = _bf(1024, 1024), _bf(3072, 1024, s=1 / 32), _bf(3072, s=0.1)
    y0 = gemm.linear(x, w, b)  # tuned eagerly
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        gemm.linear(x, w, b)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        y = gemm.linear(x, w, b)
    x.copy_(_bf(1024, 1024))
    g.replay()
    torch.cuda.synchronize()
    assert _rel(y, F.linear(x.float(), w.float(), b.float())) < 1e-2
    assert not torch.equal(y, y0)
    rows = gemm.plans()
    assert any(r["M"] == 1024 and r["N"] == 3072 and r["K"] == 1024 for r in rows)
    assert all(r["candidates"] >= 1 for r in rows)
