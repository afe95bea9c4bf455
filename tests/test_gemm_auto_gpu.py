"""Per-shape GEMM choice (ops/gemm_auto.py): every candidate is timed on graph replays, the winner's
result is what the call returns, and the decision is cached per (op, shape)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fresh(monkeypatch):
    from bioengine_worker_amd.ops import gemm_auto

    monkeypatch.delenv("BE_GEMM_AUTO", raising=False)
    gemm_auto._choice.clear()
    yield
    gemm_auto._choice.clear()


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def test_linear_and_wgrad_pick_and_match_fp32():
    from bioengine_worker_amd.ops import gemm_auto

    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(1024, 1024, generator=g).to("cuda", torch.bfloat16)
    w = (torch.randn(3072, 1024, generator=g) * 0.03).to("cuda", torch.bfloat16)
    b = torch.randn(3072, generator=g).to("cuda", torch.bfloat16)
    y = gemm_auto.linear(x, w, b)
    ref = x.float() @ w.float().t() + b.float()
    assert _rel(y, ref) < 1e-2
    dy = torch.randn(1024, 3072, generator=g).to("cuda", torch.bfloat16)
    out = torch.full((3072, 1024), float("nan"), device="cuda")
    gemm_auto.wgrad(dy, x, out)
    assert _rel(out, dy.float().t() @ x.float()) < 1e-2
    rows = gemm_auto.choices()
    assert {r["op"] for r in rows} == {"linear", "wgrad"}
    for r in rows:
        assert r["impl"] in ("hip", "lib", "pp")
        assert r["hip_ms"] > 0 and r["lib_ms"] > 0
        assert r[f"{r['impl']}_ms"] == min(v for k, v in r.items() if k.endswith("_ms"))
    # decided once: a second call neither re-times nor changes the choice
    before = dict(gemm_auto._choice)
    y2 = gemm_auto.linear(x, w, b)
    assert gemm_auto._choice == before and _rel(y2, ref) < 1e-2
