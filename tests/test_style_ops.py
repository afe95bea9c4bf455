"""Cellpose style vector + folded decoder style shifts: fused HIP kernel vs plain fp32 torch."""
import pytest
import torch

from bioengine_worker_amd.ops import style as styleops


def _ref(x, w, b, s, t, style_on):
    v = x.float().mean(dim=(1, 2))
    st = v / torch.sqrt((v * v).sum(1, keepdim=True))
    f = (st if style_on else torch.zeros_like(st)) @ w.t() + b
    return st, f * s + t


def test_style_and_shifts_cpu_matches_reference():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, 7, 5, 32, generator=g).bfloat16()
    w, b, s, t = torch.randn(96, 32, generator=g), torch.randn(96, generator=g), torch.randn(96, generator=g), torch.randn(96, generator=g)
    st, sh = styleops.style_and_shifts(x, w, b, s, t)
    rst, rsh = _ref(x, w, b, s, t, True)
    assert torch.allclose(st, rst, atol=1e-5) and torch.allclose(sh, rsh, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("style_on", [True, False])
@pytest.mark.parametrize("N,C,J", [(1, 256, 1440), (5, 256, 1440), (2, 64, 100)])
def test_style_and_shifts_gpu_matches_fp32(gpu, style_on, N, C, J):
    g = torch.Generator().manual_seed(N * C + J)
    x = torch.randn(N, 28, 28, C, generator=g).bfloat16()
    w, b, s, t = (torch.randn(J, C, generator=g) * 0.1, torch.randn(J, generator=g), torch.randn(J, generator=g),
                  torch.randn(J, generator=g))
    st, sh = styleops.style_and_shifts(*(a.to(gpu) for a in (x, w, b, s, t)), style_on=style_on)
    rst, rsh = _ref(x, w, b, s, t, style_on)
    assert (st.cpu() - rst).abs().max().item() < 1e-5
    assert (sh.cpu() - rsh).abs().max().item() < 1e-4 * max(1.0, rsh.abs().max().item())
