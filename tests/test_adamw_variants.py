"""Both fused AdamW kernels (csrc/kernels/adamw.hip: one float4 per lane per iteration, and two with
streaming accesses) against the PyTorch reference update (the CPU path of ops/train_ops.py, which
follows torch.optim.AdamW), on flat buffers with ragged tails and the bf16 mirror."""
import pytest
import torch

from bioengine_worker_amd.ops import _native, train_ops


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("n", [1, 7, 4096, 4096 * 3 + 5, 1_000_003, 2048 * 256 * 4 * 2 + 12])
def test_adamw_variants_match_reference(variant, n):
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(n)
    p0, gr, m0, v0 = (torch.randn(n, generator=g) for _ in range(4))
    v0 = v0.abs()
    ref = [t.clone() for t in (p0, gr, m0, v0)]
    train_ops.adamw_flat_(ref[0], ref[1], ref[2], ref[3], lr=1e-3, step=3, weight_decay=1e-2, grad_scale=0.5)
    _native.call("be_adamw_set_variant", variant)
    try:
        p, gd, m, v = (t.to(dev) for t in (p0, gr, m0, v0))
        mirror = torch.empty(n, device=dev, dtype=torch.bfloat16)
        train_ops.adamw_flat_(p, gd, m, v, lr=1e-3, step=3, weight_decay=1e-2, grad_scale=0.5, p_bf16=mirror)
        torch.cuda.synchronize()
    finally:
        _native.call("be_adamw_set_variant", 0)
    for got, want in ((p, ref[0]), (m, ref[2]), (v, ref[3])):
        assert torch.allclose(got.cpu(), want, rtol=1e-5, atol=1e-6), (got.cpu() - want).abs().max()
    assert torch.equal(mirror.cpu(), p.cpu().to(torch.bfloat16))  # the mirror is the kernel's own p, rounded
