"""Numerics of the ViT HIP kernels (flash attention, fused residual+LayerNorm, bias+GELU) against
plain PyTorch fp32 references, and the ViT / Cellpose-SAM engines against their fp32 modules."""
import pytest
import torch

from bioengine_worker_amd.ops.transformer import (add_layernorm, add_layernorm_ref, attention_ref, bias_gelu_,
                                                  flash_attention)


def _packed_qkv(B, N, H, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    qkv = torch.randn(B, N, 3, H, 64, generator=g).bfloat16().to(dev)
    return qkv, qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]


@pytest.mark.gpu
@pytest.mark.parametrize("B,N,H", [(2, 257, 12), (1, 1024, 4), (3, 77, 2), (1, 64, 1), (2, 33, 3)])
def test_flash_attention_matches_reference(gpu, B, N, H):
    _, q, k, v = _packed_qkv(B, N, H, gpu)
    out = flash_attention(q, k, v).float()
    ref = attention_ref(q, k, v, 64 ** -0.5)
    err = (out - ref).abs().max().item()
    assert err < 2e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize("g", [32, 8, 12])
def test_flash_attention_relpos_bias(gpu, g):
    B, H = 2, 3
    N = g * g
    _, q, k, v = _packed_qkv(B, N, H, gpu, seed=1)
    rh = torch.randn(B, H, N, g, device=gpu)
    rw = torch.randn(B, H, N, g, device=gpu)
    out = flash_attention(q, k, v, 0.125, rh, rw).float()
    ref = attention_ref(q, k, v, 0.125, rh, rw)
    assert (out - ref).abs().max().item() < 2e-2


@pytest.mark.gpu
def test_flash_attention_backward_matches_autograd(gpu):
    B, N, H = 1, 80, 2
    _, q, k, v = _packed_qkv(B, N, H, gpu, seed=2)
    rh = torch.randn(B, H, N, 8, device=gpu) * 0.1
    rw = torch.randn(B, H, N, 10, device=gpu) * 0.1
    qs, ks, vs, rhs, rws = (t.detach().clone().requires_grad_(True) for t in (q, k, v, rh, rw))
    out = flash_attention(qs, ks, vs, 0.125, rhs, rws)
    go = torch.randn_like(out.float())
    out.float().backward(go)
    qr, kr, vr, rhr, rwr = (t.detach().float().clone().requires_grad_(True) for t in (q, k, v, rh, rw))
    attention_ref(qr, kr, vr, 0.125, rhr, rwr).backward(go)
    for a, b in ((qs, qr), (ks, kr), (vs, vr), (rhs, rhr), (rws, rwr)):
        assert (a.grad.float() - b.grad).abs().max().item() < 5e-2 * max(1.0, b.grad.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("C", [768, 1024, 256, 1536])
def test_add_layernorm_kernel(gpu, C):
    x = torch.randn(333, C).bfloat16()
    y = torch.randn(333, C).bfloat16()
    g, w, b = torch.rand(C) * 0.5, torch.rand(C) + 0.5, torch.randn(C) * 0.1
    xn, ref = add_layernorm_ref(x, y, g, w, b)
    xd = x.to(gpu)
    out = add_layernorm(xd, y.to(gpu), g.to(gpu), w.to(gpu), b.to(gpu)).cpu()
    assert (xd.cpu().float() - xn.float()).abs().max().item() <= 1e-2
    assert (out.float() - ref.float()).abs().max().item() < 3e-2
    out2 = add_layernorm(x.to(gpu), None, None, w.to(gpu), b.to(gpu)).cpu()
    assert (out2.float() - add_layernorm_ref(x, None, None, w, b)[1].float()).abs().max().item() < 3e-2


@pytest.mark.gpu
def test_bias_gelu_kernel(gpu):
    h = torch.randn(100, 3072).bfloat16()
    b = torch.randn(3072)
    ref = torch.nn.functional.gelu(h.float() + b)
    out = bias_gelu_(h.to(gpu), b.to(gpu)).cpu().float()
    assert (out - ref).abs().max().item() < 3e-2


@pytest.mark.gpu
def test_vit_b14_engine_matches_fp32(gpu):
    from bioengine_worker_amd.models.vit import ViT, ViTConfig, ViTEngine

    net = ViT(ViTConfig.dinov2("vitb14")).randomize_(0).eval()
    x = torch.randn(4, 3, 224, 224)
    with torch.no_grad():
        ref = torch.nn.functional.normalize(net.to(gpu)(x.to(gpu)).float(), dim=1).cpu()
    out = ViTEngine(net, gpu).embed(x).cpu()
    cos = (out * ref).sum(1)
    assert cos.min().item() > 0.98, cos


@pytest.mark.gpu
def test_cpsam_engine_matches_fp32(gpu):
    from bioengine_worker_amd.models.cpsam import CPSAM, CPSAMEngine

    net = CPSAM(dim=256, depth=4, heads=4).randomize_(0).eval().to(gpu)
    x = torch.randn(2, 3, 256, 256, device=gpu)
    with torch.no_grad():
        ref, _ = net(x)
    out = CPSAMEngine(net, gpu)(x)
    rel = ((out - ref).norm() / ref.norm()).item()
    assert rel < 0.05, rel


@pytest.mark.gpu
@pytest.mark.parametrize("gemm", ["mt", "lib", "ltgelu"])
def test_cpsam_engine_vit_l_matches_fp32(gpu, gemm, monkeypatch):
    """The inference engine at the reference's ViT-L/8 shapes (dim 1024, 24 blocks, 16 heads, 1024
    tokens) against the fp32 CPSAM.forward, eager and replayed from its HIP graph; every linear layer
    on the in-house GEMM (default) or the library (A/B)."""
    from bioengine_worker_amd.models.cpsam import CPSAM, CPSAMEngine

    monkeypatch.setattr(CPSAMEngine, "GEMM", gemm)
    net = CPSAM().randomize_(0).eval().to(gpu)
    x = torch.randn(2, 3, 256, 256, device=gpu)
    with torch.no_grad():
        ref, _ = net(x)
    eng = CPSAMEngine(net, gpu)
    out = eng(x)
    rel = ((out - ref).norm() / ref.norm()).item()
    assert rel < 0.05, rel
    g1 = eng.graphed(x)
    g2 = eng.graphed(x * 0.5)  # replay with new input in the static buffer
    assert torch.equal(g1, out)
    rel2 = ((g2 - eng(x * 0.5)).norm() / g2.norm()).item()
    assert rel2 == 0.0, rel2
    # one graph per exact tile count (no padding), least recently used evicted past GRAPH_MAX
    monkeypatch.setattr(CPSAMEngine, "GRAPH_MAX", 2)
    g3 = eng.graphed(x[:1])
    assert torch.equal(g3, eng(x[:1]))
    x3 = torch.randn(3, 3, 256, 256, device=gpu)
    assert torch.equal(eng.graphed(x3), eng(x3))
    assert list(eng._graphs) == [(1, 3, 256, 256), (3, 3, 256, 256)]  # the 2-tile graph was the LRU
