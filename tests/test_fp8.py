"""FP8 (e4m3fn) linear path: the HIP block-scaled-MFMA GEMM and per-token quantiser against plain
PyTorch fp32 references, and the fp8 ViT engine against the fp32 DINOv2 module."""
import pytest
import torch

from bioengine_worker_amd.models.vit import ViT, ViTConfig, ViTEngine
from bioengine_worker_amd.ops.fp8 import (FP8_DTYPE, Fp8Linear, add_layernorm_fp8, linear_fp8, linear_fp8_ref,
                                          quantize_rows, quantize_rows_ref)
from bioengine_worker_amd.ops.transformer import add_layernorm_ref


def test_quantize_rows_ref_roundtrip():
    x = torch.randn(5, 256) * torch.logspace(-3, 2, 5)[:, None]
    q, s = quantize_rows_ref(x)
    assert q.dtype == FP8_DTYPE and s.shape == (5,)
    assert q.float().abs().amax(1).sub(448).abs().max() < 1e-3  # every row uses the full e4m3 range
    rel = ((q.float() * s[:, None] - x).abs() / x.abs().amax(1, keepdim=True)).max()
    assert rel < 2 ** -4  # 3 mantissa bits


def test_fp8_linear_cpu_close_to_fp32():
    g = torch.Generator().manual_seed(0)
    w = torch.randn(96, 256, generator=g) * 0.05
    b = torch.randn(96, generator=g)
    x = torch.randn(33, 256, generator=g).bfloat16()
    lin = Fp8Linear(w, b)
    y = lin(x, gelu=True).float()
    ref = torch.nn.functional.gelu(x.float() @ w.t() + b)
    err = (y - ref).abs().max() / ref.abs().max()
    assert err < 0.05, err


@pytest.mark.parametrize("fp8_gemm", ["hipblaslt", "hip"])
def test_vit_engine_fp8_cpu_embedding_close(fp8_gemm):
    cfg = ViTConfig(embed_dim=128, depth=2, num_heads=2, img_size=70)
    net = ViT(cfg).randomize_(0).eval()
    x = torch.randn(2, 3, 56, 56)
    ref = net(x)
    out = ViTEngine(net, "cpu", img_size=56, precision="fp8", fp8_gemm=fp8_gemm).embed(x, normalize=False)
    cos = torch.nn.functional.cosine_similarity(out, ref.float(), dim=1)
    assert cos.min() > 0.98, cos
    with pytest.raises(ValueError):
        ViTEngine(net, "cpu", img_size=56, precision="fp4")


@pytest.mark.gpu
@pytest.mark.parametrize("K", [128, 768, 3072])
@pytest.mark.parametrize("gelu", [False, True])
def test_quantize_rows_hip_matches_reference(gpu, K, gelu):
    x = (torch.randn(77, K) * torch.rand(77, 1) * 10).bfloat16()
    qr, sr = quantize_rows_ref(x, gelu)
    q, s = quantize_rows(x.to(gpu), gelu)
    torch.testing.assert_close(s.cpu(), sr, rtol=1e-6, atol=0)
    # x * (448/amax) vs x / (amax/448): at most one e4m3 step apart, on a handful of elements
    d = (q.cpu().float() - qr.float()).abs()
    step = qr.float().abs().clamp_min(2 ** -6) * 2 ** -3
    assert (d <= step + 1e-6).all()
    assert (d > 0).float().mean() < 0.01


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(128, 128, 128), (16448, 2304, 768), (300, 768, 3072), (1, 3072, 768),
                                   (129, 260, 256)])
@pytest.mark.parametrize("gelu", [False, True])
def test_gemm_fp8_matches_reference(gpu, M, N, K, gelu):
    g = torch.Generator().manual_seed(M + N + K)
    # asymmetric operands (cdna_hip_programming.md §3: catches transposed C-writes)
    x = (torch.randn(M, K, generator=g) + torch.arange(K) / K).bfloat16()
    w = torch.randn(N, K, generator=g) * 0.03 + torch.arange(N)[:, None] / (10 * N)
    bias = torch.randn(N, generator=g)
    lin = Fp8Linear(w, bias)
    xq, sx = quantize_rows_ref(x)
    ref = linear_fp8_ref(xq, sx, lin.wq, lin.sw, lin.bias, gelu).float()
    lin.to(gpu)
    y = linear_fp8(xq.to(gpu), sx.to(gpu), lin.wq, lin.sw, lin.bias, gelu).float().cpu()
    err = (y - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize("tile_cfg", [1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("M,N,K", [(1000, 640, 384), (257, 256, 128), (300, 516, 256), (520, 768, 3072),
                                   (16448, 2304, 768)])
def test_gemm_fp8_tile_configs(gpu, tile_cfg, M, N, K):
    g = torch.Generator().manual_seed(tile_cfg)
    x = (torch.randn(M, K, generator=g) + torch.arange(K) / K).bfloat16()
    w = torch.randn(N, K, generator=g) * 0.03 + torch.arange(N)[:, None] / (10 * N)
    lin = Fp8Linear(w, torch.randn(N, generator=g))
    xq, sx = quantize_rows_ref(x)
    ref = linear_fp8_ref(xq, sx, lin.wq, lin.sw, lin.bias).float()
    lin.to(gpu)
    y = linear_fp8(xq.to(gpu), sx.to(gpu), lin.wq, lin.sw, lin.bias, tile_cfg=tile_cfg).float().cpu()
    assert (y - ref).abs().max().item() <= 1e-2 * ref.abs().max().item() + 1e-2
    if M == 300:  # GELU epilogue on a ragged shape with two K-tiles
        refg = linear_fp8_ref(xq, sx, lin.wq.cpu(), lin.sw.cpu(), lin.bias.cpu(), gelu=True).float()
        yg = linear_fp8(xq.to(gpu), sx.to(gpu), lin.wq, lin.sw, lin.bias, True, tile_cfg=tile_cfg).float().cpu()
        assert (yg - refg).abs().max().item() <= 1e-2 * refg.abs().max().item() + 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("C", [768, 1024])
def test_add_layernorm_fp8_matches_reference(gpu, C):
    g = torch.Generator().manual_seed(C)
    x = torch.randn(300, C, generator=g).bfloat16()
    y = torch.randn(300, C, generator=g).bfloat16()
    gamma, w, b = (torch.randn(C, generator=g) for _ in range(3))
    xn_ref, out_ref = add_layernorm_ref(x, y, gamma, w, b, 1e-6)
    xg = x.to(gpu)
    q, s = add_layernorm_fp8(xg, y.to(gpu), gamma.to(gpu), w.to(gpu), b.to(gpu), 1e-6)
    torch.testing.assert_close(xg.cpu(), xn_ref)  # residual stream updated in place
    deq = q.cpu().float() * s.cpu()[:, None]
    scale = out_ref.float().abs().amax(1, keepdim=True)
    assert ((deq - out_ref.float()).abs() / scale).max() < 2 ** -4


@pytest.mark.gpu
def test_gemm_fp8_identity_exact(gpu):
    # A = I with an asymmetric B and unit scales: every output element is one exact product
    K, N = 256, 64
    xq = torch.eye(K)[:100].to(FP8_DTYPE)
    w = torch.arange(N * K).reshape(N, K).remainder(13).float() - 6
    ones_m, ones_n = torch.ones(100), torch.ones(N)
    y = linear_fp8(xq.to(gpu), ones_m.to(gpu), w.to(FP8_DTYPE).to(gpu), ones_n.to(gpu)).float().cpu()
    torch.testing.assert_close(y, w.t()[:100], rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("gemm", ["hip", "hipblaslt"])
def test_fp8_linear_backends_agree(gpu, gemm):
    g = torch.Generator().manual_seed(3)
    w, b = torch.randn(768, 768, generator=g) * 0.03, torch.randn(768, generator=g)
    x = torch.randn(2, 257, 768, generator=g).bfloat16()
    ref = Fp8Linear(w, b)(x).float()  # CPU reference
    y = Fp8Linear(w, b, gemm=gemm).to(gpu)(x.to(gpu)).float().cpu()
    assert y.shape == (2, 257, 768)
    assert (y - ref).abs().max().item() <= 1e-2 * ref.abs().max().item() + 2e-2


@pytest.mark.gpu
def test_vit_engine_fp8_gpu_embedding_close(gpu):
    net = ViT(ViTConfig.dinov2("vitb14")).randomize_(0).eval()
    x = torch.randn(4, 3, 224, 224)
    ref = ViTEngine(net, gpu).embed(x.to(gpu))
    out = ViTEngine(net, gpu, precision="fp8").embed(x.to(gpu))
    cos = torch.nn.functional.cosine_similarity(out, ref, dim=1)
    assert cos.min() > 0.99, cos


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(16448, 3072, 768), (300, 768, 3072), (129, 256, 256)])
def test_gemm_fp8_mx_epilogue_and_block_scaled_input(gpu, M, N, K):
    """fc1 -> fc2 with MX-fp8 in between (be_gemm_fp8_mx): the GELU + E8M0-block quantisation epilogue
    vs the PyTorch reference of the same math, then the block-scaled-input GEMM vs its reference on the
    SAME quantised operands (scales into the MFMA scale operand)."""
    from bioengine_worker_amd.ops.fp8 import linear_fp8_mx, mx_dequant_ref, mx_quantize_ref

    g = torch.Generator().manual_seed(M + N)
    x = (torch.randn(M, K, generator=g) + torch.arange(K) / K).bfloat16()
    w1 = torch.randn(N, K, generator=g) * K ** -0.5 + torch.arange(N)[:, None] / (10 * N)
    w2 = torch.randn(K, N, generator=g) * N ** -0.5
    l1, l2 = Fp8Linear(w1, torch.randn(N, generator=g) * 0.1), Fp8Linear(w2, torch.randn(K, generator=g) * 0.1)
    xq, sx = quantize_rows_ref(x)
    pre = (xq.float() * sx[:, None]) @ l1.wq.float().t() * l1.sw + l1.bias
    l1.to(gpu)
    l2.to(gpu)
    yq, ys = linear_fp8_mx((xq.to(gpu), sx.to(gpu)), l1.wq, l1.sw, l1.bias, gelu=True, mx_out=True)
    yq, ys = yq.cpu(), ys.cpu()
    assert ys.dtype == torch.uint8 and ys.shape == (M, N // 32)
    qr, sr = mx_quantize_ref(pre, gelu=True)
    # scales: identical except where a block's amax sits on a power-of-two boundary (fp32 order)
    assert (ys.int() - sr.int()).abs().max() <= 1 and (ys != sr).float().mean() < 1e-3
    deq, deq_r = mx_dequant_ref(yq, ys), mx_dequant_ref(qr, sr)
    ref1 = torch.nn.functional.gelu(pre)
    assert ((deq - ref1).norm() / ref1.norm()).item() < 0.05
    assert ((deq - deq_r).norm() / deq_r.norm()).item() < 0.02
    # block-scaled input GEMM on the kernel's own MX output
    y2 = linear_fp8_mx((yq.to(gpu), ys.to(gpu)), l2.wq, l2.sw, l2.bias).float().cpu()
    ref2 = deq @ l2.wq.cpu().float().t() * l2.sw.cpu() + l2.bias.cpu()
    err = (y2 - ref2).abs().max().item()
    assert err <= 1e-2 * ref2.abs().max().item() + 1e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize("qkv_gemm", ["hipblaslt", "hip"])
def test_vit_engine_fp8_hip_mx_embedding_close(gpu, qkv_gemm, monkeypatch):
    """The HIP fp8 path (MX-fp8 between fc1 and fc2; qkv on either GEMM) against the bf16 engine,
    end to end."""
    monkeypatch.setenv("BE_VIT_QKV_GEMM", qkv_gemm)
    net = ViT(ViTConfig.dinov2("vitb14")).randomize_(0).eval()
    x = torch.randn(4, 3, 224, 224)
    ref = ViTEngine(net, gpu).embed(x.to(gpu))
    out = ViTEngine(net, gpu, precision="fp8", fp8_gemm="hip").embed(x.to(gpu))
    cos = torch.nn.functional.cosine_similarity(out, ref, dim=1)
    assert cos.min() > 0.99, cos


@pytest.mark.gpu
@pytest.mark.parametrize("B,N,H", [(2, 257, 12), (1, 100, 2)])
def test_attention_mx_fp8_output_matches_reference(gpu, B, N, H):
    """Attention epilogue -> MX-fp8 (E8M0 per 32 head dims) vs the fp32 attention quantised by the
    PyTorch MX reference: the same block scales (up to a rounding-boundary flip) and dequantised
    values within one e4m3 step of the block."""
    from bioengine_worker_amd.ops.fp8 import mx_dequant_ref, mx_quantize_ref
    from bioengine_worker_amd.ops.transformer import attention_ref, flash_attention_mx

    g = torch.Generator().manual_seed(7)
    qkv = (torch.randn(B, N, 3, H, 64, generator=g) * 1.5).to(gpu).bfloat16()
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    oq, os_ = flash_attention_mx(q, k, v)
    torch.cuda.synchronize()
    ref = attention_ref(q.float(), k.float(), v.float(), 64 ** -0.5).reshape(B * N, H * 64)
    rq, rs = mx_quantize_ref(ref)
    assert os_.shape == rs.shape and oq.shape == (B, N, H * 64)
    assert (os_.cpu().int() - rs.cpu().int()).abs().max().item() <= 1
    assert (os_.cpu() == rs.cpu()).float().mean().item() > 0.99
    deq = mx_dequant_ref(oq.reshape(B * N, H * 64), os_).cpu()
    step = torch.exp2(os_.cpu().float() - 127.0).repeat_interleave(32, dim=1) * 32  # e4m3 step at the block max
    assert ((deq - ref.cpu()).abs() <= step).all()


@pytest.mark.gpu
@pytest.mark.parametrize("C", [768, 1024])
def test_add_layernorm_mx_matches_reference(gpu, C):
    """LayerNorm -> MX-fp8 (E8M0 per 32 channels): the scale bytes equal mx_quantize_ref's on the fp32
    LN output, and the dequantised values are within e4m3 rounding of it."""
    from bioengine_worker_amd.ops.fp8 import add_layernorm_mx, mx_dequant_ref, mx_quantize_ref

    g = torch.Generator().manual_seed(C + 1)
    x = torch.randn(300, C, generator=g).bfloat16()
    y = torch.randn(300, C, generator=g).bfloat16()
    gamma, w, b = (torch.randn(C, generator=g) for _ in range(3))
    xn_ref, out_ref = add_layernorm_ref(x, y, gamma, w, b, 1e-6)
    xg = x.to(gpu)
    q, s = add_layernorm_mx(xg, y.to(gpu), gamma.to(gpu), w.to(gpu), b.to(gpu), 1e-6)
    torch.testing.assert_close(xg.cpu(), xn_ref)
    _, s_ref = mx_quantize_ref(out_ref.float())
    # the reference normalises in bf16 before quantising; allow a one-step exponent difference at ties
    assert (s.cpu().int() - s_ref.int()).abs().max() <= 1
    deq = mx_dequant_ref(q.cpu(), s.cpu())
    blk = out_ref.float().reshape(300, C // 32, 32).abs().amax(-1, keepdim=True).clamp_min(1e-6)
    err = ((deq - out_ref.float()).reshape(300, C // 32, 32).abs() / blk).max()
    assert err < 2 ** -3, err
