"""ViT (DINOv2) and Cellpose-SAM: engine paths vs the fp32 module reference (CPU, small configs)."""
import torch

from bioengine_worker_amd.models.cpsam import CPSAM, CPSAMEngine, get_rel_pos
from bioengine_worker_amd.models.vit import ViT, ViTConfig, ViTEngine
from bioengine_worker_amd.ops.transformer import add_layernorm, add_layernorm_ref, attention_ref


def test_vit_engine_matches_module_cpu():
    cfg = ViTConfig(embed_dim=128, depth=2, num_heads=2, img_size=70)
    net = ViT(cfg).randomize_(0).eval()
    x = torch.randn(2, 3, 56, 56)
    ref = net(x)
    eng = ViTEngine(net, "cpu", img_size=56)
    out = eng.embed(x, normalize=False)
    assert out.shape == (2, 128)
    cos = torch.nn.functional.cosine_similarity(out, ref.float(), dim=1)
    assert cos.min() > 0.99, cos


def test_vit_state_dict_names_match_dinov2():
    net = ViT(ViTConfig.dinov2("vitb14"))
    keys = set(net.state_dict())
    for k in ("cls_token", "pos_embed", "patch_embed.proj.weight", "blocks.0.norm1.weight", "blocks.0.attn.qkv.weight",
              "blocks.0.attn.proj.bias", "blocks.0.ls1.gamma", "blocks.11.mlp.fc2.weight", "blocks.11.ls2.gamma",
              "norm.bias"):
        assert k in keys, k
    assert net.pos_embed.shape == (1, 1 + 37 * 37, 768)
    assert sum(p.numel() for p in net.parameters()) > 85e6


def test_cpsam_engine_matches_module_cpu():
    net = CPSAM(dim=128, depth=2, heads=2, ps=8, bsize=64).randomize_(1).eval()
    x = torch.randn(2, 3, 64, 64)
    with torch.no_grad():
        ref, style = net(x)
    assert ref.shape == (2, 3, 64, 64) and style.shape == (2, 256)
    out = CPSAMEngine(net, "cpu")(x)
    err = (out - ref).abs().max() / ref.abs().max()
    assert err < 0.05, err


def test_cpsam_param_names():
    keys = set(CPSAM(dim=128, depth=1, heads=2).state_dict())
    for k in ("encoder.patch_embed.proj.weight", "encoder.pos_embed", "encoder.blocks.0.attn.rel_pos_h",
              "encoder.blocks.0.mlp.lin1.weight", "encoder.neck.0.weight", "encoder.neck.1.weight", "out.weight", "W2",
              "diam_mean"):
        assert k in keys, k


def test_rel_pos_resize_and_index():
    rp = torch.arange(27, dtype=torch.float32)[:, None].repeat(1, 4)
    R = get_rel_pos(32, 32, rp)
    assert R.shape == (32, 32, 4)
    assert torch.allclose(R[5, 5], R[0, 0]) and R[31, 0, 0] > R[0, 31, 0]


def test_attention_ref_rel_bias_shapes():
    q = torch.randn(1, 16, 2, 64)
    rh, rw = torch.randn(1, 2, 16, 4), torch.randn(1, 2, 16, 4)
    o = attention_ref(q, q, q, 0.125, rh, rw)
    assert o.shape == q.shape


def test_add_layernorm_cpu_inplace():
    x = torch.randn(5, 64).bfloat16()
    y = torch.randn(5, 64).bfloat16()
    g, w, b = torch.rand(64), torch.rand(64), torch.rand(64)
    xn, ref = add_layernorm_ref(x, y, g, w, b)
    x2 = x.clone()
    out = add_layernorm(x2, y, g, w, b)
    assert torch.equal(x2, xn) and torch.allclose(out.float(), ref.float())
