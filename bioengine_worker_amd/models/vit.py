"""DINOv2-compatible Vision Transformer (ViT-S/B/L/g /14) and its HIP inference engine.

The cell-image-search app embeds nucleus crops with DINOv2 ViT-B/14 (reference
``apps/cell-image-search/embedder.py:23-99``: torch.hub ``dinov2_vitb14``, fp16, batch 64, CLS token,
L2-normalised).  Here:

* :class:`ViT` — a plain PyTorch module whose parameter names match the public DINOv2 checkpoints
  (``patch_embed.proj``, ``cls_token``, ``pos_embed``, ``blocks.{i}.norm1/attn.qkv/attn.proj/ls1.gamma/
  norm2/mlp.fc1/mlp.fc2/ls2.gamma``, ``norm``) so a ``dinov2_vitb14_pretrain.pth`` state dict loads
  with ``load_state_dict`` (``torch.load(..., weights_only=True)``).  Used as the fp32 reference and
  for training.
* :class:`ViTEngine` — the MI355X inference path: bf16 weights resident on the GPU, patch
  embedding as one GEMM over a reshaped (not unfolded) image, hipBLASLt GEMMs for qkv/proj/MLP,
  the fused flash-attention kernel reading q/k/v straight out of the packed qkv GEMM output,
  LayerScale+residual fused into the next LayerNorm, bias+GELU fused into one pass.
  ``precision="fp8"`` runs qkv/proj/fc1/fc2 as e4m3 GEMMs on the block-scaled MFMA
  (``ops/fp8.py``: per-channel weight scales, per-token activation scales, bias/GELU in the epilogue).

Offline there are no pretrained weights: ``ViT(...).randomize_(seed)`` gives DINOv2-style init
(trunc-normal 0.02, LayerScale 1e-5 → we use 1.0 for a non-degenerate random network).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.fp8 import Fp8Linear, add_layernorm_fp8, add_layernorm_mx, quantize_rows
from ..ops.transformer import add_layernorm, attention_ref, bias_gelu_, flash_attention, flash_attention_mx


@dataclass
class ViTConfig:
    embed_dim: int = 768
    depth: int = 12
    num_heads: int = 12
    mlp_ratio: float = 4.0
    patch_size: int = 14
    img_size: int = 518          # DINOv2 position grid: 518 / 14 = 37 x 37
    layerscale: bool = True
    eps: float = 1e-6

    @staticmethod
    def dinov2(name: str = "vitb14") -> "ViTConfig":
        table = {"vits14": (384, 12, 6), "vitb14": (768, 12, 12), "vitl14": (1024, 24, 16), "vitg14": (1536, 40, 24)}
        d, L, h = table[name]
        return ViTConfig(embed_dim=d, depth=L, num_heads=h)


class _Attn(nn.Module):
    def __init__(self, dim, heads):
        super().__init__()
        self.num_heads = heads
        self.qkv = nn.Linear(dim, 3 * dim, bias=True)
        self.proj = nn.Linear(dim, dim, bias=True)


class _Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)


class _LayerScale(nn.Module):
    def __init__(self, dim, init=1e-5):
        super().__init__()
        self.gamma = nn.Parameter(torch.full((dim,), init))


class _Block(nn.Module):
    def __init__(self, cfg: ViTConfig):
        super().__init__()
        d = cfg.embed_dim
        self.norm1 = nn.LayerNorm(d, eps=cfg.eps)
        self.attn = _Attn(d, cfg.num_heads)
        self.ls1 = _LayerScale(d) if cfg.layerscale else nn.Identity()
        self.norm2 = nn.LayerNorm(d, eps=cfg.eps)
        self.mlp = _Mlp(d, int(d * cfg.mlp_ratio))
        self.ls2 = _LayerScale(d) if cfg.layerscale else nn.Identity()

    def forward(self, x):
        B, N, C = x.shape
        H = self.attn.num_heads
        qkv = self.attn.qkv(self.norm1(x)).reshape(B, N, 3, H, C // H)
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        if q.dtype == torch.bfloat16:
            a = flash_attention(q, k, v).reshape(B, N, C)
        else:  # fp32 reference path
            a = attention_ref(q, k, v, 1.0 / math.sqrt(C // H)).to(q.dtype).reshape(B, N, C)
        y = self.attn.proj(a)
        x = x + (self.ls1.gamma * y if isinstance(self.ls1, _LayerScale) else y)
        m = self.mlp.fc2(F.gelu(self.mlp.fc1(self.norm2(x))))
        return x + (self.ls2.gamma * m if isinstance(self.ls2, _LayerScale) else m)


class _PatchEmbed(nn.Module):
    def __init__(self, cfg: ViTConfig, in_chans=3):
        super().__init__()
        self.proj = nn.Conv2d(in_chans, cfg.embed_dim, cfg.patch_size, cfg.patch_size)


class ViT(nn.Module):
    def __init__(self, cfg: ViTConfig | None = None):
        super().__init__()
        self.cfg = cfg = cfg or ViTConfig()
        self.patch_embed = _PatchEmbed(cfg)
        g = cfg.img_size // cfg.patch_size
        self.cls_token = nn.Parameter(torch.zeros(1, 1, cfg.embed_dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, 1 + g * g, cfg.embed_dim))
        self.blocks = nn.ModuleList([_Block(cfg) for _ in range(cfg.depth)])
        self.norm = nn.LayerNorm(cfg.embed_dim, eps=cfg.eps)

    @torch.no_grad()
    def randomize_(self, seed: int = 0, layerscale: float = 1.0) -> "ViT":
        gen = torch.Generator().manual_seed(seed)
        for name, p in self.named_parameters():
            if name.endswith("gamma"):
                p.fill_(layerscale)
            elif "norm" in name:
                p.fill_(1.0 if name.endswith("weight") else 0.0)
            elif name.endswith("bias"):
                p.zero_()
            else:
                p.copy_(torch.randn(p.shape, generator=gen).clamp_(-2, 2) * 0.02)
        return self

    def interpolate_pos(self, gh: int, gw: int) -> torch.Tensor:
        """DINOv2 bicubic interpolation of the patch position grid to (gh, gw); CLS position kept."""
        pe = self.pos_embed
        M = int(math.sqrt(pe.shape[1] - 1))
        if gh == M and gw == M:
            return pe
        patch = pe[:, 1:].reshape(1, M, M, -1).permute(0, 3, 1, 2).float()
        patch = F.interpolate(patch, size=(gh, gw), mode="bicubic", align_corners=False)
        patch = patch.permute(0, 2, 3, 1).reshape(1, gh * gw, -1)
        return torch.cat([pe[:, :1].float(), patch], 1).to(pe.dtype)

    def forward_features(self, x: torch.Tensor) -> torch.Tensor:
        B, _, Hh, Ww = x.shape
        p = self.cfg.patch_size
        t = self.patch_embed.proj(x).flatten(2).transpose(1, 2)
        t = torch.cat([self.cls_token.expand(B, -1, -1).to(t.dtype), t], 1)
        t = t + self.interpolate_pos(Hh // p, Ww // p).to(t.dtype)
        for blk in self.blocks:
            t = blk(t)
        return self.norm(t)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """CLS embedding (the torch.hub DINOv2 ``model(x)`` output)."""
        return self.forward_features(x)[:, 0]


class ViTEngine:
    """bf16 HIP inference engine for a :class:`ViT` (see module docstring)."""

    def __init__(self, net: ViT, device, img_size: int = 224, precision: str = "bf16", fp8_gemm: str = "hip"):
        if precision not in ("bf16", "fp8"):
            raise ValueError(f"precision must be 'bf16' or 'fp8', got {precision!r}")
        self.precision = precision
        self.device = torch.device(device)
        self.cfg = cfg = net.cfg
        self.p = cfg.patch_size
        self.g = img_size // cfg.patch_size
        self.img_size = img_size
        bf = lambda t: t.detach().to(self.device, torch.bfloat16).contiguous()
        f32 = lambda t: t.detach().to(self.device, torch.float32).contiguous()
        w = net.patch_embed.proj.weight  # [D, 3, p, p]
        self.pe_w = bf(w.reshape(w.shape[0], -1))
        self.pe_b = bf(net.patch_embed.proj.bias)
        with torch.no_grad():
            pos = net.interpolate_pos(self.g, self.g)[0]
            self.cls_pos = bf(net.cls_token[0, 0] + pos[0])
            self.patch_pos = bf(pos[1:])
        self.blocks = []
        for blk in net.blocks:
            ls = lambda m, d=cfg.embed_dim: f32(m.gamma) if isinstance(m, _LayerScale) else torch.ones(d, device=self.device)
            self.blocks.append(dict(
                n1w=f32(blk.norm1.weight), n1b=f32(blk.norm1.bias), qkv_w=bf(blk.attn.qkv.weight),
                qkv_b=bf(blk.attn.qkv.bias), proj_w=bf(blk.attn.proj.weight), proj_b=bf(blk.attn.proj.bias),
                g1=ls(blk.ls1), n2w=f32(blk.norm2.weight), n2b=f32(blk.norm2.bias),
                fc1_w=bf(blk.mlp.fc1.weight), fc1_b=f32(blk.mlp.fc1.bias), fc2_w=bf(blk.mlp.fc2.weight),
                fc2_b=bf(blk.mlp.fc2.bias), g2=ls(blk.ls2)))
        self.nw, self.nb = f32(net.norm.weight), f32(net.norm.bias)
        if precision == "fp8":
            # e4m3 weights with per-output-channel scales; the bf16 copies are dropped.  Every
            # projection, qkv included, runs on the HIP block-scaled MX-fp8 GEMM by default: qkv reads
            # the MX-fp8 (E8M0 scale per 32 channels) that the fused add+LayerNorm+quantise kernel
            # writes.  Round 5 measured 16,300 img/s against 16,449 for hipBLASLt _scaled_mm on
            # per-token e4m3 (within 1 %), cosine 0.993 vs bf16 (profiles/r05/vit/vit_qkv_mx_ab_s23.jsonl).
            # BE_VIT_QKV_GEMM=lib selects the hipBLASLt arm.  Embeddings from the two arms differ at
            # the quantisation level, so a search index ingested before round 5 (qkv on hipBLASLt)
            # carries slightly different vectors than one ingested now; re-ingest, or pin the arm
            # the index was built with.
            qkv_gemm = os.environ.get("BE_VIT_QKV_GEMM", fp8_gemm)
            for b in self.blocks:
                for name in ("qkv", "proj", "fc1", "fc2"):
                    b[name + "_q"] = Fp8Linear(b.pop(name + "_w"), b.pop(name + "_b"),
                                               gemm=qkv_gemm if name == "qkv" else fp8_gemm)

    def patchify(self, x: torch.Tensor) -> torch.Tensor:
        """[B, C, H, W] -> [B, gh*gw, C*p*p] in conv-weight order (c, ky, kx) — a reshape + one copy."""
        B, C, H, W = x.shape
        p = self.p
        return (x.reshape(B, C, H // p, p, W // p, p).permute(0, 2, 4, 1, 3, 5)
                .reshape(B, (H // p) * (W // p), C * p * p))

    @torch.no_grad()
    def features(self, x: torch.Tensor) -> torch.Tensor:
        """x: [B, 3, S, S] float (ImageNet-normalised) -> final-norm tokens [B, 1 + g*g, D] bf16."""
        cfg = self.cfg
        B = x.shape[0]
        D, Hh = cfg.embed_dim, cfg.num_heads
        x = x.to(self.device, torch.bfloat16)
        tok = F.linear(self.patchify(x), self.pe_w, self.pe_b) + self.patch_pos  # [B, g*g, D]
        N = tok.shape[1] + 1
        t = torch.empty(B, N, D, device=self.device, dtype=torch.bfloat16)
        t[:, 0] = self.cls_pos
        t[:, 1:] = tok
        blocks = self.blocks
        fp8 = self.precision == "fp8"
        if fp8:
            return self._blocks_fp8(t, B, N)
        h = add_layernorm(t, None, None, blocks[0]["n1w"], blocks[0]["n1b"], cfg.eps)
        for i, b in enumerate(blocks):
            qkv = F.linear(h, b["qkv_w"], b["qkv_b"]).view(B, N, 3, Hh, D // Hh)
            a = flash_attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]).view(B, N, D)
            y = F.linear(a, b["proj_w"], b["proj_b"])
            h2 = add_layernorm(t, y, b["g1"], b["n2w"], b["n2b"], cfg.eps)
            m = bias_gelu_(F.linear(h2, b["fc1_w"]), b["fc1_b"])
            m = F.linear(m, b["fc2_w"], b["fc2_b"])
            if i + 1 < len(blocks):
                h = add_layernorm(t, m, b["g2"], blocks[i + 1]["n1w"], blocks[i + 1]["n1b"], cfg.eps)
            else:
                h = add_layernorm(t, m, b["g2"], self.nw, self.nb, cfg.eps)
        return h

    def _blocks_fp8(self, t: torch.Tensor, B: int, N: int) -> torch.Tensor:
        """fp8 encoder blocks: LayerNorms emit e4m3 + per-token scales straight into the qkv / fc1
        GEMMs; the attention output is re-quantised per token for proj (hipBLASLt) or leaves the
        attention kernel as MX-fp8 for proj's block-scaled MFMA (HIP GEMM).  fc1 -> fc2: with the HIP GEMM
        the GELU and an MX-fp8 quantisation (E8M0 scale per 32 outputs) run in fc1's epilogue and the
        block scales go into fc2's MFMA scale operand; with hipBLASLt, GELU + per-token quantisation
        run as one pass between the two library GEMMs."""
        cfg, blocks = self.cfg, self.blocks
        D, Hh = cfg.embed_dim, cfg.num_heads
        # qkv on the block-scaled HIP GEMM reads MX-fp8 (E8M0 per 32 channels) straight from the LayerNorm;
        # on hipBLASLt it reads per-token-scaled e4m3
        ln_q = add_layernorm_mx if blocks[0]["qkv_q"].gemm == "hip" else add_layernorm_fp8
        hq = ln_q(t, None, None, blocks[0]["n1w"], blocks[0]["n1b"], cfg.eps)
        for i, b in enumerate(blocks):
            qkv = b["qkv_q"](hq).view(B, N, 3, Hh, D // Hh)
            if b["proj_q"].gemm == "hip":  # attention epilogue -> MX-fp8 -> proj's MFMA scale operand
                aq, as_ = flash_attention_mx(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2])
                y = b["proj_q"]((aq.view(B * N, D), as_)).view(B, N, D)
            else:
                a = flash_attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]).view(B, N, D)
                y = b["proj_q"](a)
            h2q = add_layernorm_fp8(t, y, b["g1"], b["n2w"], b["n2b"], cfg.eps)
            if b["fc1_q"].gemm == "hip":  # GELU + MX-fp8 in fc1's epilogue, block scales into fc2's MFMA
                m = b["fc2_q"](b["fc1_q"](h2q, mx_out=True))
            else:
                m = b["fc2_q"](quantize_rows(b["fc1_q"](h2q), gelu=True))
            if i + 1 < len(blocks):
                hq = ln_q(t, m, b["g2"], blocks[i + 1]["n1w"], blocks[i + 1]["n1b"], cfg.eps)
        return add_layernorm(t, m, blocks[-1]["g2"], self.nw, self.nb, cfg.eps)

    @torch.no_grad()
    def embed(self, x: torch.Tensor, normalize: bool = True) -> torch.Tensor:
        """CLS embeddings [B, D] fp32 (L2-normalised like embedder.py:89-92)."""
        cls = self.features(x)[:, 0].float()
        return F.normalize(cls, dim=1, eps=1e-9) if normalize else cls

    #: batch buckets of :meth:`embed_graphed` (a request batch is padded up to the next one)
    GRAPH_BUCKETS = (1, 2, 4, 8, 16, 32, 64)
    #: capture attempts per bucket before it stays eager for the process
    GRAPH_MAX_TRIES = 3

    @torch.no_grad()
    def embed_graphed(self, x: torch.Tensor) -> torch.Tensor:
        """:meth:`embed` replayed from a HIP graph per batch bucket: a serving batch of a few
        queries is ~150 kernel launches of microseconds each, so launches, not the GPU, set its
        latency.  The batch is zero-padded to the bucket; the graph (captured on first use of the
        bucket, after one eager warm-up) reads a static input buffer."""
        B = x.shape[0]
        if not x.is_cuda or B > self.GRAPH_BUCKETS[-1]:
            return self.embed(x)
        bucket = next(b for b in self.GRAPH_BUCKETS if b >= B)
        graphs = self.__dict__.setdefault("_graphs", {})
        key = (bucket, tuple(x.shape[1:]), x.dtype)
        ent = graphs.get(key)
        if isinstance(ent, int):  # earlier capture attempts failed
            if ent >= self.GRAPH_MAX_TRIES:
                return self.embed(x)
            ent = None
        if ent is None:
            xs = torch.zeros((bucket,) + tuple(x.shape[1:]), device=x.device, dtype=x.dtype)
            xs[:B] = x
            side = torch.cuda.Stream(x.device)
            side.wait_stream(torch.cuda.current_stream(x.device))
            with torch.cuda.stream(side):
                self.embed(xs)  # lazy state, kernels, allocator
            torch.cuda.current_stream(x.device).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            try:
                # thread_local: another thread's eager work on this device (e.g. the search app's
                # ingestion embedding) neither breaks this capture nor is broken by it
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    out = self.embed(xs)
            except Exception:  # noqa: BLE001 -- counted: a transient failure is retried on later calls
                graphs[key] = int(graphs.get(key) or 0) + 1
                return self.embed(x)
            ent = graphs[key] = (g, xs, out)
        g, xs, out = ent
        xs[:B].copy_(x)
        if B < bucket:
            xs[B:].zero_()
        g.replay()
        return out[:B].clone()
