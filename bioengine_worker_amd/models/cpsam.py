"""Cellpose-SAM ("cpsam", cellpose 4) network and its HIP inference engine.

The reference cellpose-finetuning app runs Cellpose-SAM (``Transformer(dtype=bf16)``,
``apps/cellpose-finetuning/main.py:126-127``): a SAM ViT-L image encoder with an
8-pixel patch embedding (256x256 crops -> 32x32 = 1024 tokens, dim 1024, 24 blocks, 16 heads, all
blocks global attention with SAM's decomposed relative-position bias), the SAM neck
(1x1 conv 1024->256, LayerNorm2d, 3x3 conv, LayerNorm2d), a 1x1 readout to 3 x 8 x 8 per patch and
a pixel-shuffle back to 3 x 256 x 256 (dY, dX, cellprob).

* :class:`CPSAM` — PyTorch module with cellpose-4 parameter names (``encoder.patch_embed.proj``,
  ``encoder.pos_embed``, ``encoder.blocks.{i}.{norm1,attn.qkv,attn.proj,attn.rel_pos_h,
  attn.rel_pos_w,norm2,mlp.lin1,mlp.lin2}``, ``encoder.neck.{0..3}``, ``out``, ``W2``,
  ``diam_labels``, ``diam_mean``) so a ``cpsam`` checkpoint loads with ``weights_only=True``.
  Reference path + training (``rdrop`` per-sample stochastic depth as cellpose 4 does).
* :class:`CPSAMEngine` — bf16 inference on the framework's kernels: every linear layer on hipBLASLt
  (default) or the macro-tile MFMA GEMM (``ops/gemm_mt.py``, bias / bias + GELU in its epilogue), the
  flash-attention kernel with the decomposed rel-pos bias fused into the score tile (the 1024x1024
  bias never exists), residual fused into LayerNorm, the neck's 3x3 conv on the NHWC MFMA conv
  kernel, and the readout + pixel shuffle as one GEMM + reshape.  :meth:`CPSAMEngine.graphed`
  replays the whole forward (~170 launches) from one HIP graph per tile count.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

import os

from ..ops.conv import PackedConv, fused_conv2d
from ..ops.transformer import add_layernorm, attention_ref, bias_gelu_, flash_attention
from ..ops.vit_train import relpos_fwd


def get_rel_pos(q_size: int, k_size: int, rel_pos: torch.Tensor) -> torch.Tensor:
    """SAM ``get_rel_pos``: [2*max-1, C] table (linearly resized if needed) -> [q_size, k_size, C]."""
    max_rel = int(2 * max(q_size, k_size) - 1)
    if rel_pos.shape[0] != max_rel:
        r = F.interpolate(rel_pos.float().reshape(1, rel_pos.shape[0], -1).permute(0, 2, 1), size=max_rel,
                          mode="linear")
        rel_pos = r.reshape(-1, max_rel).permute(1, 0).to(rel_pos.dtype)
    qc = torch.arange(q_size, device=rel_pos.device)[:, None] * max(k_size / q_size, 1.0)
    kc = torch.arange(k_size, device=rel_pos.device)[None, :] * max(q_size / k_size, 1.0)
    rc = (qc - kc) + (k_size - 1) * max(q_size / k_size, 1.0)
    return rel_pos[rc.long()]


def rel_pos_terms(q: torch.Tensor, Rh: torch.Tensor, Rw: torch.Tensor, gh: int, gw: int):
    """q [B, N, H, D] (unscaled), Rh [gh, gh, D], Rw [gw, gw, D] -> rel_h [B, H, N, gh], rel_w [B, H, N, gw]."""
    B, N, H, D = q.shape
    r = q.float().reshape(B, gh, gw, H, D)
    rel_h = torch.einsum("byxhc,ykc->bhyxk", r, Rh.float()).reshape(B, H, N, gh)
    rel_w = torch.einsum("byxhc,xkc->bhyxk", r, Rw.float()).reshape(B, H, N, gw)
    return rel_h, rel_w


class _SamAttn(nn.Module):
    def __init__(self, dim, heads, grid):
        super().__init__()
        self.num_heads = heads
        self.qkv = nn.Linear(dim, 3 * dim, bias=True)
        self.proj = nn.Linear(dim, dim)
        hd = dim // heads
        self.rel_pos_h = nn.Parameter(torch.zeros(2 * grid - 1, hd))
        self.rel_pos_w = nn.Parameter(torch.zeros(2 * grid - 1, hd))


class _SamMlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.lin1 = nn.Linear(dim, hidden)
        self.lin2 = nn.Linear(hidden, dim)


class _SamBlock(nn.Module):
    def __init__(self, dim, heads, grid, mlp_ratio=4.0):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = _SamAttn(dim, heads, grid)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = _SamMlp(dim, int(dim * mlp_ratio))

    def forward(self, x):  # x [B, gh, gw, C]
        B, gh, gw, C = x.shape
        H = self.attn.num_heads
        N = gh * gw
        qkv = self.attn.qkv(self.norm1(x).reshape(B, N, C)).reshape(B, N, 3, H, C // H)
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        Rh = get_rel_pos(gh, gh, self.attn.rel_pos_h)
        Rw = get_rel_pos(gw, gw, self.attn.rel_pos_w)
        rel_h, rel_w = rel_pos_terms(q, Rh, Rw, gh, gw)
        scale = (C // H) ** -0.5
        if q.dtype == torch.bfloat16 and q.is_cuda:
            a = flash_attention(q, k, v, scale, rel_h, rel_w)
        else:
            a = attention_ref(q, k, v, scale, rel_h, rel_w).to(q.dtype)
        x = x + self.attn.proj(a.reshape(B, N, C)).reshape(B, gh, gw, C)
        return x + self.mlp.lin2(F.gelu(self.mlp.lin1(self.norm2(x))))


class _LayerNorm2d(nn.Module):
    def __init__(self, c, eps=1e-6):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))
        self.eps = eps

    def forward(self, x):  # NCHW
        u = x.mean(1, keepdim=True)
        s = (x - u).pow(2).mean(1, keepdim=True)
        x = (x - u) / torch.sqrt(s + self.eps)
        return self.weight[:, None, None] * x + self.bias[:, None, None]


class _Encoder(nn.Module):
    def __init__(self, dim, depth, heads, ps, grid, out_chans=256):
        super().__init__()
        self.patch_embed = nn.Module()
        self.patch_embed.proj = nn.Conv2d(3, dim, ps, ps)
        self.pos_embed = nn.Parameter(torch.zeros(1, grid, grid, dim))
        self.blocks = nn.ModuleList([_SamBlock(dim, heads, grid) for _ in range(depth)])
        self.neck = nn.Sequential(nn.Conv2d(dim, out_chans, 1, bias=False), _LayerNorm2d(out_chans),
                                  nn.Conv2d(out_chans, out_chans, 3, padding=1, bias=False), _LayerNorm2d(out_chans))


class CPSAM(nn.Module):
    """Cellpose-SAM network (ViT-L/8 by default; ``dim/depth/heads`` shrink it for tests)."""

    def __init__(self, dim: int = 1024, depth: int = 24, heads: int = 16, ps: int = 8, bsize: int = 256,
                 nout: int = 3, rdrop: float = 0.4):
        super().__init__()
        self.ps, self.bsize, self.nout, self.rdrop = ps, bsize, nout, rdrop
        self.grid = bsize // ps
        self.encoder = _Encoder(dim, depth, heads, ps, self.grid)
        self.out = nn.Conv2d(256, nout * ps * ps, 1)
        self.W2 = nn.Parameter(torch.eye(nout * ps * ps).reshape(nout * ps * ps, nout, ps, ps), requires_grad=False)
        self.diam_labels = nn.Parameter(torch.tensor([30.0]), requires_grad=False)
        self.diam_mean = nn.Parameter(torch.tensor([30.0]), requires_grad=False)

    @torch.no_grad()
    def randomize_(self, seed: int = 0) -> "CPSAM":
        gen = torch.Generator().manual_seed(seed)
        for name, p in self.named_parameters():
            if name in ("W2", "diam_labels", "diam_mean"):
                continue
            if "norm" in name or name.startswith("encoder.neck.1") or name.startswith("encoder.neck.3"):
                p.fill_(1.0 if name.endswith("weight") else 0.0)
            elif name.endswith("bias"):
                p.zero_()
            elif "rel_pos" in name or "pos_embed" in name:
                p.copy_(torch.randn(p.shape, generator=gen) * 0.02)
            else:
                fan_in = p[0].numel() if p.dim() > 1 else p.numel()
                p.copy_(torch.randn(p.shape, generator=gen) * (1.0 / fan_in) ** 0.5)
        return self

    def forward(self, x: torch.Tensor, keep: torch.Tensor | None = None):
        """x [B, 3, bsize, bsize] -> (flows [B, nout, bsize, bsize], style placeholder [B, 256]).

        Training-mode stochastic depth as cellpose 4's ``Transformer.forward``: per sample, block i
        is replaced by the identity with probability ``linspace(0, rdrop, nlay)[i]``
        (``x * mask + blk(x) * (1 - mask)``).  ``keep`` [B, nlay] (0/1) overrides the random draw."""
        e = self.encoder
        t = e.patch_embed.proj(x).permute(0, 2, 3, 1)
        t = t + e.pos_embed.to(t.dtype)
        nl = len(e.blocks)
        if keep is None and self.training and self.rdrop > 0:
            keep = (torch.rand(x.shape[0], nl, device=x.device) >=
                    torch.linspace(0, self.rdrop, nl, device=x.device)[None]).to(t.dtype)
        for i, blk in enumerate(e.blocks):
            if keep is None:
                t = blk(t)
            else:
                k = keep[:, i].to(t.dtype)[:, None, None, None]
                t = t * (1 - k) + blk(t) * k
        y = e.neck(t.permute(0, 3, 1, 2))
        y = self.out(y)
        y = F.conv_transpose2d(y, self.W2.to(y.dtype), stride=self.ps)
        return y, torch.zeros(x.shape[0], 256, device=x.device, dtype=y.dtype)


class CPSAMEngine:
    """bf16 HIP inference path of :class:`CPSAM` (see module docstring)."""

    def __init__(self, net: CPSAM, device):
        self.device = torch.device(device)
        self.net = net
        e = net.encoder
        bf = lambda t: t.detach().to(self.device, torch.bfloat16).contiguous()
        f32 = lambda t: t.detach().to(self.device, torch.float32).contiguous()
        self.ps, self.grid, self.nout = net.ps, net.grid, net.nout
        w = e.patch_embed.proj.weight
        self.dim = w.shape[0]
        self.heads = e.blocks[0].attn.num_heads
        self.pe_w, self.pe_b = bf(w.reshape(w.shape[0], -1)), bf(e.patch_embed.proj.bias)
        self.pos = bf(e.pos_embed[0].reshape(-1, self.dim))
        self.blocks = []
        g = self.grid
        for blk in e.blocks:
            self.blocks.append(dict(
                n1w=f32(blk.norm1.weight), n1b=f32(blk.norm1.bias), qkv_w=bf(blk.attn.qkv.weight),
                qkv_b=bf(blk.attn.qkv.bias), proj_w=bf(blk.attn.proj.weight), proj_b=bf(blk.attn.proj.bias),
                Rh=f32(get_rel_pos(g, g, blk.attn.rel_pos_h.detach())),
                Rw=f32(get_rel_pos(g, g, blk.attn.rel_pos_w.detach())),
                # the [2g-1, c] tables themselves for the MFMA rel-pos kernel (gather inside)
                tab_h=f32(blk.attn.rel_pos_h) if blk.attn.rel_pos_h.shape[0] == 2 * g - 1 else None,
                tab_w=f32(blk.attn.rel_pos_w) if blk.attn.rel_pos_w.shape[0] == 2 * g - 1 else None,
                n2w=f32(blk.norm2.weight), n2b=f32(blk.norm2.bias), l1_w=bf(blk.mlp.lin1.weight),
                l1_b=f32(blk.mlp.lin1.bias), l2_w=bf(blk.mlp.lin2.weight), l2_b=bf(blk.mlp.lin2.bias)))
        self.neck0 = bf(e.neck[0].weight.reshape(e.neck[0].weight.shape[0], -1))
        self.ln1w, self.ln1b = f32(e.neck[1].weight), f32(e.neck[1].bias)
        self.neck2 = PackedConv.from_weight(e.neck[2].weight.detach().float()).to(self.device)
        self.ln2w, self.ln2b = f32(e.neck[3].weight), f32(e.neck[3].bias)
        self.out_w = bf(net.out.weight.reshape(net.out.weight.shape[0], -1))
        self.out_b = bf(net.out.bias)

    #: GEMM backend of the inference engine: "ltgelu" (default: hipBLASLt, lin1 with its GELU_BIAS
    #: epilogue = tanh-approximated GELU fused into the GEMM), "lib" (hipBLASLt + the exact-erf HIP
    #: bias_gelu_ pass) or "mt" / "hyb" (the framework's macro-tile MFMA GEMM).  Measured on MI355X,
    #: 72 tiles of 256^2 (profiles/r06/cpsam/gelu_ab_s13.jsonl): ltgelu 62.9 ms, lib 66.8 ms per
    #: forward; flows cosine 0.99992 against the exact-GELU path (max abs 0.07 of 4.8).  Earlier:
    #: lib 99.7 img/s, mt 84.4 (profiles/r05/cpsam/infer_mt_vs_lib_s23.jsonl).  Fine-tuning
    #: (train/cpsam_engine.py) keeps the exact GELU.
    GEMM = os.environ.get("BE_CPSAM_INFER_GEMM", "ltgelu")
    #: rel-pos terms: "hip" (relpos.hip MFMA kernel, default) or "torch" (fp32 einsums; A/B only)
    RELPOS = os.environ.get("BE_CPSAM_RELPOS", "hip")

    def _gemms(self):
        if self.GEMM in ("lib", "hyb"):
            def lin(x, w, b=None):
                return F.linear(x, w, b)

            if self.GEMM == "hyb":  # lin1 on the macro-tile GEMM with bias + exact GELU fused
                from ..ops import gemm_mt

                return lin, gemm_mt.linear_gelu_only

            def lin_gelu(x, w, b):
                return bias_gelu_(F.linear(x, w), b)
            return lin, lin_gelu
        if self.GEMM == "ltgelu":  # hipBLASLt GELU_BIAS epilogue (tanh-approximated GELU); A/B
            def lin(x, w, b=None):
                return F.linear(x, w, b)

            def lin_gelu(x, w, b):
                return torch._addmm_activation(b.to(x.dtype), x, w.t(), use_gelu=True)
            return lin, lin_gelu
        from ..ops import gemm_mt

        return gemm_mt.linear, gemm_mt.linear_gelu_only

    @torch.no_grad()
    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        """x [B, 3, bsize, bsize] float -> flows [B, nout, bsize, bsize] fp32."""
        B = x.shape[0]
        ps, g, D, Hh = self.ps, self.grid, self.dim, self.heads
        N = g * g
        lin, lin_gelu = self._gemms()
        x = x.to(self.device, torch.bfloat16)
        patches = x.reshape(B, 3, g, ps, g, ps).permute(0, 2, 4, 1, 3, 5).reshape(B * N, 3 * ps * ps)
        t = (lin(patches, self.pe_w, self.pe_b).view(B, N, D) + self.pos).contiguous()
        blocks = self.blocks
        h = add_layernorm(t, None, None, blocks[0]["n1w"], blocks[0]["n1b"])
        for i, b in enumerate(blocks):
            qkv = lin(h.view(B * N, D), b["qkv_w"], b["qkv_b"]).view(B, N, 3, Hh, D // Hh)
            q = qkv[:, :, 0]
            if b["tab_h"] is not None and b["tab_w"] is not None and q.is_cuda and self.RELPOS == "hip":
                # relpos.hip (the training engine's kernel): q . R on MFMA straight from the strided
                # q view; the fp32 einsums it replaces were ~21 % of the forward's kernel time
                # (q.float() copies, permuted outputs, fp32 library GEMMs; profiles/r05/kt/cpi_stats.txt)
                rel_h, rel_w = relpos_fwd(q, b["tab_h"], b["tab_w"])
            else:
                rel_h, rel_w = rel_pos_terms(q, b["Rh"], b["Rw"], g, g)
            a = flash_attention(q, qkv[:, :, 1], qkv[:, :, 2], (D // Hh) ** -0.5, rel_h, rel_w).view(B * N, D)
            y = lin(a, b["proj_w"], b["proj_b"]).view(B, N, D)
            h2 = add_layernorm(t, y, None, b["n2w"], b["n2b"])
            m = lin(lin_gelu(h2.view(B * N, D), b["l1_w"], b["l1_b"]), b["l2_w"], b["l2_b"]).view(B, N, D)
            if i + 1 < len(blocks):
                h = add_layernorm(t, m, None, blocks[i + 1]["n1w"], blocks[i + 1]["n1b"])
            else:
                t.add_(m)
        # neck: 1x1 conv (GEMM) -> LN2d -> 3x3 conv (NHWC MFMA kernel) -> LN2d
        n0 = lin(t.view(B * N, D), self.neck0).view(B, N, -1)          # [B, N, 256]
        n0 = add_layernorm(n0, None, None, self.ln1w, self.ln1b)
        n2 = fused_conv2d(n0.view(B, g, g, -1), self.neck2)            # NHWC [B, g, g, 256]
        n2 = add_layernorm(n2.view(B, N, -1), None, None, self.ln2w, self.ln2b)
        o = lin(n2.view(B * N, -1), self.out_w, self.out_b).float()    # [B * N, nout*ps*ps]
        # conv_transpose2d with the identity W2 == pixel shuffle
        o = o.view(B, g, g, self.nout, ps, ps).permute(0, 3, 1, 4, 2, 5).reshape(B, self.nout, g * ps, g * ps)
        return o

    #: graphs kept by :meth:`graphed`, one per exact tile count, least recently used evicted: each
    #: holds a private memory pool with the whole forward's intermediates, so a server seeing images
    #: of many sizes must not keep one per size forever.  Exact counts, not padded buckets: padding the
    #: 9 tiles of one 512^2 image to a 16-tile bucket cost 40 % of the batch-1 latency (15.3 vs 11.0 ms,
    #: profiles/r06/bench_1gpu_s12.json), and a 72-tile batch above a 64 bucket ran eagerly.
    GRAPH_MAX = int(os.environ.get("BE_CPSAM_GRAPH_MAX", "8"))
    #: largest tile count replayed from a graph (larger batches run eagerly)
    GRAPH_MAX_TILES = 256
    #: capture attempts per tile count before that count stays eager for the process
    GRAPH_MAX_TRIES = 3
    #: BE_CPSAM_GRAPH=0 turns graph replay off (every call runs the eager forward)
    GRAPH = os.environ.get("BE_CPSAM_GRAPH", "1") != "0"

    @torch.no_grad()
    def graphed(self, x: torch.Tensor) -> torch.Tensor:
        """:meth:`__call__` replayed from a HIP graph per tile count (static input buffer; the output
        is a fresh copy), at most GRAPH_MAX graphs alive (LRU).  Falls back to the eager forward
        off-GPU, above GRAPH_MAX_TILES, with BE_CPSAM_GRAPH=0, and when a capture fails (counted per
        tile count: after GRAPH_MAX_TRIES failures that count stays eager)."""
        import collections

        B = x.shape[0]
        if (not (x.is_cuda and self.device.type == "cuda") or not self.GRAPH or B > self.GRAPH_MAX_TILES
                or self.GRAPH_MAX <= 0):
            return self(x)
        graphs = self.__dict__.setdefault("_graphs", collections.OrderedDict())
        fails = self.__dict__.setdefault("_graph_fails", {})
        key = tuple(x.shape)
        if fails.get(key, 0) >= self.GRAPH_MAX_TRIES:
            return self(x)
        ent = graphs.get(key)
        if ent is None:
            while len(graphs) >= self.GRAPH_MAX:
                graphs.popitem(last=False)  # least recently used: its pool returns to the allocator
            xs = torch.empty(x.shape, device=self.device, dtype=torch.bfloat16)
            xs.copy_(x)
            side = torch.cuda.Stream(self.device)
            side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(side):
                self(xs)  # lazy state (kernel attributes, workspaces) outside the capture
            torch.cuda.current_stream(self.device).wait_stream(side)
            gr = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(gr, capture_error_mode="thread_local"):
                    out = self(xs)
            except Exception:  # noqa: BLE001 -- counted; the request itself runs eagerly
                fails[key] = fails.get(key, 0) + 1
                return self(x)
            ent = graphs[key] = (gr, xs, out)
        graphs.move_to_end(key)
        gr, xs, out = ent
        xs.copy_(x)
        gr.replay()
        return out.clone()

