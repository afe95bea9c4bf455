"""Cellpose-SAM (``cpsam``) training engine: explicit forward + backward on the framework's kernels.

The reference fine-tunes Cellpose-SAM (``apps/cellpose-finetuning/main.py:1278-1713``; net in
fp32 after a bf16 load, ``:1350-1358``; AdamW ``:1451-1453``; ``_loss_fn_seg`` ``:1514-1517``;
SURVEY.md §2.5 K8) through PyTorch autograd.  Here the ViT-L/8 step is written out by hand so every
hot op is ours and the whole step can be one HIP graph:

forward, per block (pre-norm SAM block, global attention, decomposed rel-pos bias)::

    h1, st1   = LN1(t_in)                                 fused add+LN kernel (stats saved)
    qkv       = h1 Wqkv^T + b                             hipBLASLt
    rel_h/w   = q . R_h / R_w                             MFMA per (b, h, grid line) (relpos.hip)
    a, lse    = flash_attn(q, k, v, rel_h, rel_w)         HIP MFMA kernel (attention.hip)
    y         = a Wproj^T + b
    t_mid,h2  = t_in + k_b * y, LN2(t_mid)                fused add+LN (k_b = stochastic-depth keep)
    f         = h2 W1^T ;  g = gelu(f + b1)               hipBLASLt + HIP GELU
    m         = g W2^T + b2
    t_out     = t_mid + k_b * m                           fused into the next block's LN1

backward mirrors it with the HIP LayerNorm/GELU/cast backward kernels (``vit_train.hip``), the
flash-attention backward with rel-pos gradients (``attention_bwd.hip``), and hipBLASLt dgrad/wgrad
GEMMs whose fp32 weight gradients land directly in the flat gradient buffer the fused AdamW reads.

Stochastic depth follows cellpose 4's ``Transformer.forward``: per sample and layer, a block is
dropped with probability ``linspace(0, rdrop, nlay)[layer]`` (``x*mask + blk(x)*(1-mask)``).  Since
the mask is 0/1, ``t_in + k (y + m)`` with ``t_mid = t_in + k y`` is the same function and the
same gradients, and keeps every kernel's shape static (graph-capturable).

Precision: bf16 operands with fp32 accumulation, fp32 master weights, LayerNorm statistics,
softmax, residual-stream gradients and optimizer state (the reference runs fp32; the numerics test
bounds the difference against an fp32 autograd oracle).  On CPU every op runs its fp32 PyTorch
reference, so the same engine code is checked against autograd in the CPU suite.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from ..models.cpsam import CPSAM, get_rel_pos
import os as _os

# GEMM backend of the engine.  "auto" = per shape, the fastest of the in-house bf16 MFMA GEMMs with
# fused epilogues (ops/gemm_bf16.py, ops/gemm_pp.py) and the library GEMM (ops/gemm_auto.py,
# decided on the eager warm-up steps); "hip" / "lib" pin one side.  The default is the library: on
# the whole graphed step it measured 11.35 / 31.70 ms at batch 1 / 8 against 12.69 / 32.67 for
# "auto" (profiles/r04/cpsam/cpsam_gemm_*.jsonl).  The first per-shape timing bracketed single
# eager calls and so measured launch overhead; in the graph the library's kernels are the faster
# ones (profiles/r04/cpsam/kt_step_b1_*.txt), and gemm_auto now times graph replays.
_GEMM = _os.environ.get("BE_CPSAM_GEMM", "lib")
if _GEMM == "lib":
    from ..ops import gemm
elif _GEMM == "mt":
    from ..ops import gemm_mt as gemm
elif _GEMM == "hip":
    from ..ops import gemm_bf16 as gemm
else:
    from ..ops import gemm_auto as gemm
from ..ops import vit_train as vt
from ..ops.conv import PackedConv, fused_conv2d
from ..ops.conv_train import conv_wgrad
from ..parallel.ddp import FlatParams

#: smallest token count m at which the <= 192-tile weight gradients run split-K 4 (A/B knob; at batch 1,
#: m = 1024, splitting measured slower: 11.39-11.74 vs 11.91-12.02 ms, profiles/r03/cpsam/wgrad_split_b1_ab.txt)
_SPLIT_MIN_M = int(os.environ.get("BE_WGRAD_SPLIT_MIN_M", "4096"))
_MM_MODE: int | None = None  # 2: mm(out_dtype=fp32, out=grad view), 1: mm(out_dtype=fp32) + copy, 0: bf16 mm + copy


def _wgrad(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor) -> None:
    """out (fp32 [n, k]) = dy^T x with dy [m, n], x [m, k].  On GPU the bf16 GEMM writes fp32 straight
    into the parameter's view of the flat gradient buffer when this torch supports it."""
    global _MM_MODE
    out2 = out.view(out.shape[0], -1)
    if dy.dtype != torch.bfloat16:
        torch.mm(dy.t(), x, out=out2)
        return
    if _MM_MODE is None:
        _MM_MODE = 0
        for mode in (2, 1):
            try:
                probe = torch.empty(dy.shape[1], x.shape[1], device=dy.device, dtype=torch.float32)
                if mode == 2:
                    torch.mm(dy.t(), x, out_dtype=torch.float32, out=probe)
                else:
                    torch.mm(dy.t(), x, out_dtype=torch.float32)
                _MM_MODE = mode
                break
            except Exception:  # noqa: BLE001
                continue
    m, n, k = dy.shape[0], dy.shape[1], x.shape[1]
    # the 4096-wide fc1 / fc2 weight gradients: hipBLASLt runs them as one 128x128 tile per CU (256
    # tiles, K = 8192 each); split-K 2 + the vectorised slab sum measured 34.42 -> 33.37 ms per batch-8
    # step (profiles/r03/cpsam/wgrad_split_wide_ab.txt; split 4: 33.45).  BE_WGRAD_SPLIT_WIDE=0 turns it off.
    wide_split = int(os.environ.get("BE_WGRAD_SPLIT_WIDE", "2"))
    if _MM_MODE == 2 and wide_split > 1 and m >= 4096 and m % wide_split == 0 and n * k > 3072 * 1024:
        ws = torch.empty(wide_split, n, k, device=dy.device, dtype=torch.float32)
        torch.bmm(dy.reshape(wide_split, m // wide_split, n).transpose(1, 2), x.reshape(wide_split, m // wide_split, k),
                  out_dtype=torch.float32, out=ws)
        vt.sum_slabs(ws, out2)
    elif _MM_MODE == 2 and m >= _SPLIT_MIN_M and m % 4 == 0 and n * k <= 3072 * 1024:
        # split-K: the [n, k] output is <= 192 hipBLASLt 128x128 tiles, under one per CU, so the
        # m = B*N reduction runs as 4 batched slices + an fp32 sum (profiles/r02/attn/wgrad.jsonl:
        # proj 57.8 -> 37.7 us, qkv 87.6 -> 74.6 us; the 4096-wide fc1 / fc2 outputs gain nothing)
        ws = torch.empty(4, n, k, device=dy.device, dtype=torch.float32)
        torch.bmm(dy.reshape(4, m // 4, n).transpose(1, 2), x.reshape(4, m // 4, k), out_dtype=torch.float32, out=ws)
        vt.sum_slabs(ws, out2)
    elif _MM_MODE == 2:
        torch.mm(dy.t(), x, out_dtype=torch.float32, out=out2)
    elif _MM_MODE == 1:
        out2.copy_(torch.mm(dy.t(), x, out_dtype=torch.float32))
    else:
        out2.copy_(torch.mm(dy.t(), x))


class _Blk:
    __slots__ = ("p", "w")

    def __init__(self):
        self.p = {}
        self.w = {}


class CPSAMTrainEngine:
    """Forward + backward of :class:`CPSAM` at a fixed batch shape ``[B, 3, bsize, bsize]``."""

    #: the neck's 3x3 conv (fwd, dgrad, wgrad) on the NHWC MFMA / implicit-GEMM HIP kernels
    #: (BE_CPSAM_NECK=miopen: the library convolution it replaces, A/B only)
    NECK_HIP = os.environ.get("BE_CPSAM_NECK", "hip") != "miopen"

    def __init__(self, net: CPSAM, fp: FlatParams, B: int, device, eps: float = 1e-6,
                 side_wgrad: bool | None = None):
        self.net, self.fp, self.B = net, fp, int(B)
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        # Optional: weight-gradient GEMMs (and bias column sums) on a second stream, off the dgrad
        # critical path (fork/join are stream waits, so the step stays graph-capturable).  Measured
        # slower on MI355X at both batch sizes (profiles/r03/cpsam/side_wgrad_ab.jsonl: batch 1 12.47
        # -> 13.74 ms, batch 8 33.74 -> 35.01 ms: two GEMMs sharing the CUs run longer than they
        # overlap), so it is off unless asked for (side_wgrad=True / BE_CPSAM_SIDE_WGRAD=1).
        if side_wgrad is None and os.environ.get("BE_CPSAM_SIDE_WGRAD", "") in ("0", "1"):
            side_wgrad = os.environ["BE_CPSAM_SIDE_WGRAD"] == "1"  # A/B override
        self._side_wgrad = side_wgrad
        self._side: torch.cuda.Stream | None = None
        self._side_keep: list = []
        self.cdt = torch.bfloat16 if self.cuda else torch.float32
        self.eps = eps
        e = net.encoder
        self.ps, self.g, self.nout = net.ps, net.grid, net.nout
        self.D = e.patch_embed.proj.weight.shape[0]
        self.H = e.blocks[0].attn.num_heads
        self.hd = self.D // self.H
        self.N = self.g * self.g
        self.scale = self.hd ** -0.5
        self.mirror = fp.flat.to(self.cdt) if self.cdt != torch.float32 else fp.flat
        off = {id(p): o for p, o in zip(fp.params, fp.offsets)}
        W = lambda p: self.mirror[off[id(p)]: off[id(p)] + p.numel()].view_as(p)
        self._W = W
        self.pe = (e.patch_embed.proj.weight, e.patch_embed.proj.bias)
        self.pos = e.pos_embed
        self.blocks = []
        for blk in e.blocks:
            b = _Blk()
            b.p = dict(n1w=blk.norm1.weight, n1b=blk.norm1.bias, qkv_w=blk.attn.qkv.weight, qkv_b=blk.attn.qkv.bias,
                       proj_w=blk.attn.proj.weight, proj_b=blk.attn.proj.bias, rph=blk.attn.rel_pos_h,
                       rpw=blk.attn.rel_pos_w, n2w=blk.norm2.weight, n2b=blk.norm2.bias, l1_w=blk.mlp.lin1.weight,
                       l1_b=blk.mlp.lin1.bias, l2_w=blk.mlp.lin2.weight, l2_b=blk.mlp.lin2.bias)
            b.w = {k: W(v) for k, v in b.p.items()}
            self.blocks.append(b)
        self.neck = e.neck
        self.outc = net.out
        nw = self.neck[2].weight.detach().float()
        self._neck_pc = PackedConv.from_weight(nw).to(self.device)                                 # forward
        self._neck_pcT = PackedConv.from_weight(nw.flip(2, 3).transpose(0, 1).contiguous()).to(self.device)  # dgrad
        g = self.g
        ar = torch.arange(g, device=self.device)
        self.rel_idx = (ar[:, None] - ar[None, :] + (g - 1)).long()  # get_rel_pos index at q == k size
        for blk in e.blocks:
            if blk.attn.rel_pos_h.shape[0] != 2 * g - 1:
                raise ValueError("CPSAMTrainEngine needs rel-pos tables sized for the training grid")

    def refresh_mirror(self) -> None:
        """Re-derive the bf16 weight mirror from the fp32 master (after a load / broadcast)."""
        if self.mirror is not self.fp.flat:
            self.mirror.copy_(self.fp.flat)

    # ------------------------------------------------------------------ helpers
    def _rel_terms(self, q: torch.Tensor, Rh: torch.Tensor, Rw: torch.Tensor):
        """q [B, N, H, c] -> rel_h [B, H, N, g], rel_w [B, H, N, g] (fp32) as batched GEMMs."""
        B, g, H, c = self.B, self.g, self.H, self.hd
        q5 = q.reshape(B, g, g, H, c)
        # rel_h[b,h,y,x,k] = sum_c q[b,y,x,h,c] Rh[y,k,c]: batch over y
        qy = q5.permute(1, 0, 2, 3, 4).reshape(g, B * g * H, c).float()
        rh = torch.bmm(qy, Rh.transpose(1, 2)).reshape(g, B, g, H, g).permute(1, 3, 0, 2, 4)
        qx = q5.permute(2, 0, 1, 3, 4).reshape(g, B * g * H, c).float()
        rw = torch.bmm(qx, Rw.transpose(1, 2)).reshape(g, B, g, H, g).permute(1, 3, 2, 0, 4)
        return rh.reshape(B, H, self.N, g).contiguous(), rw.reshape(B, H, self.N, g).contiguous()

    def _rel_bwd(self, q, Rh, Rw, drh, drw):
        """-> (dq_rel [B, N, H, c] fp32, dRh [g, g, c], dRw [g, g, c])."""
        B, g, H, c = self.B, self.g, self.H, self.hd
        drh5 = drh.reshape(B, H, g, g, g)  # b h y x k
        drw5 = drw.reshape(B, H, g, g, g)
        # dq[b,y,x,h,c] = sum_k drh[b,h,y,x,k] Rh[y,k,c] + sum_k drw[b,h,y,x,k] Rw[x,k,c]
        a = drh5.permute(2, 0, 3, 1, 4).reshape(g, B * g * H, g)          # y, (b x h), k
        dq_h = torch.bmm(a, Rh).reshape(g, B, g, H, c).permute(1, 0, 2, 3, 4)
        bw = drw5.permute(3, 0, 2, 1, 4).reshape(g, B * g * H, g)          # x, (b y h), k
        dq_w = torch.bmm(bw, Rw).reshape(g, B, g, H, c).permute(1, 2, 0, 3, 4)
        q5 = q.reshape(B, g, g, H, c).float()
        qy = q5.permute(1, 0, 2, 3, 4).reshape(g, B * g * H, c)            # y, (b x h), c
        dRh = torch.bmm(a.transpose(1, 2), qy)                              # y, k, c
        qx = q5.permute(2, 0, 1, 3, 4).reshape(g, B * g * H, c)            # x, (b y h), c
        dRw = torch.bmm(bw.transpose(1, 2), qx)
        return (dq_h + dq_w).reshape(B, self.N, H, c), dRh, dRw

    def _use_side(self) -> bool:
        if not self.cuda:
            return False
        return bool(self._side_wgrad)

    def _off_path(self, fn, *keep: torch.Tensor) -> None:
        """Run ``fn`` (weight-gradient work) on the side stream after everything queued so far on the
        current stream; the operands stay referenced until :meth:`_join_side`, so the allocator
        cannot hand their memory to later main-stream work while the side stream still reads it."""
        if self._side is None:
            fn()
            return
        self._side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self._side):
            fn()
        self._side_keep.extend(keep)

    def _join_side(self) -> None:
        if self._side is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._side)
            self._side_keep.clear()

    def _table_grad(self, dR: torch.Tensor, out: torch.Tensor) -> None:
        out.zero_()
        out.index_add_(0, self.rel_idx.reshape(-1), dR.reshape(-1, dR.shape[-1]))

    # ------------------------------------------------------------------ forward
    @torch.no_grad()
    def forward(self, x: torch.Tensor, keep: torch.Tensor | None = None, save: bool = True) -> torch.Tensor:
        """x [B, C<=3, S, S] float -> flows [B, nout, S, S] (compute dtype).  ``keep`` [B, nlay] 0/1
        (stochastic depth; None = keep all)."""
        B, ps, g, D, N, H = self.B, self.ps, self.g, self.D, self.N, self.H
        assert x.shape[0] == B and x.shape[-1] == g * ps and x.shape[-2] == g * ps
        if x.shape[1] < 3:
            x = torch.cat([x, x.new_zeros(B, 3 - x.shape[1], *x.shape[2:])], 1)
        W = self._W
        patches = x.to(self.cdt).reshape(B, 3, g, ps, g, ps).permute(0, 2, 4, 1, 3, 5).reshape(B * N, 3 * ps * ps)
        t = gemm.linear(patches, W(self.pe[0]).reshape(D, -1), W(self.pe[1]))
        t = (t.view(B, N, D) + W(self.pos).reshape(1, N, D)).reshape(B * N, D).contiguous()
        saved = {"patches": patches, "keep": keep, "blocks": []}
        nl = len(self.blocks)
        # LN1 of block 0
        _, h1, st1 = vt.ln_fwd(t, self.blocks[0].p["n1w"], self.blocks[0].p["n1b"], eps=self.eps)
        for i, b in enumerate(self.blocks):
            w, p = b.w, b.p
            kb = keep[:, i].contiguous() if keep is not None else None
            qkv = gemm.linear(h1, w["qkv_w"], w["qkv_b"]).view(B, N, 3, H, self.hd)
            q, k_, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
            if self.cuda:  # tables gathered inside relpos.hip (no get_rel_pos index kernels)
                Rh, Rw = p["rph"].detach(), p["rpw"].detach()
                rel_h, rel_w = vt.relpos_fwd(q, Rh, Rw)
            else:
                Rh = get_rel_pos(g, g, p["rph"].detach()).float()
                Rw = get_rel_pos(g, g, p["rpw"].detach()).float()
                rel_h, rel_w = self._rel_terms(q, Rh, Rw)
            a, lse = vt.attn_fwd(q, k_, v, self.scale, rel_h, rel_w)
            a2 = a.reshape(B * N, D)
            y = gemm.linear(a2, w["proj_w"], w["proj_b"])
            t_mid, h2, st2 = vt.ln_fwd(t, p["n2w"], p["n2b"], y=y, rs=kb, rpn=N, eps=self.eps)
            gg, f = gemm.linear_gelu(h2, w["l1_w"], w["l1_b"])  # f: pre-activation (epilogue aux output)
            m = gemm.linear(gg, w["l2_w"], w["l2_b"])
            if save:
                saved["blocks"].append(dict(t_in=t, st1=st1, h1=h1, qkv=qkv, rel_h=rel_h, rel_w=rel_w, Rh=Rh, Rw=Rw,
                                            a=a, lse=lse, t_mid=t_mid, st2=st2, h2=h2, f=f, g=gg, keep=kb))
            if i + 1 < nl:
                nb = self.blocks[i + 1].p
                t, h1, st1 = vt.ln_fwd(t_mid, nb["n1w"], nb["n1b"], y=m, rs=kb, rpn=N, eps=self.eps)
            else:
                t = self._residual(t_mid, m, kb)
        # neck: 1x1 conv (GEMM) -> LN2d -> 3x3 conv -> LN2d -> readout -> pixel shuffle
        n0 = gemm.linear(t, W(self.neck[0].weight).reshape(256, D))
        _, n1, sn1 = vt.ln_fwd(n0, self.neck[1].weight, self.neck[1].bias, eps=self.eps)
        n1i = n1.view(B, g, g, 256).permute(0, 3, 1, 2)  # NCHW view of NHWC memory (channels_last)
        if self.NECK_HIP and n1.is_cuda and n1.dtype == torch.bfloat16:
            # the 3x3 neck conv on the NHWC MFMA kernel (conv2d_nhwc.hip), weights re-packed from the
            # bf16 mirror every step (a few device copies; graph-capturable)
            self._neck_pc.refresh(W(self.neck[2].weight).float())
            n2r = fused_conv2d(n1.view(B, g, g, 256), self._neck_pc).view(B * N, 256)
        else:
            n2 = F.conv2d(n1i, W(self.neck[2].weight), padding=1)
            n2r = n2.permute(0, 2, 3, 1).reshape(B * N, 256).contiguous()
        _, n3, sn3 = vt.ln_fwd(n2r, self.neck[3].weight, self.neck[3].bias, eps=self.eps)
        o = gemm.linear(n3, W(self.outc.weight).reshape(self.outc.weight.shape[0], 256), W(self.outc.bias))
        yout = o.view(B, g, g, self.nout, ps, ps).permute(0, 3, 1, 4, 2, 5).reshape(B, self.nout, g * ps, g * ps)
        if save:
            saved.update(t_last=t, n0=n0, n1=n1, n1i=n1i, sn1=sn1, n2r=n2r, sn3=sn3, n3=n3)
            self._saved = saved
        return yout

    @staticmethod
    def _residual(x, y, kb):
        if kb is None:
            return x + y
        B = kb.shape[0]
        return (x.view(B, -1) + y.view(B, -1) * kb.to(x.dtype)[:, None]).view(x.shape)

    # ------------------------------------------------------------------ backward
    @torch.no_grad()
    def backward(self, dyout: torch.Tensor, on_params_ready=None) -> None:
        """dyout [B, nout, S, S] -> parameter gradients written into ``fp.grad`` (overwritten).
        ``on_params_ready(params)`` fires as each group's gradients are final (DDP bucket launch)."""
        if self.cuda:  # LayerNorm / bias column reductions batched into a few launches
            with vt.defer_colsums() as dc:
                self._backward(dyout, on_params_ready, dc)
        else:
            self._backward(dyout, on_params_ready, None)

    def _backward(self, dyout: torch.Tensor, on_params_ready, dc) -> None:
        if self._use_side():
            if self._side is None:
                self._side = torch.cuda.Stream(self.device)
        else:
            self._side = None
        if on_params_ready is None:
            ready = lambda ps: None  # noqa: E731
        else:
            def ready(ps):  # a bucket's consumer reads these gradients on the main stream
                if dc is not None:
                    dc.flush()
                self._join_side()
                on_params_ready(ps)
        s = self._saved
        B, ps, g, D, N, H, hd = self.B, self.ps, self.g, self.D, self.N, self.H, self.hd
        W = self._W
        cd = self.cdt
        # pixel unshuffle of the output gradient -> [B*N, nout*ps*ps]
        do = dyout.to(cd).reshape(B, self.nout, g, ps, g, ps).permute(0, 2, 4, 1, 3, 5).reshape(B * N, -1).contiguous()
        outw = W(self.outc.weight).reshape(self.outc.weight.shape[0], 256)
        vt.colsum_bf16(do, self.outc.bias.grad)
        gemm.wgrad(do, s["n3"], self.outc.weight.grad)
        dn3 = gemm.mm(do, outw)
        _, dn2, _, _, _ = vt.ln_bwd(dn3, s["n2r"], s["sn3"], self.neck[3].weight, want_dx=False, want_dxb=True,
                                    out_dw=self.neck[3].weight.grad, out_db=self.neck[3].bias.grad)
        cw = W(self.neck[2].weight)
        if self.NECK_HIP and dn2.is_cuda and dn2.dtype == torch.bfloat16 and s["n1"].dtype == torch.bfloat16:
            # data gradient = 3x3 conv of dy with the flipped, transposed weights (same MFMA kernel);
            # weight gradient = the implicit-GEMM wgrad kernel (conv_train.hip), accumulated into a
            # zeroed slice of the flat gradient
            dn2h = dn2.reshape(B, g, g, 256).contiguous()
            self._neck_pcT.refresh(cw.float().flip(2, 3).transpose(0, 1).contiguous())
            dn1 = fused_conv2d(dn2h, self._neck_pcT).view(B * N, 256)
            gw = self.neck[2].weight.grad
            gw.zero_()
            conv_wgrad(s["n1"].view(B, g, g, 256).contiguous(), dn2h, ks=3, cin_valid=256, cout_valid=256, dw=gw)
        else:
            dn2i = dn2.view(B, g, g, 256).permute(0, 3, 1, 2)
            dn1i, dcw, _ = torch.ops.aten.convolution_backward(dn2i, s["n1i"], cw, None, [1, 1], [1, 1], [1, 1], False,
                                                               [0, 0], 1, [True, True, False])
            self.neck[2].weight.grad.copy_(dcw)
            dn1 = dn1i.permute(0, 2, 3, 1).reshape(B * N, 256).contiguous()
        _, dn0, _, _, _ = vt.ln_bwd(dn1, s["n0"], s["sn1"], self.neck[1].weight, want_dx=False, want_dxb=True,
                                    out_dw=self.neck[1].weight.grad, out_db=self.neck[1].bias.grad)
        n0w = W(self.neck[0].weight).reshape(256, D)
        gemm.wgrad(dn0, s["t_last"], self.neck[0].weight.grad)
        G = gemm.mm(dn0, n0w).float()  # d t_out of the last block (fp32 residual-stream gradient)
        ready([self.outc.weight, self.outc.bias, self.neck[3].weight, self.neck[3].bias, self.neck[2].weight,
               self.neck[1].weight, self.neck[1].bias, self.neck[0].weight])
        for i in range(len(self.blocks) - 1, -1, -1):
            G = self._block_bwd(self.blocks[i], s["blocks"][i], G)
            ready(list(self.blocks[i].p.values()))
        # patch embedding + position embedding
        vt._colsum(G.view(B, N * D), self.pos.grad.view(-1))
        Gb, _ = vt.scale_cast(G, dtype=cd, out_col=self.pe[1].grad)
        gemm.wgrad(Gb, s["patches"], self.pe[0].grad)
        self._join_side()
        ready([self.pos, self.pe[0], self.pe[1]])
        self._saved = None

    def _block_bwd(self, b: _Blk, s: dict, G: torch.Tensor) -> torch.Tensor:
        B, N, D, H, hd = self.B, self.N, self.D, self.H, self.hd
        w, p = b.w, b.p
        kb = s["keep"]
        # MLP: t_out = t_mid + k m
        dm, _ = vt.scale_cast(G, kb, N, dtype=self.cdt, out_col=p["l2_b"].grad)
        self._off_path(lambda: gemm.wgrad(dm, s["g"], p["l2_w"].grad), dm)
        # lin2 dgrad with the GELU backward and lin1's bias gradient in the GEMM epilogue
        df = gemm.mm_dgelu(dm, w["l2_w"], s["f"], out_db=p["l1_b"].grad)
        self._off_path(lambda: gemm.wgrad(df, s["h2"], p["l1_w"].grad), df)
        dh2 = gemm.mm(df, w["l1_w"])
        dt_mid, _, _, _, _ = vt.ln_bwd(dh2, s["t_mid"], s["st2"], p["n2w"], r1=G, out_dw=p["n2w"].grad,
                                       out_db=p["n2b"].grad)
        # attention: t_mid = t_in + k y
        dy, _ = vt.scale_cast(dt_mid, kb, N, dtype=self.cdt, out_col=p["proj_b"].grad)
        self._off_path(lambda: gemm.wgrad(dy, s["a"].reshape(B * N, D), p["proj_w"].grad), dy)
        da = gemm.mm(dy, w["proj_w"]).view(B, N, H, hd)
        qkv = s["qkv"]
        dqkv = torch.empty(B, N, 3, H, hd, device=G.device, dtype=self.cdt)
        dq, _, _, drh, drw = vt.attn_bwd(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], s["a"], da, s["lse"], self.scale,
                                         s["rel_h"], s["rel_w"], dk=dqkv[:, :, 1], dv=dqkv[:, :, 2])
        if self.cuda:  # relpos.hip: dq + dq_rel -> the bf16 q slot, table grads gathered in place
            vt.relpos_bwd_(qkv[:, :, 0], s["Rh"], s["Rw"], drh, drw, dq, dqkv[:, :, 0], p["rph"].grad, p["rpw"].grad,
                           self.rel_idx)
        else:
            dq_rel, dRh, dRw = self._rel_bwd(qkv[:, :, 0], s["Rh"], s["Rw"], drh, drw)
            dqkv[:, :, 0] = (dq + dq_rel).to(self.cdt)
            self._table_grad(dRh, p["rph"].grad)
            self._table_grad(dRw, p["rpw"].grad)
        dqkv2 = dqkv.view(B * N, 3 * D)
        def qkv_grads():
            vt.colsum_bf16(dqkv2, p["qkv_b"].grad)
            gemm.wgrad(dqkv2, s["h1"], p["qkv_w"].grad)

        self._off_path(qkv_grads, dqkv2)
        dh1 = gemm.mm(dqkv2, w["qkv_w"])
        dt_in, _, _, _, _ = vt.ln_bwd(dh1, s["t_in"], s["st1"], p["n1w"], r1=dt_mid, out_dw=p["n1w"].grad,
                                      out_db=p["n1b"].grad)
        return dt_in

    # ------------------------------------------------------------------ step
    def loss_and_backward(self, x: torch.Tensor, lbl: torch.Tensor, keep: torch.Tensor | None = None,
                          on_params_ready=None):
        from ..ops import train_ops

        y = self.forward(x, keep)
        if self.cuda:
            loss, dy = train_ops.seg_loss_and_grad(y, lbl)
        else:
            yr = y.detach().float().requires_grad_(True)
            loss = train_ops.seg_loss_ref(yr, lbl)
            (dy,) = torch.autograd.grad(loss, yr)
            loss = loss.detach()
        self.backward(dy, on_params_ready)
        return loss


def stochastic_depth_keep(B: int, nlay: int, rdrop: float, device, generator=None) -> torch.Tensor:
    """cellpose 4 ``Transformer.forward``: layer i of sample b is dropped with probability
    ``linspace(0, rdrop, nlay)[i]``.  Returns the 0/1 keep mask [B, nlay] (fp32)."""
    r = torch.rand(B, nlay, generator=generator).to(device)
    return (r >= torch.linspace(0, rdrop, nlay, device=device)[None]).float()
