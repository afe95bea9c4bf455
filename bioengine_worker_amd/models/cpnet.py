"""Cellpose CPnet (cyto3-style residual U-Net with style vector), MI355X-native.

Two views of the same network:

* :class:`CPnet` — an ``nn.Module`` whose module tree and parameter names mirror cellpose 3's
  ``CPnet`` (``downsample.down.res_down_k``, ``upsample.up.res_up_k``, ``make_style``, ``output``,
  ``diam_mean``/``diam_labels``), so a cellpose ``state_dict`` loads unchanged.  It is the fp32
  PyTorch oracle and the autograd path for training.  The architecture is re-derived from the
  cellpose algorithm (the reference only reaches it through the EXT ``cellpose==3.1.1.2`` pin,
  ``apps/model-runner/runtime_deployment.py:19``; cyto3 named at
  ``apps/cellpose-finetuning/main.py:2234``).
* :class:`CPnetEngine` — the inference engine: NHWC bf16 activations, every conv a single fused
  HIP kernel launch (BN fold + ReLU + style shift + skip add + maxpool/upsample in the loader,
  residual add + bias in the epilogue), style vector from a fused HIP reduction.

Default channel plan: ``nbase = [2, 32, 64, 128, 256]``, 3 outputs (dY, dX, cellprob).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

import os

from ..ops import conv as convops
from ..ops import conv_pair as pairops
from ..ops import style as styleops


def _norm(c: int, kind: str) -> nn.Module:
    if kind == "batch":
        return nn.BatchNorm2d(c, eps=1e-5, momentum=0.05)
    if kind == "group":
        g = 8 if c % 8 == 0 else 1
        return nn.GroupNorm(g, c, eps=1e-5)
    raise ValueError(kind)


def batchconv(cin, cout, sz, norm="batch"):
    return nn.Sequential(_norm(cin, norm), nn.ReLU(inplace=True), nn.Conv2d(cin, cout, sz, padding=sz // 2))


def batchconv0(cin, cout, sz, norm="batch"):
    return nn.Sequential(_norm(cin, norm), nn.Conv2d(cin, cout, sz, padding=sz // 2))


class resdown(nn.Module):
    def __init__(self, cin, cout, sz, norm="batch"):
        super().__init__()
        self.conv = nn.Sequential()
        self.proj = batchconv0(cin, cout, 1, norm)
        for t in range(4):
            self.conv.add_module(f"conv_{t}", batchconv(cin if t == 0 else cout, cout, sz, norm))

    def forward(self, x):
        x = self.proj(x) + self.conv[1](self.conv[0](x))
        x = x + self.conv[3](self.conv[2](x))
        return x


class downsample(nn.Module):
    def __init__(self, nbase, sz, norm="batch"):
        super().__init__()
        self.down = nn.Sequential()
        self.maxpool = nn.MaxPool2d(2, 2)
        for n in range(len(nbase) - 1):
            self.down.add_module(f"res_down_{n}", resdown(nbase[n], nbase[n + 1], sz, norm))

    def forward(self, x):
        xd = []
        for n in range(len(self.down)):
            y = self.maxpool(xd[n - 1]) if n > 0 else x
            xd.append(self.down[n](y))
        return xd


class batchconvstyle(nn.Module):
    def __init__(self, cin, cout, style_channels, sz, norm="batch"):
        super().__init__()
        self.concatenation = False
        self.conv = batchconv(cin, cout, sz, norm)
        self.full = nn.Linear(style_channels, cout)

    def forward(self, style, x, y=None):
        if y is not None:
            x = x + y
        feat = self.full(style)
        return self.conv(x + feat.unsqueeze(-1).unsqueeze(-1))


class resup(nn.Module):
    def __init__(self, cin, cout, style_channels, sz, norm="batch"):
        super().__init__()
        self.conv = nn.Sequential()
        self.conv.add_module("conv_0", batchconv(cin, cout, sz, norm))
        self.conv.add_module("conv_1", batchconvstyle(cout, cout, style_channels, sz, norm))
        self.conv.add_module("conv_2", batchconvstyle(cout, cout, style_channels, sz, norm))
        self.conv.add_module("conv_3", batchconvstyle(cout, cout, style_channels, sz, norm))
        self.proj = batchconv0(cin, cout, 1, norm)

    def forward(self, x, y, style):
        x = self.proj(x) + self.conv[1](style, self.conv[0](x), y=y)
        x = x + self.conv[3](style, self.conv[2](style, x))
        return x


class make_style(nn.Module):
    def __init__(self):
        super().__init__()
        self.flatten = nn.Flatten()

    def forward(self, x0):
        style = F.avg_pool2d(x0, kernel_size=x0.shape[2:])
        style = self.flatten(style)
        return style / torch.sum(style ** 2, dim=1, keepdim=True) ** 0.5


class upsample(nn.Module):
    def __init__(self, nbase, sz, norm="batch"):
        super().__init__()
        self.upsampling = nn.Upsample(scale_factor=2, mode="nearest")
        self.up = nn.Sequential()
        for n in range(1, len(nbase)):
            self.up.add_module(f"res_up_{n - 1}", resup(nbase[n], nbase[n - 1], nbase[-1], sz, norm))

    def forward(self, style, xd):
        x = self.up[-1](xd[-1], xd[-1], style)
        for n in range(len(self.up) - 2, -1, -1):
            x = self.upsampling(x)
            x = self.up[n](x, xd[n], style)
        return x


class CPnet(nn.Module):
    """cellpose-3 compatible CPnet (module/parameter names match cellpose ``CPnet``)."""

    def __init__(self, nbase=(2, 32, 64, 128, 256), nout=3, sz=3, diam_mean=30.0, norm="batch", style_on=True):
        super().__init__()
        nbase = list(nbase)
        self.nbase = nbase
        self.nout = nout
        self.sz = sz
        self.norm_kind = norm
        self.style_on = style_on
        self.downsample = downsample(nbase, sz, norm)
        nbaseup = nbase[1:] + [nbase[-1]]
        self.upsample = upsample(nbaseup, sz, norm)
        self.make_style = make_style()
        self.output = batchconv(nbaseup[0], nout, 1, norm)
        self.diam_mean = nn.Parameter(torch.ones(1) * diam_mean, requires_grad=False)
        self.diam_labels = nn.Parameter(torch.ones(1) * diam_mean, requires_grad=False)

    @property
    def nchan(self):
        return self.nbase[0]

    def forward(self, data):
        T0 = self.downsample(data)
        style = self.make_style(T0[-1])
        style0 = style
        if not self.style_on:
            style = style * 0
        T1 = self.upsample(style, T0)
        T1 = self.output(T1)
        return T1, style0, T0

    def randomize_(self, seed: int = 0) -> "CPnet":
        """Random-init weights *and* BN running statistics (the benches run on random-init models)."""
        g = torch.Generator().manual_seed(seed)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                fan_in = m.in_channels * m.kernel_size[0] * m.kernel_size[1]
                m.weight.data = torch.randn(m.weight.shape, generator=g) * (1.0 / fan_in) ** 0.5
                if m.bias is not None:
                    m.bias.data = torch.randn(m.bias.shape, generator=g) * 0.01
            elif isinstance(m, nn.Linear):
                m.weight.data = torch.randn(m.weight.shape, generator=g) * (1.0 / m.in_features) ** 0.5
                m.bias.data = torch.randn(m.bias.shape, generator=g) * 0.01
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data = 1.0 + 0.1 * torch.randn(m.weight.shape, generator=g)
                m.bias.data = 0.1 * torch.randn(m.bias.shape, generator=g)
                m.running_mean.data = 0.1 * torch.randn(m.running_mean.shape, generator=g)
                m.running_var.data = 1.0 + 0.1 * torch.rand(m.running_var.shape, generator=g)
            elif isinstance(m, nn.GroupNorm):
                m.weight.data = 1.0 + 0.1 * torch.randn(m.weight.shape, generator=g)
                m.bias.data = 0.1 * torch.randn(m.bias.shape, generator=g)
        return self


# ----------------------------------------------------------------------------------------------
# Fused inference engine
# ----------------------------------------------------------------------------------------------

def _bn_fold(bn: nn.Module, device) -> tuple[torch.Tensor, torch.Tensor]:
    if isinstance(bn, nn.BatchNorm2d):
        s = bn.weight.detach().float() / torch.sqrt(bn.running_var.detach().float() + bn.eps)
        t = bn.bias.detach().float() - bn.running_mean.detach().float() * s
        return s.to(device).contiguous(), t.to(device).contiguous()
    raise TypeError("CPnetEngine folds eval-mode BatchNorm only; GroupNorm nets run the autograd path")


def _pad_vec(v: torch.Tensor, n: int, fill: float) -> torch.Tensor:
    if v.numel() == n:
        return v
    out = torch.full((n,), fill, dtype=v.dtype, device=v.device)
    out[: v.numel()] = v
    return out


class _FConv:
    """One fused conv: packed weights + folded pre-activation affine."""

    def __init__(self, seq: nn.Sequential, relu: bool, device, cin_pad=None, cout_pad_to=None):
        bn, conv = seq[0], seq[-1]
        self.pc = convops.PackedConv.from_weight(conv.weight, conv.bias, cin_pad=cin_pad, cout_pad_to=cout_pad_to).to(device)
        s, t = _bn_fold(bn, device)
        self.scale = _pad_vec(s, self.pc.cin_pad, 0.0)
        self.shift = _pad_vec(t, self.pc.cin_pad, 0.0)
        self.relu = relu

    def __call__(self, x, *, x2=None, shift=None, residual=None, inmode="none", out_nchw_f32=False, cout_valid=None):
        return convops.fused_conv2d(x, self.pc, x2=x2, scale=self.scale, shift=self.shift if shift is None else shift,
                                    relu=self.relu, residual=residual, inmode=inmode, out_nchw_f32=out_nchw_f32,
                                    cout_valid=cout_valid)


class _PPConv:
    """A 3x3 conv on the ping-pong implicit-GEMM kernel (ops/gemm_pp.py): weights [Cout][3][3][Cin]."""

    def __init__(self, conv: nn.Conv2d, device):
        from ..ops import gemm_pp as ppops

        self.cout = conv.weight.shape[0]
        self.wp = ppops.pack_conv3(conv.weight).to(device)
        self.bias = None if conv.bias is None else conv.bias.detach().float().to(device).contiguous()
        cfg = os.environ.get("BE_CPNET_PP_CFG")
        self.cfg = None if cfg is None else int(cfg)


def _igc(x, pk, **kw):
    """(out, aout) of one deep 3x3 conv on the implicit-GEMM path the engine was built with."""
    if isinstance(pk, _PPConv):
        from ..ops import gemm_pp as ppops

        return ppops.conv3(x, pk.wp, pk.bias, cfg=pk.cfg, **kw)
    from ..ops import conv_igemm as igops

    return igops.conv3_igemm(x, pk, **kw)


class CPnetEngine:
    """Inference engine for an eval-mode (BatchNorm) :class:`CPnet`.

    ``forward(x)``: ``x`` NHWC bf16 [B, H, W, cin_pad] (H, W multiples of 8) ->
    (flows+cellprob NCHW fp32 [B, nout, H, W], style fp32 [B, nbase[-1]]).
    """

    def __init__(self, net: CPnet, device):
        net = net.eval()
        self.device = torch.device(device)
        self.nout = net.nout
        self.nchan = net.nchan
        self.cin_pad = convops._round_up(net.nchan, 8)
        d = self.device
        self.down = []
        for n, blk in enumerate(net.downsample.down):
            cin_pad = self.cin_pad if n == 0 else None
            self.down.append(dict(
                proj=_FConv(blk.proj, False, d, cin_pad),
                c0=_FConv(blk.conv[0], True, d, cin_pad),
                c1=_FConv(blk.conv[1], True, d),
                c2=_FConv(blk.conv[2], True, d),
                c3=_FConv(blk.conv[3], True, d),
            ))
        self.up = []
        for blk in net.upsample.up:
            e = dict(proj=_FConv(blk.proj, False, d), c0=_FConv(blk.conv[0], True, d))
            for k in (1, 2, 3):
                bcs = blk.conv[k]
                e[f"c{k}"] = _FConv(bcs.conv, True, d)
                e[f"full{k}"] = (bcs.full.weight.detach().float().to(d), bcs.full.bias.detach().float().to(d))
            self.up.append(e)
        self.out = _FConv(net.output, True, d, cout_pad_to=16)
        self.style_on = net.style_on
        # Stack every style Linear into one GEMM: feats = style @ Wall^T + ball, then per-conv
        # shift[n, c] = feat[n, c] * s[c] + t[c]  (batchconvstyle folded into the next conv prologue).
        ws, bs, ss, ts = [], [], [], []
        self._feat_slices = []
        off = 0
        for i, e in enumerate(self.up):
            for k in (1, 2, 3):
                w, b = e[f"full{k}"]
                conv = e[f"c{k}"]
                ws.append(w); bs.append(b)
                ss.append(conv.scale[: w.shape[0]]); ts.append(conv.shift[: w.shape[0]])
                self._feat_slices.append((i, k, off, w.shape[0]))
                off += w.shape[0]
        self.style_w = torch.cat(ws, 0).contiguous()
        self.style_b = torch.cat(bs, 0).contiguous()
        self.style_s = torch.cat(ss, 0).contiguous()
        self.style_t = torch.cat(ts, 0).contiguous()
        self.pair = self._build_pairs(net) if os.environ.get("BE_CPNET_PAIR", "1") != "0" else {}
        # deepest level on the implicit-GEMM kernels (BE_CPNET_IGEMM=1, BE_CPNET_IGEMM_LEVELS=3 by
        # default): whole-network A/B on MI355X 14.38 vs 14.62 ms per 288 tiles for the per-layer
        # path (profiles/r04/conv/engine_ab_L3.jsonl).  On both deep levels the producer-side
        # activated copies cost more HBM traffic than the DMA-fed main loop saves at 56^2 (14.68;
        # engine_ab_v2.jsonl); BE_CPNET_IGEMM=0 / pp select the per-layer / ping-pong kernels
        self.ig_kind = os.environ.get("BE_CPNET_IGEMM", "1")
        self.ig = self._build_igemm(net) if self.ig_kind in ("1", "pp") else {}
        # output layer fused into the last half-block's epilogue (ops/conv_pair.py HeadSpec)
        self.head = None
        if ("up", 0, 1) in self.pair and self.out.relu and self.nout <= 16 and os.environ.get("BE_CPNET_HEAD", "1") != "0":
            self.head = pairops.HeadSpec.build(self.out.scale, self.out.shift, net.output[-1].weight.to(d),
                                               None if net.output[-1].bias is None else net.output[-1].bias.to(d))

    # ------------------------------------------------------------------ fused half-blocks
    def _build_pairs(self, net: CPnet) -> dict:
        """Fused two-conv kernels (ops/conv_pair.py) for the 32/64-channel levels, where the
        per-layer path is HBM bound.  Keys: ("down", n, 0|1) / ("up", i, 0|1)."""
        nb = list(net.nbase)
        if len(nb) < 3 or nb[1] != 32 or nb[2] != 64 or self.cin_pad != 8 or net.sz != 3:
            return {}
        pairs = {}

        def spec(a: _FConv, b: _FConv, inmode="none", proj: _FConv | None = None, style_b=False):
            bias = b.pc.bias if b.pc.bias is not None else torch.zeros(b.pc.cout, device=self.device)
            if proj is not None and proj.pc.bias is not None:
                bias = bias + proj.pc.bias
            tb = None if style_b else pairops.fold_bias(b.shift, b.scale, a.pc.bias).contiguous()
            return pairops.PairSpec(pa=a.pc, pb=b.pc, sa=a.scale, ta=a.shift, sb=b.scale, tb=tb,
                                    bias=bias.float().contiguous(), inmode=inmode,
                                    pp=None if proj is None else proj.pc, sp=None if proj is None else proj.scale,
                                    tp=None if proj is None else proj.shift)

        d0, d1 = self.down[0], self.down[1]
        pairs[("down", 0, 0)] = spec(d0["c0"], d0["c1"], "none", proj=d0["proj"])
        pairs[("down", 0, 1)] = spec(d0["c2"], d0["c3"])
        pairs[("down", 1, 0)] = spec(d1["c0"], d1["c1"], "pool2")
        pairs[("down", 1, 1)] = spec(d1["c2"], d1["c3"])
        nup = len(self.up)
        for i in (0, 1):
            if i >= nup - 1:
                continue
            e = self.up[i]
            pairs[("up", i, 0)] = spec(e["c0"], e["c1"], "up2", style_b=True)
            pairs[("up", i, 1)] = spec(e["c2"], e["c3"], style_b=True)
            # the per-image actB shifts come out of the stacked style GEMM: fold convA's bias into
            # their constant term there (t + s * biasA), once, instead of per forward
            for (ii, k, off, c) in self._feat_slices:
                if ii == i and k in (1, 3):
                    prev = e["c0"] if k == 1 else e["c2"]
                    if prev.pc.bias is not None:
                        self.style_t[off: off + c] += self.style_s[off: off + c] * prev.pc.bias[:c].to(self.device)
        # BE_CPNET_PAIR_LEVELS (default "0,1"): the levels (0 = 32 ch at full res, 1 = 64 ch) that
        # run on the fused pair kernels; the others fall to the igemm / per-layer paths (A/B)
        keep = {int(v) for v in os.environ.get("BE_CPNET_PAIR_LEVELS", "0,1").split(",") if v.strip()}
        pairs = {k: v for k, v in pairs.items() if k[1] in keep}
        for key, sp in pairs.items():
            has_x2 = key[0] == "up" and key[2] == 0
            res = "none" if key == ("down", 0, 0) else ("up2" if has_x2 else "full")
            assert sp.supports(has_x2, res), key
        return pairs

    def _build_igemm(self, net: CPnet) -> dict:
        """Implicit-GEMM 3x3 convs (ops/conv_igemm.py) for the deep levels the fused pairs do not
        cover: every 3x3 conv whose input is NOT resampled (pool2 / up2 inputs stay on the
        per-layer kernel, which writes its consumer's activated input instead).  Keys:
        ("down", n, k) / ("up", i, k)."""
        from ..ops import conv_igemm as igops
        from ..ops import gemm_pp as ppops

        ig = {}

        def add(key, conv: nn.Conv2d):
            cout, cin, kh, _ = conv.weight.shape
            if self.ig_kind == "pp":
                if kh == 3 and ppops.conv3_supported(cin, cout):
                    ig[key] = _PPConv(conv, self.device)
            elif kh == 3 and cin % 16 == 0 and cout % 64 == 0:
                ig[key] = igops.IgemmConv.from_weight(conv.weight, conv.bias).to(self.device)

        nup = len(net.upsample.up)
        for n, blk in enumerate(net.downsample.down):
            if ("down", n, 0) in self.pair or n == 0:
                continue
            for k in (1, 2, 3):
                add(("down", n, k), blk.conv[k][-1])
        for i, blk in enumerate(net.upsample.up):
            if ("up", i, 0) in self.pair:
                continue
            if i == nup - 1:
                add(("up", i, 0), blk.conv[0][-1])
            for k in (1, 2, 3):
                add(("up", i, k), blk.conv[k].conv[-1])
        # a level runs on the igemm path only when all of its 3x3 convs do; BE_CPNET_IGEMM_LEVELS
        # (e.g. "3") restricts it to the listed down levels and the up blocks at their resolution
        levels = {}
        for (kind, idx, k) in ig:
            levels.setdefault((kind, idx), set()).add(k)
        full = {lv for lv, ks in levels.items() if ks >= {1, 2, 3}}
        only = os.environ.get("BE_CPNET_IGEMM_LEVELS", "3")
        if only:
            keep = {int(v) for v in only.split(",") if v.strip()}
            # up block i writes level i's resolution (the last one stays at the deepest level's)
            full = {lv for lv in full if lv[1] in keep}
        return {key: v for key, v in ig.items() if (key[0], key[1]) in full}

    def _ig_level(self, kind: str, idx: int, x: torch.Tensor, H: int, W: int) -> bool:
        from ..ops import conv_igemm as igops

        pk = self.ig.get((kind, idx, 1))
        if pk is None or not x.is_cuda:
            return False
        if isinstance(pk, _PPConv):
            return True  # no halo budget: any image geometry
        return igops.supported(x.shape[0], H, W, pk.cout, pk.bn)

    def _down_ig(self, n: int, e: dict, src: torch.Tensor, next_act=None) -> torch.Tensor:
        """resdown on the igemm path: every conv's output is written already activated for its
        consumer (producer-side pre-activation), so the 3x3 convs stage their inputs by DMA.
        ``next_act`` = (scale, shift) of the following up block's first conv, which reads this
        block's output through the igemm path too (written as a second, activated copy)."""
        ig = self.ig
        proj = e["proj"](src, inmode="pool2")
        c1, c2, c3 = e["c1"], e["c2"], e["c3"]
        ha = convops.fused_conv2d(src, e["c0"].pc, scale=e["c0"].scale, shift=e["c0"].shift, relu=True, inmode="pool2",
                                  post_scale=c1.scale, post_shift=c1.shift, post_relu=True)
        x1, x1a = _igc(ha, ig[("down", n, 1)], residual=proj, ascale=c2.scale, ashift=c2.shift)
        _, h2a = _igc(x1a, ig[("down", n, 2)], want_out=False, ascale=c3.scale, ashift=c3.shift)
        if next_act is None:
            xd, _ = _igc(h2a, ig[("down", n, 3)], residual=x1)
            return xd, None
        return _igc(h2a, ig[("down", n, 3)], residual=x1, ascale=next_act[0], ashift=next_act[1])

    def _up_ig(self, i: int, e: dict, xcur: torch.Tensor, y: torch.Tensor, shifts: dict, xcur_act=None):
        ig = self.ig
        c1, c2, c3 = e["c1"], e["c2"], e["c3"]
        if ("up", i, 0) in ig:  # same resolution: c0 on the igemm path, its input activated upstream
            proj = e["proj"](xcur)
            _, h0a = _igc(xcur_act, ig[("up", i, 0)], residual=y, want_out=False, ascale=c1.scale,
                                       ashift=shifts[(i, 1)])
        else:
            proj = e["proj"](xcur, inmode="up2")
            h0a = convops.fused_conv2d(xcur, e["c0"].pc, scale=e["c0"].scale, shift=e["c0"].shift, relu=True,
                                       inmode="up2", residual=y, post_scale=c1.scale, post_shift=shifts[(i, 1)],
                                       post_relu=True)
        x1, x1a = _igc(h0a, ig[("up", i, 1)], residual=proj, ascale=c2.scale, ashift=shifts[(i, 2)])
        _, h2a = _igc(x1a, ig[("up", i, 2)], want_out=False, ascale=c3.scale, ashift=shifts[(i, 3)])
        out, _ = _igc(h2a, ig[("up", i, 3)], residual=x1)
        return out

    def _style_shifts(self, style: torch.Tensor) -> dict:
        st = style if self.style_on else torch.zeros_like(style)
        return self._split_shifts(styleops.style_shifts(st, self.style_w, self.style_b, self.style_s, self.style_t))

    def _split_shifts(self, shifts_all: torch.Tensor) -> dict:
        out = {}
        for (i, k, off, c) in self._feat_slices:  # row-strided views: the conv reads them in place
            out[(i, k)] = shifts_all[:, off: off + c]
        return out

    @torch.no_grad()
    def forward(self, x: torch.Tensor):
        xd = []
        h = x
        P = self.pair
        nup = len(self.up)
        top_act = None  # the deepest level's output, activated for up[nup-1].c0 (igemm path)
        for n, e in enumerate(self.down):
            im = "pool2" if n > 0 else "none"
            src = x if n == 0 else xd[-1]
            if n > 0 and ("down", n, 1) in self.ig and self._ig_level("down", n, src, src.shape[1] // 2,
                                                                       src.shape[2] // 2):
                last = n == len(self.down) - 1 and ("up", nup - 1, 0) in self.ig
                nxt = (self.up[nup - 1]["c0"].scale, self.up[nup - 1]["c0"].shift) if last else None
                xdn, top_act = self._down_ig(n, e, src, nxt)
                xd.append(xdn)
                continue
            if ("down", n, 0) in P:
                if n == 0:  # stem: projection computed inside the fused kernel (K concatenation)
                    x1 = pairops.conv_pair(src, P[("down", 0, 0)])
                else:
                    x1 = pairops.conv_pair(src, P[("down", n, 0)], res=e["proj"](src, inmode=im), res_mode="full")
                xd.append(pairops.conv_pair(x1, P[("down", n, 1)], res=x1, res_mode="full"))
                continue
            proj = e["proj"](src, inmode=im)
            h = e["c0"](src, inmode=im)
            x1 = e["c1"](h, residual=proj)
            h = e["c2"](x1)
            xd.append(e["c3"](h, residual=x1))
        style, shifts_all = styleops.style_and_shifts(xd[-1], self.style_w, self.style_b, self.style_s, self.style_t,
                                                      self.style_on)
        shifts = self._split_shifts(shifts_all)
        xcur = xd[-1]
        for i in range(nup - 1, -1, -1):
            e = self.up[i]
            im = "none" if i == nup - 1 else "up2"
            y = xd[i] if i < nup - 1 else xd[-1]
            H2, W2 = (xcur.shape[1], xcur.shape[2]) if i == nup - 1 else (2 * xcur.shape[1], 2 * xcur.shape[2])
            if ("up", i, 1) in self.ig and (("up", i, 0) not in self.ig or top_act is not None) and \
                    self._ig_level("up", i, xcur, H2, W2):
                xcur = self._up_ig(i, e, xcur, y, shifts, top_act if i == nup - 1 else None)
                continue
            if ("up", i, 0) in P:
                # 1x1 projection commutes with nearest upsampling: run it at half resolution and
                # let the fused kernel read it through an up2 residual
                proj_lr = e["proj"](xcur)
                x1 = pairops.conv_pair(xcur, P[("up", i, 0)], tb=shifts[(i, 1)], x2=y, res=proj_lr, res_mode="up2")
                if i == 0 and self.head is not None:
                    y = pairops.conv_pair_head(x1, P[("up", 0, 1)], self.head, ta=shifts[(0, 2)], tb=shifts[(0, 3)],
                                               res=x1)
                    return y, style
                xcur = pairops.conv_pair(x1, P[("up", i, 1)], ta=shifts[(i, 2)], tb=shifts[(i, 3)], res=x1,
                                         res_mode="full")
                continue
            proj = e["proj"](xcur, inmode=im)
            # the skip add (conv1's input is c0(x) + y) runs in c0's residual epilogue, so conv1
            # reads one tensor instead of two (the two-input variant was ~1.7x slower per layer)
            h0 = e["c0"](xcur, inmode=im, residual=y)
            x1 = e["c1"](h0, shift=shifts[(i, 1)], residual=proj)
            h2 = e["c2"](x1, shift=shifts[(i, 2)])
            xcur = e["c3"](h2, shift=shifts[(i, 3)], residual=x1)
        y = self.out(xcur, out_nchw_f32=True, cout_valid=self.nout)
        return y, style

    __call__ = forward


def to_nhwc_input(x_nchw: torch.Tensor, cin_pad: int) -> torch.Tensor:
    """NCHW float -> NHWC bf16 with channels zero-padded to ``cin_pad``."""
    N, C, H, W = x_nchw.shape
    out = torch.zeros(N, H, W, cin_pad, dtype=torch.bfloat16, device=x_nchw.device)
    out[..., :C] = x_nchw.permute(0, 2, 3, 1)
    return out
