"""Hand-written CPnet training engine: forward + backward of the Cellpose U-Net on the HIP kernels.

The reference fine-tunes through PyTorch autograd inside the cellpose package
(``apps/cellpose-finetuning/main.py:1483-1546``: ``net(x)`` -> ``_loss_fn_seg`` -> ``backward`` ->
AdamW).  On MI355X the autograd path launches ~1,600 small kernels per step (BatchNorm, casts,
adds, MIOpen convs; ``profiles/``), so this engine runs the whole training step as ~250 fused
launches on activations that live in NHWC bf16:

forward, per BN input ("site"): one statistics launch (batch mean/var -> conv-prologue affine, running
stats), then one fused conv launch per conv reading the pre-BN tensor (BN affine, ReLU, max-pool /
upsample, skip add and style feature folded into the conv's halo loader; residual add + bias in the
epilogue) — the same kernel as inference, so no activation is materialised twice.

backward, per conv: dgrad = the forward conv kernel on dOut with flipped/transposed weights;
wgrad = MFMA implicit GEMM over pixels with the activation recomputed from the saved pre-BN input;
per site: one reduction (dgamma, dbeta, BN coefficients, style-feature grad) and one apply that
routes the input gradient through max-pool / upsample adjoints into the (shared) source gradients.

Parameters and gradients are the :class:`~bioengine_worker_amd.parallel.ddp.FlatParams` buffers:
every kernel writes its parameter gradient straight into the flat fp32 grad buffer, so the fused
AdamW and the bucketed RCCL all-reduce work unchanged.  The engine's schedule is static for a
given (batch, crop) shape, which makes the whole step capturable in a HIP graph.

On CPU every op runs its PyTorch fp32 reference, so the engine's gradients are checked against
autograd exactly (tests/test_cpnet_engine_cpu.py).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch
import torch.nn as nn

from ..models.cpnet import CPnet
from ..ops import conv as convops
from ..ops import conv_train as ct
from ..ops import train_ops
from ..parallel.ddp import FlatParams


@dataclass
class _Conv:
    """One conv of the net: fp32 master views + packed bf16 layouts for forward and dgrad."""

    name: str
    conv: nn.Conv2d
    ks: int
    cin: int
    cin_pad: int
    cout: int
    fwd: convops.PackedConv
    bwd: convops.PackedConv | None
    dw: torch.Tensor        # grad view [cout, cin, k, k]
    db: torch.Tensor | None


@dataclass
class _Site:
    bn: ct.BnSite
    units: list
    C: int


@dataclass
class _Block:
    kind: str                      # "down" / "up"
    idx: int
    convs: dict                    # proj, c0..c3 -> _Conv
    sites: list                    # 4 _Site: (proj, c0), c1, c2, c3
    full: list = field(default_factory=list)  # up blocks: Linear modules of c1..c3 (style)


def _packed_meta(conv: nn.Conv2d, cin_pad: int, cout_pad_to: int | None = None, transpose: bool = False):
    """PackedConv geometry (no data) for the forward or the dgrad (transposed) layout."""
    cout, cin, ks, _ = conv.weight.shape
    if transpose:
        cout, cin = cin_pad, cout  # dgrad: outputs = layer inputs (padded), inputs = layer outputs
        cin_pad_t = convops._round_up(cin, 8)
        if cin_pad_t % 32 and cin_pad_t != 8:
            cin_pad_t = convops._round_up(cin_pad_t, 32)
        cin_pad = cin_pad_t
    ck, tco = convops.PackedConv.choose(cin_pad, cout)
    cout_k = max(cout, cout_pad_to or 0)
    cout_pad = convops._round_up(cout_k, tco)
    kp = ((ks * ks * ck + 31) // 32) * 32
    return dict(ks=ks, cin=cin, cin_pad=cin_pad, cout=cout, cout_pad=cout_pad, ck=ck, tco=tco, kp=kp)


class CPnetTrainEngine:
    """Static-shape training step for a BatchNorm :class:`CPnet` (batch ``B`` of ``S x S`` crops)."""

    def __init__(self, net: CPnet, fp: FlatParams, B: int, S: int, device, momentum: float = 0.05,
                 act_dtype: torch.dtype | None = None):
        if net.norm_kind not in ("batch", "group"):
            raise ValueError(f"CPnetTrainEngine implements BatchNorm / GroupNorm nets, not {net.norm_kind!r}")
        self.groupnorm = net.norm_kind == "group"
        if S % 16:
            raise ValueError("crop size must be a multiple of 16 (4 pooling levels)")
        self.net = net
        self.fp = fp
        self.B, self.S = B, S
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        # activation storage dtype: bf16 on GPU (the kernels' format); CPU defaults to fp32 (exact oracle)
        # and can emulate the GPU's bf16 storage with act_dtype=torch.bfloat16
        self.act_dtype = act_dtype or (torch.bfloat16 if self.cuda else torch.float32)
        self.momentum = momentum
        self.nout = net.nout
        self.cin_pad = convops._round_up(net.nchan, 8)
        self._convs: list[_Conv] = []
        self._sites: list[_Site] = []
        self._build()
        self._alloc()

    # ------------------------------------------------------------------ construction
    def _mk_conv(self, name, seq: nn.Sequential, cin_pad=None, cout_pad_to=None, need_dgrad=True) -> _Conv:
        conv = seq[-1]
        cout, cin, ks, _ = conv.weight.shape
        cin_pad = cin_pad or cin
        m = _packed_meta(conv, cin_pad, cout_pad_to)
        fwd = convops.PackedConv(w=conv.weight, bias=conv.bias, **m)
        bwd = None
        if need_dgrad:
            mb = _packed_meta(conv, cin_pad, None, transpose=True)
            bwd = convops.PackedConv(w=conv.weight, bias=None, **mb)
        c = _Conv(name, conv, ks, cin, cin_pad, cout, fwd, bwd, conv.weight.grad, conv.bias.grad if conv.bias is not None else None)
        self._convs.append(c)
        return c

    def _mk_site(self, bns: list, relus: list, C: int, c_valid: int | None = None) -> _Site:
        units = []
        for bn, relu in zip(bns, relus):
            units.append(ct.BnUnit(gamma=bn.weight, beta=bn.bias, run_mean=getattr(bn, "running_mean", None),
                                   run_var=getattr(bn, "running_var", None), relu=relu, scale=None, shift=None,
                                   dgamma=bn.weight.grad, dbeta=bn.bias.grad))
        s = _Site(bn=None, units=units, C=C)
        s.c_valid = c_valid or C
        # GroupNorm: groups of the site's norm (shared-input units have the same channel count)
        s.groups = int(bns[0].num_groups) if isinstance(bns[0], nn.GroupNorm) else 0
        self._sites.append(s)
        return s

    def _build(self):
        net = self.net
        self.down: list[_Block] = []
        for n, blk in enumerate(net.downsample.down):
            cin_pad = self.cin_pad if n == 0 else None
            cv = dict(proj=self._mk_conv(f"d{n}.proj", blk.proj, cin_pad),
                      c0=self._mk_conv(f"d{n}.c0", blk.conv[0], cin_pad),
                      c1=self._mk_conv(f"d{n}.c1", blk.conv[1]),
                      c2=self._mk_conv(f"d{n}.c2", blk.conv[2]),
                      c3=self._mk_conv(f"d{n}.c3", blk.conv[3]))
            cin = cv["c0"].cin_pad
            cout = cv["c0"].cout
            sites = [self._mk_site([blk.proj[0], blk.conv[0][0]], [False, True], cin, net.nbase[n] if n == 0 else None),
                     self._mk_site([blk.conv[1][0]], [True], cout),
                     self._mk_site([blk.conv[2][0]], [True], cout),
                     self._mk_site([blk.conv[3][0]], [True], cout)]
            self.down.append(_Block("down", n, cv, sites))
        self.up: list[_Block] = []
        for i, blk in enumerate(net.upsample.up):
            cv = dict(proj=self._mk_conv(f"u{i}.proj", blk.proj), c0=self._mk_conv(f"u{i}.c0", blk.conv[0]))
            for k in (1, 2, 3):
                cv[f"c{k}"] = self._mk_conv(f"u{i}.c{k}", blk.conv[k].conv)
            cin = cv["c0"].cin
            cout = cv["c0"].cout
            sites = [self._mk_site([blk.proj[0], blk.conv[0][0]], [False, True], cin),
                     self._mk_site([blk.conv[1].conv[0]], [True], cout),
                     self._mk_site([blk.conv[2].conv[0]], [True], cout),
                     self._mk_site([blk.conv[3].conv[0]], [True], cout)]
            self.up.append(_Block("up", i, cv, sites, full=[blk.conv[k].full for k in (1, 2, 3)]))
        self.head = self._mk_conv("out", net.output, cout_pad_to=16)
        self.head_site = self._mk_site([net.output[0]], [True], self.head.cin)

    def _alloc(self):
        d, B, S = self.device, self.B, self.S
        f32 = torch.float32
        # ---- BN workspaces (one arena, zeroed once per step) + prologue affines
        sizes = [ct.BnSite.stat_numel(B, s.C, s.groups) for s in self._sites]
        self._bn_scratch = torch.empty(ct.SCRATCH_FLOATS, device=d, dtype=f32) if self.cuda else None
        tot = sum(sizes) + 2 * len(self._sites) + 64
        self._ws_arena = torch.zeros(tot, device=d, dtype=f32)
        off = 0
        tickets = self._ws_arena[sum(sizes):].view(torch.int32)
        for i, (s, n) in enumerate(zip(self._sites, sizes)):
            for u in s.units:
                u.scale = torch.zeros((B, s.C) if s.groups else (s.C,), device=d, dtype=f32)
                u.shift = torch.zeros(B, s.C, device=d, dtype=f32)
            s.bn = ct.BnSite(B, s.C, s.c_valid, s.units, self._ws_arena[off: off + n], tickets[2 * i: 2 * i + 2],
                             momentum=self.momentum, scratch=self._bn_scratch, groups=s.groups)
            off += n
        # ---- packed weights: one bf16 arena + descriptor table (repacked from the fp32 master each step)
        descs, arena_off, max_e = [], 0, 0
        flat_ptr = self.fp.flat.data_ptr()
        entries = []
        for c in self._convs:
            for pc, tr in ((c.fwd, False), (c.bwd, True)):
                if pc is None:
                    continue
                n = pc.cout_pad * (pc.cin_pad // pc.ck) * pc.kp
                src = (c.conv.weight.data_ptr() - flat_ptr) // 4
                descs.append([src, arena_off, c.cout, c.cin, c.ks, pc.cout_pad, pc.cin_pad, pc.ck, pc.kp, int(tr)])
                entries.append((pc, arena_off, n))
                arena_off += (n + 7) // 8 * 8
                max_e = max(max_e, n)
        self._pack_arena = torch.zeros(arena_off, device=d, dtype=torch.bfloat16)
        for pc, o, n in entries:
            pc.wp = self._pack_arena[o: o + n].view(pc.cout_pad, pc.cin_pad // pc.ck, pc.kp)
        self._descs = torch.tensor(descs, dtype=torch.int32, device=d)
        self._ndesc, self._max_e = len(descs), max_e
        # ---- wgrad split-K workspace (largest need over convs)
        need = 0
        for c, H in self._conv_res():
            sp = ct.wgrad_splits(B, H, H, c.cin_pad, max(8, c.cout), c.ks)
            need = max(need, sp * c.cout * c.ks * c.ks * c.cin_pad + sp * c.cout)
        self._wg_ws = torch.empty(max(need, 1), device=d, dtype=f32)
        # style GEMM operands
        self._style_full = [m for blk in self.up for m in blk.full]

    def _conv_res(self):
        S = self.S
        for n, blk in enumerate(self.down):
            H = S >> n
            for c in blk.convs.values():
                yield c, H
        nup = len(self.up)
        for i, blk in enumerate(self.up):
            H = S >> i
            for c in blk.convs.values():
                yield c, H
        yield self.head, S

    # ------------------------------------------------------------------ helpers
    def _pack(self):
        if self.cuda:
            ct.pack_weights(self._descs, self._ndesc, self._max_e, self.fp.flat, self._pack_arena)
        else:  # CPU reference path reads fp32 weights; dgrad uses the flipped/transposed view
            for c in self._convs:
                if c.bwd is not None:
                    c.bwd.w = c.conv.weight.detach().flip(2, 3).transpose(0, 1)
                    if c.bwd.w.shape[0] < c.bwd.cout:
                        c.bwd.w = torch.nn.functional.pad(c.bwd.w, (0, 0, 0, 0, 0, 0, 0, c.bwd.cout - c.bwd.w.shape[0]))

    def _conv(self, c: _Conv, x, unit, inmode="none", x2=None, residual=None, out_nchw_f32=False):
        return convops.fused_conv2d(x, c.fwd, x2=x2, scale=unit.scale, shift=unit.shift, relu=unit.relu,
                                    residual=residual, inmode=inmode, out_nchw_f32=out_nchw_f32,
                                    cout_valid=self.nout if out_nchw_f32 else None)

    def _dgrad(self, c: _Conv, g):
        return convops.fused_conv2d(g, c.bwd)

    def _wgrad(self, c: _Conv, x, g, unit, inmode="none", x2=None):
        ct.conv_wgrad(x, g, ks=c.ks, cin_valid=c.cin, cout_valid=c.cout, dw=c.dw, db=c.db, inmode=inmode, x2=x2,
                      scale=unit.scale, shift=unit.shift, relu=unit.relu, ws=self._wg_ws if self.cuda else None)

    def _grad(self, key, like):
        """Gradient buffer of activation ``key``; returns (buffer, accumulate?)."""
        if key in self._g:
            return self._g[key], True
        buf = torch.empty_like(like)
        self._g[key] = buf
        return buf, False

    # ------------------------------------------------------------------ step
    @torch.no_grad()
    def forward(self, x_nchw: torch.Tensor):
        """x_nchw: [B, nchan, S, S] float -> net output [B, nout, S, S] fp32 (saves what backward needs)."""
        self._pack()
        self._ws_arena.zero_()
        act = {}
        xin = convops_to_nhwc(x_nchw, self.cin_pad, self.act_dtype)
        act["in"] = xin
        for n, blk in enumerate(self.down):
            src = xin if n == 0 else act[f"xd{n - 1}"]
            T = "none" if n == 0 else "pool2"
            c, s = blk.convs, blk.sites
            s[0].bn.stats(src, T)
            p = self._conv(c["proj"], src, s[0].units[0], T)
            h0 = self._conv(c["c0"], src, s[0].units[1], T)
            s[1].bn.stats(h0)
            x1 = self._conv(c["c1"], h0, s[1].units[0], residual=p)
            s[2].bn.stats(x1)
            h2 = self._conv(c["c2"], x1, s[2].units[0])
            s[3].bn.stats(h2)
            xd = self._conv(c["c3"], h2, s[3].units[0], residual=x1)
            act.update({f"d{n}.h0": h0, f"d{n}.x1": x1, f"d{n}.h2": h2, f"xd{n}": xd})
        nd = len(self.down)
        xlast = act[f"xd{nd - 1}"]
        # style = GAP / ||GAP||  (cellpose make_style) -> per-up-conv features
        from ..ops import style as styleops

        g = styleops.nhwc_channel_sum(xlast) / float(xlast.shape[1] * xlast.shape[2])
        gn = torch.sqrt((g * g).sum(1, keepdim=True))
        style = g / gn
        st = style if self.net.style_on else torch.zeros_like(style)
        act["style"], act["gnorm"] = style, gn
        wall = torch.cat([m.weight for m in self._style_full], 0)
        ball = torch.cat([m.bias for m in self._style_full], 0)
        feats_all = torch.addmm(ball, st, wall.t())
        feats, off = [], 0
        for m in self._style_full:
            feats.append(feats_all[:, off: off + m.out_features].contiguous())
            off += m.out_features
        act["feats"] = feats
        xcur = xlast
        nup = len(self.up)
        for i in range(nup - 1, -1, -1):
            blk = self.up[i]
            c, s = blk.convs, blk.sites
            T = "none" if i == nup - 1 else "up2"
            y = act[f"xd{i}"]
            f1, f2, f3 = feats[3 * i: 3 * i + 3]
            s[0].bn.stats(xcur, T)
            p = self._conv(c["proj"], xcur, s[0].units[0], T)
            h0 = self._conv(c["c0"], xcur, s[0].units[1], T)
            s[1].bn.stats(h0, x2=y, feat=f1)
            x1 = self._conv(c["c1"], h0, s[1].units[0], x2=y, residual=p)
            s[2].bn.stats(x1, feat=f2)
            h2 = self._conv(c["c2"], x1, s[2].units[0])
            s[3].bn.stats(h2, feat=f3)
            xo = self._conv(c["c3"], h2, s[3].units[0], residual=x1)
            act.update({f"u{i}.src": xcur, f"u{i}.h0": h0, f"u{i}.x1": x1, f"u{i}.h2": h2, f"u{i}.out": xo})
            xcur = xo
        self.head_site.bn.stats(xcur)
        y = self._conv(self.head, xcur, self.head_site.units[0], out_nchw_f32=True)
        act["head_in"] = xcur
        self._act = act
        return y

    @torch.no_grad()
    def backward(self, dy_nchw: torch.Tensor, on_params_ready=None) -> None:
        """dy_nchw: dLoss/dOutput [B, nout, S, S] fp32.  Writes every parameter gradient into the flat
        grad buffer.  ``on_params_ready(list_of_param_tensors)`` is called as groups complete (DDP)."""
        act = self._act
        self._g = {}
        B = self.B
        if self.cuda:  # wgrad split-K reductions accumulate into the flat gradient
            self.fp.grad.zero_()
        ready = on_params_ready or (lambda ps: None)
        # ---- head: 1x1 conv 32 -> nout, BN + ReLU on its input
        g8 = convops_to_nhwc(dy_nchw, 8, self.act_dtype)
        hu = self.head_site.units[0]
        xin = act["head_in"]
        dA = self._dgrad(self.head, g8)
        self._wgrad(self.head, xin, g8, hu)
        self.head_site.bn.bwd_reduce(xin, [dA])
        gbuf, acc = self._grad("u0.out", xin)
        self.head_site.bn.bwd_apply(xin, [dA], dx=gbuf, dx_acc=acc)
        ready(self._params_of([self.head], [self.head_site]))
        # ---- decoder (reverse of forward: block 0 first)
        nup = len(self.up)
        dfeats = [None] * (3 * nup)
        for i in range(nup):
            blk = self.up[i]
            c, s = blk.convs, blk.sites
            T = "none" if i == nup - 1 else "up2"
            src = act[f"u{i}.src"]
            y = act[f"xd{i}"]
            h0, x1, h2 = act[f"u{i}.h0"], act[f"u{i}.x1"], act[f"u{i}.h2"]
            f1, f2, f3 = act["feats"][3 * i: 3 * i + 3]
            gout = self._g[f"u{i}.out"]
            df = [torch.empty_like(f) for f in (f1, f2, f3)]
            dfeats[3 * i: 3 * i + 3] = df
            # c3 (input h2, feat f3), output residual = x1
            dA = self._dgrad(c["c3"], gout)
            self._wgrad(c["c3"], h2, gout, s[3].units[0])
            s[3].bn.bwd_reduce(h2, [dA], feat=f3, dfeat=df[2])
            gh2, _ = self._grad(f"u{i}.h2", h2)
            s[3].bn.bwd_apply(h2, [dA], feat=f3, dx=gh2)
            # c2 (input x1, feat f2): g_x1 = gout + du  (accumulate into gout's buffer)
            dA = self._dgrad(c["c2"], gh2)
            self._wgrad(c["c2"], x1, gh2, s[2].units[0])
            s[2].bn.bwd_reduce(x1, [dA], feat=f2, dfeat=df[1])
            s[2].bn.bwd_apply(x1, [dA], feat=f2, dx=gout, dx_acc=True)
            gx1 = gout
            # c1 (input h0 + skip y, feat f1), residual = proj output
            dA = self._dgrad(c["c1"], gx1)
            self._wgrad(c["c1"], h0, gx1, s[1].units[0], x2=y)
            s[1].bn.bwd_reduce(h0, [dA], x2=y, feat=f1, dfeat=df[0])
            gh0, _ = self._grad(f"u{i}.h0", h0)
            gy, yacc = self._grad(f"xd{i}", y)
            s[1].bn.bwd_apply(h0, [dA], x2=y, feat=f1, dx=gh0, dx2=gy, dx2_acc=yacc)
            # proj (1x1, from gx1) + c0 (from gh0) share the BN input T(src)
            dAp = self._dgrad(c["proj"], gx1)
            dA0 = self._dgrad(c["c0"], gh0)
            self._wgrad(c["proj"], src, gx1, s[0].units[0], inmode=T)
            self._wgrad(c["c0"], src, gh0, s[0].units[1], inmode=T)
            s[0].bn.bwd_reduce(src, [dAp, dA0], inmode=T)
            skey = f"u{i + 1}.out" if i < nup - 1 else f"xd{nup - 1}"
            gsrc, sacc = self._grad(skey, src)
            s[0].bn.bwd_apply(src, [dAp, dA0], inmode=T, dx=gsrc, dx_acc=sacc)
            ready(self._params_of(list(c.values()), s))
        # ---- style: feats = st @ W^T + b; st = g / |g|; g = mean_hw(xd_last)
        style, gn = act["style"], act["gnorm"]
        st = style if self.net.style_on else torch.zeros_like(style)
        dst = torch.zeros_like(style)
        for m, dfk in zip(self._style_full, dfeats):
            m.weight.grad.copy_(dfk.t() @ st)
            m.bias.grad.copy_(dfk.sum(0))
            dst += dfk @ m.weight
        nd = len(self.down)
        xlast = act[f"xd{nd - 1}"]
        gl, _ = self._grad(f"xd{nd - 1}", xlast)
        if self.net.style_on:
            dg = (dst - style * (style * dst).sum(1, keepdim=True)) / gn
            hw = float(xlast.shape[1] * xlast.shape[2])
            gl.copy_((gl.float() + (dg / hw)[:, None, None, :]).to(gl.dtype))
        ready(self._style_params())
        # ---- encoder
        for n in range(nd - 1, -1, -1):
            blk = self.down[n]
            c, s = blk.convs, blk.sites
            src = act["in"] if n == 0 else act[f"xd{n - 1}"]
            T = "none" if n == 0 else "pool2"
            h0, x1, h2 = act[f"d{n}.h0"], act[f"d{n}.x1"], act[f"d{n}.h2"]
            gout = self._g[f"xd{n}"]
            dA = self._dgrad(c["c3"], gout)
            self._wgrad(c["c3"], h2, gout, s[3].units[0])
            s[3].bn.bwd_reduce(h2, [dA])
            gh2, _ = self._grad(f"d{n}.h2", h2)
            s[3].bn.bwd_apply(h2, [dA], dx=gh2)
            dA = self._dgrad(c["c2"], gh2)
            self._wgrad(c["c2"], x1, gh2, s[2].units[0])
            s[2].bn.bwd_reduce(x1, [dA])
            s[2].bn.bwd_apply(x1, [dA], dx=gout, dx_acc=True)
            gx1 = gout
            dA = self._dgrad(c["c1"], gx1)
            self._wgrad(c["c1"], h0, gx1, s[1].units[0])
            s[1].bn.bwd_reduce(h0, [dA])
            gh0, _ = self._grad(f"d{n}.h0", h0)
            s[1].bn.bwd_apply(h0, [dA], dx=gh0)
            dAp = self._dgrad(c["proj"], gx1)
            dA0 = self._dgrad(c["c0"], gh0)
            self._wgrad(c["proj"], src, gx1, s[0].units[0], inmode=T)
            self._wgrad(c["c0"], src, gh0, s[0].units[1], inmode=T)
            s[0].bn.bwd_reduce(src, [dAp, dA0], inmode=T)
            if n > 0:
                gsrc, sacc = self._grad(f"xd{n - 1}", src)
                s[0].bn.bwd_apply(src, [dAp, dA0], inmode=T, dx=gsrc, dx_acc=sacc)
            ready(self._params_of(list(c.values()), s))
        self._g = {}

    # ------------------------------------------------------------------ param bookkeeping (DDP readiness)
    @staticmethod
    def _params_of(convs, sites):
        ps = []
        for c in convs:
            ps.append(c.conv.weight)
            if c.conv.bias is not None:
                ps.append(c.conv.bias)
        for s in sites:
            for u in s.units:
                ps += [u.gamma, u.beta]
        return ps

    def _style_params(self):
        return [p for m in self._style_full for p in (m.weight, m.bias)]

    def loss_and_backward(self, x_nchw: torch.Tensor, lbl: torch.Tensor, on_params_ready=None) -> torch.Tensor:
        y = self.forward(x_nchw)
        if self.cuda:
            loss, dy = train_ops.seg_loss_and_grad(y, lbl)
        else:
            with torch.enable_grad():
                yv = y.detach().requires_grad_(True)
                loss = train_ops.seg_loss_ref(yv, lbl)
                (dy,) = torch.autograd.grad(loss, yv)
            loss = loss.detach()
        self.backward(dy, on_params_ready)
        return loss


def convops_to_nhwc(x_nchw: torch.Tensor, cpad: int, dtype: torch.dtype) -> torch.Tensor:
    """NCHW float -> NHWC ``dtype`` with channels zero-padded to ``cpad``."""
    N, C, H, W = x_nchw.shape
    out = torch.zeros(N, H, W, cpad, dtype=dtype, device=x_nchw.device)
    out[..., :C] = x_nchw.permute(0, 2, 3, 1)
    return out
