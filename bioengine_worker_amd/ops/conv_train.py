"""Training ops for the fused pre-activation conv family (HIP kernels in ``csrc/kernels/conv_train.hip``).

A CPnet "unit" is ``out = conv_k(relu?(BN_train(T(x) [+ x2] [+ feat[n]]))) [+ bias] [+ residual]``
(cellpose ``batchconv`` / ``batchconv0`` / ``batchconvstyle``; SURVEY.md §2.5 K1, trained by the
reference through autograd at ``apps/cellpose-finetuning/main.py:1483-1546``).  The ops here are its
forward statistics and its backward:

* :class:`BnSite` — BatchNorm-train statistics of one BN input shared by one or two units
  (``stats``), and the backward reduction / apply (``bwd_reduce`` / ``bwd_apply``).
* :func:`conv_wgrad` — weight (+ bias) gradient, activation recomputed in the kernel's loader.
* :func:`pack_weights` — every conv's bf16 forward / dgrad weight layout from the fp32 master in one
  launch.

Every op has a CPU path that implements the same math with PyTorch (fp32); the engine runs on CPU
unchanged, which is how the backward math is checked against autograd without a GPU.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn.functional as F

from . import _native
from .conv import INMODES, _act_ref


# ------------------------------------------------------------------ transforms (CPU reference)

def _t_ref(x: torch.Tensor, inmode: str) -> torch.Tensor:
    """NHWC float -> transformed NHWC float."""
    if inmode == "none":
        return x
    xt = x.permute(0, 3, 1, 2)
    xt = F.interpolate(xt, scale_factor=2, mode="nearest") if inmode == "up2" else F.max_pool2d(xt, 2, 2)
    return xt.permute(0, 2, 3, 1)


def _tT_ref(du: torch.Tensor, x: torch.Tensor, inmode: str) -> torch.Tensor:
    """Adjoint of the transform: du at output resolution -> gradient at source resolution."""
    if inmode == "none":
        return du
    N, H, W, C = du.shape
    if inmode == "up2":
        return du.reshape(N, H // 2, 2, W // 2, 2, C).sum((2, 4))
    # max-pool: route to the first maximum of each 2x2 window ((0,0),(0,1),(1,0),(1,1) order)
    xs = x.float().reshape(N, H, 2, W, 2, C).permute(0, 1, 3, 2, 4, 5).reshape(N, H, W, 4, C)
    am = xs.argmax(3)  # torch.argmax returns the first maximal index
    oh = F.one_hot(am, 4).permute(0, 1, 2, 4, 3).to(du.dtype)  # [N, H, W, 4, C]
    g = oh * du.unsqueeze(3)
    return g.reshape(N, H, W, 2, 2, C).permute(0, 1, 3, 2, 4, 5).reshape(N, 2 * H, 2 * W, C)


def _store(dst: torch.Tensor, val: torch.Tensor, acc: bool) -> None:
    if acc:
        dst.copy_((dst.float() + val).to(dst.dtype))
    else:
        dst.copy_(val.to(dst.dtype))


# ------------------------------------------------------------------ BatchNorm (train) site

#: floats of the per-block partial scratch of the GPU BN reductions (~2k blocks x 4 x 256 channels)
SCRATCH_FLOATS = 2048 * 4 * 256

@dataclass
class BnUnit:
    """One BatchNorm2d feeding one conv: its parameters (views into the flat fp32 master), running
    statistics, and the conv-prologue affine computed from the batch statistics."""

    gamma: torch.Tensor
    beta: torch.Tensor
    run_mean: torch.Tensor | None
    run_var: torch.Tensor | None
    relu: bool
    scale: torch.Tensor      # [C] fp32 (BatchNorm) or [N, C] (GroupNorm)
    shift: torch.Tensor      # [N, C] fp32
    dgamma: torch.Tensor | None = None
    dbeta: torch.Tensor | None = None


class BnSite:
    """BN statistics + backward of one BN input ``u = T(x) [+ x2] [+ feat]`` shared by 1-2 units.

    ``groups = 0``: BatchNorm (train-mode batch statistics per channel).  ``groups = G``: GroupNorm --
    statistics per image and group of ``c_valid / G`` channels, so the conv-prologue affine, the
    mean / rstd and the backward coefficients are per image ([N, C]).
    ``stat`` is a slice of an arena the engine zeroes once per step; ``ticket`` two int32 counters."""

    def __init__(self, N: int, C: int, c_valid: int, units: list[BnUnit], stat: torch.Tensor, ticket: torch.Tensor,
                 eps: float = 1e-5, momentum: float = 0.05, scratch: torch.Tensor | None = None, groups: int = 0):
        assert 1 <= len(units) <= 2
        self.N, self.C, self.c_valid = N, C, c_valid
        self.groups = int(groups)
        if self.groups:
            assert c_valid % self.groups == 0, "GroupNorm groups must divide the channel count"
        self.units = units
        self.stat = stat
        self.ticket = ticket
        # per-block partial sums of the GPU reductions; may be shared by every site of an engine
        if scratch is None and stat.is_cuda:
            scratch = torch.empty(SCRATCH_FLOATS, device=stat.device, dtype=torch.float32)
        self.scratch = scratch
        self.eps, self.momentum = eps, momentum
        assert stat.numel() >= self.stat_numel(N, C, self.groups)

    @staticmethod
    def stat_numel(N: int, C: int, groups: int = 0) -> int:
        return 6 * N * C + 4 * (N * C if groups else C)

    @property
    def _cc(self) -> int:
        return self.N * self.C if self.groups else self.C

    # stat layout (matches conv_train.hip): sum, sq, mean, rstd, sdy0, sdyx0, sdy1, sdyx1, B0, B1
    def _v(self, off: int, n: int) -> torch.Tensor:
        return self.stat[off: off + n]

    @property
    def mean(self):
        m = self._v(2 * self.N * self.C, self._cc)
        return m.view(self.N, self.C) if self.groups else m

    @property
    def rstd(self):
        r = self._v(2 * self.N * self.C + self._cc, self._cc)
        return r.view(self.N, self.C) if self.groups else r

    def _sums(self):
        NC = self.N * self.C
        return self._v(0, NC).view(self.N, self.C), self._v(NC, NC).view(self.N, self.C)

    def _bwd(self, k):
        NC = self.N * self.C
        o = 2 * NC + 2 * self._cc + 2 * k * NC
        return self._v(o, NC).view(self.N, self.C), self._v(o + NC, NC).view(self.N, self.C)

    def _b(self):
        o = 6 * self.N * self.C + 2 * self._cc
        b0, b1 = self._v(o, self._cc), self._v(o + self._cc, self._cc)
        if self.groups:
            return b0.view(self.N, self.C), b1.view(self.N, self.C)
        return b0, b1

    def _rows(self, t):
        """Per-image view [N, 1, 1, C] of a coefficient (BN: broadcast [C])."""
        return t[:, None, None, :] if t.dim() == 2 else t

    def _call(self, which, x, x2, feat, inmode, H, W, dacts=(None, None), dfeat=None, dx=None, dx_acc=False, dx2=None,
              dx2_acc=False):
        N, Hs, Ws, C = x.shape
        u = self.units + [None] * (2 - len(self.units))
        args = []
        for k in range(2):
            uk = u[k]
            if uk is None:
                args += [None, None, None, None, None, None, 0, None, None, None]
            else:
                args += [uk.gamma, uk.beta, uk.scale, uk.shift, uk.run_mean, uk.run_var, int(uk.relu), dacts[k],
                         uk.dgamma, uk.dbeta]
        P = _native.ptr
        conv = [P(a) if (a is None or isinstance(a, torch.Tensor)) else a for a in args]
        _native.call("be_bn_train", which, P(x), P(x2), P(feat), N, Hs, Ws, H, W, C, self.c_valid, INMODES[inmode],
                     len(self.units), float(self.eps), float(self.momentum), self.groups, P(self.stat), P(self.ticket),
                     *conv,
                     P(dfeat), P(dx), int(dx_acc), P(dx2), int(dx2_acc), P(self.scratch), self.scratch.numel(),
                     _native.stream(x.device))

    # -------------------------------------------------------------- forward statistics
    def stats(self, x: torch.Tensor, inmode: str = "none", x2: torch.Tensor | None = None,
              feat: torch.Tensor | None = None, update_running: bool = True) -> None:
        N, Hs, Ws, C = x.shape
        H, W = _out_hw(Hs, Ws, inmode)
        if x.is_cuda:
            if not update_running:
                saved = [(uk.run_mean, uk.run_var) for uk in self.units]
                for uk in self.units:
                    uk.run_mean = uk.run_var = None
            self._call(0, x, x2, feat, inmode, H, W)
            if not update_running:
                for uk, (rm, rv) in zip(self.units, saved):
                    uk.run_mean, uk.run_var = rm, rv
            return
        v = self._vref(x, inmode, x2)
        s, q = self._sums()
        s.copy_(v.sum((1, 2)))
        q.copy_((v * v).sum((1, 2)))
        f = feat.float() if feat is not None else torch.zeros(N, C)
        HW = H * W
        if self.groups:
            return self._gn_stats_ref(s, q, f, HW)
        cnt = N * HW
        s1 = (s + HW * f).sum(0)
        qq = (q + 2 * f * s + HW * f * f).sum(0)
        mean = s1 / cnt
        var = (qq / cnt - mean * mean).clamp_min(0)
        valid = torch.arange(C) < self.c_valid
        rstd = torch.where(valid, 1.0 / torch.sqrt(var + self.eps), torch.zeros(()))
        self.mean.copy_(torch.where(valid, mean, torch.zeros(())))
        self.rstd.copy_(rstd)
        for uk in self.units:
            g = _pad_to(uk.gamma, C)
            b = _pad_to(uk.beta, C)
            sc = torch.where(valid, g * rstd, torch.zeros(()))
            uk.scale.copy_(sc)
            uk.shift.copy_(torch.where(valid, (f - mean) * sc + b, torch.zeros(())))
            if update_running and uk.run_mean is not None:
                m = self.momentum
                cv = self.c_valid
                uk.run_mean.mul_(1 - m).add_(m * mean[:cv])
                uk.run_var.mul_(1 - m).add_(m * var[:cv] * cnt / max(cnt - 1, 1))

    def _gn_stats_ref(self, s, q, f, HW):
        N, C, G, cv = self.N, self.C, self.groups, self.c_valid
        cg = cv // G
        s1 = (s + HW * f)[:, :cv].reshape(N, G, cg).sum(2)
        qq = (q + 2 * f * s + HW * f * f)[:, :cv].reshape(N, G, cg).sum(2)
        cnt = HW * cg
        mean = s1 / cnt
        rstd = 1.0 / torch.sqrt((qq / cnt - mean * mean).clamp_min(0) + self.eps)
        mc = torch.zeros(N, C)
        rc = torch.zeros(N, C)
        mc[:, :cv] = mean.repeat_interleave(cg, 1)
        rc[:, :cv] = rstd.repeat_interleave(cg, 1)
        self.mean.copy_(mc)
        self.rstd.copy_(rc)
        valid = (torch.arange(C) < cv)[None]
        for uk in self.units:
            sc = torch.where(valid, _pad_to(uk.gamma, C)[None] * rc, torch.zeros(()))
            uk.scale.copy_(sc)
            uk.shift.copy_(torch.where(valid, (f - mc) * sc + _pad_to(uk.beta, C)[None], torch.zeros(())))

    @staticmethod
    def _vref(x, inmode, x2):
        v = _t_ref(x.float(), inmode)
        if x2 is not None:
            v = v + x2.float()
        return v

    # -------------------------------------------------------------- backward
    def bwd_reduce(self, x: torch.Tensor, dacts: list[torch.Tensor], inmode: str = "none",
                   x2: torch.Tensor | None = None, feat: torch.Tensor | None = None,
                   dfeat: torch.Tensor | None = None) -> None:
        N, Hs, Ws, C = x.shape
        H, W = _out_hw(Hs, Ws, inmode)
        if x.is_cuda:
            d = list(dacts) + [None] * (2 - len(dacts))
            self._call(1, x, x2, feat, inmode, H, W, dacts=d, dfeat=dfeat)
            return
        v = self._vref(x, inmode, x2)
        f = feat.float() if feat is not None else torch.zeros(N, C)
        xh = (v + f[:, None, None, :] - self._rows(self.mean)) * self._rows(self.rstd)
        if self.groups:
            return self._gn_reduce_ref(v, xh, dacts, f, H * W, dfeat)
        cnt = N * H * W
        b0 = torch.zeros(C)
        b1 = torch.zeros(C)
        valid = torch.arange(C) < self.c_valid
        for k, (uk, da) in enumerate(zip(self.units, dacts)):
            dy = self._masked(uk, v, da)
            sdy, sdyx = self._bwd(k)
            sdy.copy_(dy.sum((1, 2)))
            sdyx.copy_((dy * xh).sum((1, 2)))
            tdy, tdyx = sdy.sum(0), sdyx.sum(0)
            b0 -= uk.scale * tdy / cnt
            b1 -= uk.scale * tdyx / cnt
            cv = self.c_valid
            if uk.dgamma is not None:
                uk.dgamma.copy_(tdyx[:cv])
            if uk.dbeta is not None:
                uk.dbeta.copy_(tdy[:cv])
        B0, B1 = self._b()
        B0.copy_(b0)
        B1.copy_(b1)
        if dfeat is not None:
            s, _ = self._sums()
            sx = (s + H * W * (f - self.mean)) * self.rstd
            sdy, _ = self._bwd(0)
            val = self.units[0].scale * sdy + H * W * b0 + b1 * sx
            dfeat.copy_(torch.where(valid, val, torch.zeros(())))

    def _gn_reduce_ref(self, v, xh, dacts, f, HW, dfeat):
        N, C, G, cv = self.N, self.C, self.groups, self.c_valid
        cg = cv // G
        M = HW * cg
        b0 = torch.zeros(N, G)
        b1 = torch.zeros(N, G)
        for k, (uk, da) in enumerate(zip(self.units, dacts)):
            dy = self._masked(uk, v, da)
            sdy, sdyx = self._bwd(k)
            sdy.copy_(dy.sum((1, 2)))
            sdyx.copy_((dy * xh).sum((1, 2)))
            b0 -= (uk.scale * sdy)[:, :cv].reshape(N, G, cg).sum(2) / M
            b1 -= (uk.scale * sdyx)[:, :cv].reshape(N, G, cg).sum(2) / M
            if uk.dgamma is not None:
                uk.dgamma.copy_(sdyx.sum(0)[:cv])
            if uk.dbeta is not None:
                uk.dbeta.copy_(sdy.sum(0)[:cv])
        B0, B1 = self._b()
        B0.zero_()
        B1.zero_()
        B0[:, :cv] = b0.repeat_interleave(cg, 1)
        B1[:, :cv] = b1.repeat_interleave(cg, 1)
        if dfeat is not None:
            s, _ = self._sums()
            sx = (s + HW * (f - self.mean)) * self.rstd
            sdy, _ = self._bwd(0)
            val = self.units[0].scale * sdy + HW * B0 + B1 * sx
            valid = (torch.arange(C) < cv)[None]
            dfeat.copy_(torch.where(valid, val, torch.zeros(())))

    @staticmethod
    def _masked(uk: BnUnit, v: torch.Tensor, da: torch.Tensor) -> torch.Tensor:
        dy = da.float()
        if uk.relu:
            sc = uk.scale[:, None, None, :] if uk.scale.dim() == 2 else uk.scale
            y = v * sc + uk.shift[:, None, None, :]
            dy = torch.where(y > 0, dy, torch.zeros(()))
        return dy

    def bwd_apply(self, x: torch.Tensor, dacts: list[torch.Tensor], inmode: str = "none",
                  x2: torch.Tensor | None = None, feat: torch.Tensor | None = None,
                  dx: torch.Tensor | None = None, dx_acc: bool = False,
                  dx2: torch.Tensor | None = None, dx2_acc: bool = False) -> None:
        N, Hs, Ws, C = x.shape
        H, W = _out_hw(Hs, Ws, inmode)
        if dx is None and dx2 is None:
            return
        if x.is_cuda:
            d = list(dacts) + [None] * (2 - len(dacts))
            self._call(2, x, x2, feat, inmode, H, W, dacts=d, dx=dx, dx_acc=dx_acc, dx2=dx2, dx2_acc=dx2_acc)
            return
        v = self._vref(x, inmode, x2)
        f = feat.float() if feat is not None else torch.zeros(N, C)
        xh = (v + f[:, None, None, :] - self._rows(self.mean)) * self._rows(self.rstd)
        B0, B1 = self._b()
        du = self._rows(B0) + self._rows(B1) * xh
        for uk, da in zip(self.units, dacts):
            du = du + self._rows(uk.scale) * self._masked(uk, v, da)
        if dx2 is not None:
            _store(dx2, du, dx2_acc)
        if dx is not None:
            _store(dx, _tT_ref(du, x, inmode), dx_acc)


def _out_hw(Hs: int, Ws: int, inmode: str) -> tuple[int, int]:
    if inmode == "up2":
        return Hs * 2, Ws * 2
    if inmode == "pool2":
        return Hs // 2, Ws // 2
    return Hs, Ws


def _pad_to(v: torch.Tensor, n: int) -> torch.Tensor:
    if v.numel() == n:
        return v.float()
    out = torch.zeros(n, dtype=torch.float32, device=v.device)
    out[: v.numel()] = v
    return out


# ------------------------------------------------------------------ weight gradient

def wgrad_splits(N: int, H: int, W: int, cin: int, cout: int, ks: int, target_blocks: int = 512) -> int:
    """Split-K count: enough blocks to fill 256 CUs twice, at least 4 pixel tiles (4x32) per split."""
    ntiles = N * ((H + 3) // 4) * ((W + 31) // 32)
    ck = 8 if cin == 8 else 32
    tco = 16 if cout <= 16 else (32 if cout <= 32 else 64)
    blocks_per_split = max(1, cin // ck) * ((cout + tco - 1) // tco)
    s = max(1, target_blocks // blocks_per_split)
    return max(1, min(s, ntiles // 4 if ntiles >= 4 else 1))


def conv_wgrad(x: torch.Tensor, dy: torch.Tensor, *, ks: int, cin_valid: int, cout_valid: int, dw: torch.Tensor,
               db: torch.Tensor | None = None, inmode: str = "none", x2: torch.Tensor | None = None,
               scale: torch.Tensor | None = None, shift: torch.Tensor | None = None, relu: bool = False,
               ws: torch.Tensor | None = None, splits: int | None = None) -> None:
    """dw[co, ci, ky, kx] = sum_{n,y,x} dy[n, y, x, co] * act(x)[n, y+ky-k/2, x+kx-k/2, ci]; db = sum dy.

    ``x`` NHWC [N, Hs, Ws, Cin] (pre-transform, pre-BN), ``dy`` NHWC [N, H, W, Cy >= cout_valid].
    On GPU ``dw``/``db`` are ACCUMULATED into (split-K partials are atomically added: zero them first,
    e.g. the engine zeroes the flat gradient buffer once per step); the CPU path overwrites."""
    N, Hs, Ws, Cin = x.shape
    H, W = _out_hw(Hs, Ws, inmode)
    if not x.is_cuda:
        a = _act_ref(x.float(), x2, scale, shift, relu, inmode)  # NCHW
        a = a[:, :cin_valid]
        g = dy.float()[..., :cout_valid].permute(0, 3, 1, 2)
        w = torch.nn.grad.conv2d_weight(a, (cout_valid, cin_valid, ks, ks), g, padding=ks // 2)
        dw.copy_(w.reshape(dw.shape))
        if db is not None:
            db.copy_(g.sum((0, 2, 3)))
        return
    Cy = dy.shape[-1]
    assert x.dtype == torch.bfloat16 and dy.dtype == torch.bfloat16 and x.is_contiguous() and dy.is_contiguous()
    assert dy.shape[:3] == (N, H, W) and Cy % 8 == 0 and cout_valid <= Cy
    assert Cin == 8 or Cin % 32 == 0, "wgrad needs Cin == 8 or Cin % 32 == 0"
    assert dw.dtype == torch.float32 and dw.is_contiguous() and dw.numel() == cout_valid * cin_valid * ks * ks
    if x2 is not None:
        assert inmode == "none" and x2.shape == (N, H, W, Cin) and x2.is_contiguous()
    pscale_ns = 0
    if scale is not None:
        assert scale.numel() in (Cin, N * Cin) and scale.dtype == torch.float32 and scale.is_contiguous()
        pscale_ns = Cin if scale.dim() == 2 else 0
    pshift_ns = 0
    if shift is not None:
        assert shift.dtype == torch.float32 and shift.is_contiguous()
        pshift_ns = Cin if shift.dim() == 2 else 0
    splits = splits or wgrad_splits(N, H, W, Cin, Cy, ks)
    need = splits * cout_valid * ks * ks * Cin + splits * cout_valid
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, device=x.device, dtype=torch.float32)
    wsb = ws[splits * cout_valid * ks * ks * Cin:]
    _native.call("be_conv_wgrad", _native.ptr(x), _native.ptr(x2), _native.ptr(scale), _native.ptr(shift), pshift_ns,
                 pscale_ns, int(bool(relu)), _native.ptr(dy), _native.ptr(ws), _native.ptr(wsb), _native.ptr(dw), _native.ptr(db),
                 N, H, W, Hs, Ws, Cin, cin_valid, Cy, cout_valid, ks, INMODES[inmode], splits,
                 _native.stream(x.device))


# ------------------------------------------------------------------ weight packing

PACK_FIELDS = 10


def pack_weights(descs: torch.Tensor, n: int, max_elems: int, flat: torch.Tensor, arena: torch.Tensor) -> None:
    """descs: int32 [n, 10] device table (src_off, dst_off, cout, cin, ks, rows_pad, in_pad, ck, kp, transpose)."""
    _native.call("be_pack_conv_weights", _native.ptr(descs), n, max_elems, _native.ptr(flat), _native.ptr(arena),
                 _native.stream(flat.device))


def pack_ref(w: torch.Tensor, rows_pad: int, in_pad: int, ck: int, kp: int, transpose: bool) -> torch.Tensor:
    """CPU reference of one descriptor: fp32 W [cout, cin, k, k] -> packed [rows_pad, in_pad/ck, kp]."""
    if transpose:
        w = w.flip(2, 3).transpose(0, 1)
    rows, cin, ks, _ = w.shape
    nchunk = in_pad // ck
    wz = torch.zeros(rows_pad, in_pad, ks, ks, dtype=torch.float32, device=w.device)
    wz[:rows, :cin] = w
    t = wz.permute(0, 2, 3, 1).reshape(rows_pad, ks * ks, nchunk, ck).permute(0, 2, 1, 3)
    t = t.reshape(rows_pad, nchunk, ks * ks * ck)
    if kp > ks * ks * ck:
        t = F.pad(t, (0, kp - ks * ks * ck))
    return t
