"""Fused pre-activation NHWC conv2d (HIP kernel ``csrc/kernels/conv2d_nhwc.hip``).

``fused_conv2d`` computes::

    out = conv_k( relu?( (inxform(x) [+ x2]) * scale[c] + shift[n, c] ) ) [+ bias] [+ residual]

with ``inxform`` in {identity, nearest-upsample x2, maxpool 2x2}.  This covers every conv in the
Cellpose CPnet (cellpose ``batchconv``/``batchconv0``/``batchconvstyle``: BN -> ReLU -> Conv, the
style-vector add and the skip add; reference reaches these via cellpose EXT modules, SURVEY.md §2.5
K1) and the pre-activation blocks of BioImage.IO U-Nets.

Activations are NHWC bf16 (channels padded to a multiple of 8); weights are repacked once into the
kernel's tap-major K layout by :class:`PackedConv`.
"""
from __future__ import annotations

import os

from dataclasses import dataclass

import torch
import torch.nn.functional as F

from . import _native

#: input-channel chunk of 1x1 convs whose padded Cin is a multiple of 64 (32 or 64)
CK_1X1 = 64

INMODES = {"none": 0, "up2": 1, "pool2": 2}


def _round_up(v: int, m: int) -> int:
    return (v + m - 1) // m * m


@dataclass
class PackedConv:
    """Conv weights repacked for the MFMA kernel.

    ``wp``  : bf16 [cout_pad, nchunk, KP] (device tensor), K index = tap * ck + c within a chunk.
    ``w``   : fp32 [cout, cin, ks, ks] original weights (reference path / re-packing).
    """

    w: torch.Tensor
    bias: torch.Tensor | None
    ks: int
    cin: int
    cin_pad: int
    cout: int
    cout_pad: int
    ck: int
    tco: int
    kp: int
    wp: torch.Tensor | None = None

    @staticmethod
    def choose(cin_pad: int, cout: int, ks: int = 3) -> tuple[int, int]:
        ck = 8 if cin_pad % 32 else 32
        # 1x1 convs (the resblock projections) have one K step per 32-channel chunk, so their
        # chunk loop is pure load latency: wider chunks halve the serial steps (BE_CONV_CK1)
        ck1 = int(os.environ.get("BE_CONV_CK1", CK_1X1))
        if ks == 1 and ck1 == 64 and cin_pad % 64 == 0:
            ck = 64
        if cout <= 16:
            tco = 16
        elif cout <= 32:
            tco = 32
        else:
            tco = 64
        return ck, tco

    @classmethod
    def from_weight(cls, weight: torch.Tensor, bias: torch.Tensor | None = None, cin_pad: int | None = None,
                    cout_pad_to: int | None = None, exact_cin: bool = False, ck16: bool = False) -> "PackedConv":
        """``exact_cin``: keep a multiple-of-8 channel count as is (8-channel K chunks) instead of
        padding it to a multiple of 32 (the 3-D U-Net's 16-channel layers, see ops/conv3d.py);
        ``ck16``: 16-channel K chunks when the count is an odd multiple of 16 (3x3 only; the z-tap
        kernel's CK = 16 build)."""
        cout, cin, ks, ks2 = weight.shape
        assert ks == ks2 and ks in (1, 3), "only 1x1 / 3x3 convs"
        cin_pad = cin_pad or _round_up(cin, 8)
        if cin_pad % 32 and cin_pad != 8 and not (exact_cin and cin_pad % 8 == 0):
            cin_pad = _round_up(cin_pad, 32)
        ck, tco = cls.choose(cin_pad, cout, ks)
        if ck16 and ks == 3 and ck == 8 and cin_pad % 16 == 0:
            ck = 16
        cout_k = max(cout, cout_pad_to or 0)
        cout_pad = _round_up(cout_k, tco)
        kp = ((ks * ks * ck + 31) // 32) * 32
        w = weight.detach().float()
        pc = cls(w=w, bias=None if bias is None else bias.detach().float(), ks=ks, cin=cin, cin_pad=cin_pad,
                 cout=cout, cout_pad=cout_pad, ck=ck, tco=tco, kp=kp)
        pc.wp = pc._pack(w)
        return pc

    def _pack(self, w: torch.Tensor) -> torch.Tensor:
        ks, ck = self.ks, self.ck
        nchunk = self.cin_pad // ck
        wz = torch.zeros(self.cout_pad, self.cin_pad, ks, ks, dtype=torch.float32, device=w.device)
        wz[: self.cout, : self.cin] = w
        # [Cout, ks, ks, Cin] -> [Cout, taps, nchunk, ck] -> [Cout, nchunk, taps*ck]
        t = wz.permute(0, 2, 3, 1).reshape(self.cout_pad, ks * ks, nchunk, ck)
        t = t.permute(0, 2, 1, 3).reshape(self.cout_pad, nchunk, ks * ks * ck)
        if self.kp > ks * ks * ck:
            t = F.pad(t, (0, self.kp - ks * ks * ck))
        return t.to(torch.bfloat16).contiguous()

    def to(self, device) -> "PackedConv":
        self.w = self.w.to(device)
        if self.bias is not None:
            self.bias = self.bias.to(device)
        if self.wp is not None:
            self.wp = self.wp.to(device)
        return self

    def refresh(self, weight: torch.Tensor, bias: torch.Tensor | None = None) -> None:
        """Re-pack after a weight update (training)."""
        self.w = weight.detach().float()
        if bias is not None:
            self.bias = bias.detach().float()
        self.wp = self._pack(self.w)


register = _native.register_hip_signatures


def _act_ref(x, x2, scale, shift, relu, inmode):
    # x: NHWC float
    xt = x.permute(0, 3, 1, 2)
    if inmode == "up2":
        xt = F.interpolate(xt, scale_factor=2, mode="nearest")
    elif inmode == "pool2":
        xt = F.max_pool2d(xt, 2, 2)
    if x2 is not None:
        xt = xt + x2.permute(0, 3, 1, 2).float()
    C = xt.shape[1]
    if scale is not None:
        xt = xt * (scale.view(-1, C, 1, 1) if scale.dim() == 2 else scale.view(1, C, 1, 1))
    if shift is not None:
        sh = shift.view(-1, C, 1, 1) if shift.dim() == 2 else shift.view(1, C, 1, 1)
        xt = xt + sh
    if relu:
        xt = torch.relu(xt)
    return xt


def fused_conv2d_ref(x, pc: PackedConv, x2=None, scale=None, shift=None, relu=False, residual=None,
                     inmode="none", out_nchw_f32=False, cout_valid=None, act_dtype=torch.bfloat16, post_relu=False,
                     no_bias=False):
    """PyTorch fp32 reference (and CPU path).  The activated input is rounded to ``act_dtype``
    exactly like the kernel's LDS staging, so GPU-vs-reference differences are accumulation-order only."""
    a = _act_ref(x.float(), x2, scale, shift, relu, inmode)
    if act_dtype is not None:
        a = a.to(act_dtype).float()
    w = pc.w.to(a.device)
    if w.shape[1] < a.shape[1]:
        w = F.pad(w, (0, 0, 0, 0, 0, a.shape[1] - w.shape[1]))
    wq = w.to(torch.bfloat16).float() if act_dtype is not None else w
    y = F.conv2d(a, wq, None, padding=pc.ks // 2)
    if pc.bias is not None and not no_bias:
        y = y + pc.bias.to(y.device).view(1, -1, 1, 1)
    if out_nchw_f32:
        cv = cout_valid or pc.cout
        y = y[:, :cv].contiguous()
        return torch.relu(y) if post_relu else y
    y = y.permute(0, 2, 3, 1)
    if residual is not None:
        y = y + residual.float()
    if post_relu:
        y = torch.relu(y)
    return y.to(x.dtype).contiguous()


#: waves per workgroup (tile = 2*nw rows x 32 cols); overridable per call and per (ks, cin, cout).
NW_POLICY: dict = {}
DEFAULT_NW = None  # None = shape policy below; 4 / 8 forces one value (sweeps)


def choose_nw(pc: PackedConv, H: int, W: int, inmode: str = "none", has_x2: bool = False) -> int:
    """Measured on MI355X (tools/conv_sweep2.py, profiles/conv_sweep.md): the persistent
    small-channel variants (tco <= 32) prefer 8 waves (more halo reuse per weight fetch); the
    64-channel variants prefer 4 waves (two blocks/CU hide the barrier) except when the halo loader
    does the 2x2 max-pool at <= 28x28 output (8 waves amortise the 4x wider input read; measured
    again in round 3, profiles/r03/conv_deep_ab.md: at 56x56 the 4-wave tiles are 11 % faster).  The skip-add (x2) 64-channel
    variant only fits without spills at 4 waves."""
    key = (pc.ks, pc.cin_pad, pc.cout, inmode)
    if key in NW_POLICY:
        return NW_POLICY[key]
    if DEFAULT_NW is not None:
        return DEFAULT_NW
    if pc.tco <= 32:
        return 8
    if has_x2:
        return 4
    if inmode == "pool2" and pc.ks == 3 and H * W <= 28 * 28:
        return 8  # 8 waves amortise the 4x wider pooled input read (56x56 and up: 4 waves, conv_deep_ab)
    return 4


def _affine_stride(t: torch.Tensor | None, N: int, C: int) -> int:
    """Row stride (elements) of a per-image [N, C] fp32 affine, 0 for a shared [C] one."""
    if t is None:
        return 0
    assert t.dtype == torch.float32
    if t.dim() == 2:
        assert t.shape == (N, C) and t.stride(1) == 1, "per-image affine must be [N, C] with unit column stride"
        ns = t.stride(0) if N > 1 else C
        assert ns % 4 == 0 and t.data_ptr() % 16 == 0, "per-image affine rows must be 16-byte aligned"
        return ns
    assert t.is_contiguous() and t.numel() == C
    return 0


def fused_conv2d(x: torch.Tensor, pc: PackedConv, *, x2=None, scale=None, shift=None, relu=False, residual=None,
                 inmode: str = "none", out_nchw_f32: bool = False, cout_valid: int | None = None,
                 nw: int | None = None, post_relu: bool = False, out: torch.Tensor | None = None,
                 no_bias: bool = False, post_scale=None, post_shift=None) -> torch.Tensor:
    """Fused conv on NHWC activations.  ``x`` is [N, Hs, Ws, Cin_pad] bf16 (GPU) or any float (CPU).
    ``relu`` applies to the pre-activation input, ``post_relu`` to the output (after bias/residual).
    ``out`` (bf16 NHWC, contiguous) receives the result in place of a new tensor; it may be the
    ``residual`` itself (every output element reads its residual before it is stored).
    ``no_bias`` skips ``pc.bias`` (partial sums of a depth-decomposed 3-D conv).
    ``post_scale`` [Cout] / ``post_shift`` ([Cout] or row-strided [N, Cout]) apply the NEXT conv's
    pre-activation to the stored value (``y = bf16(y) * post_scale + post_shift``, then ``post_relu``):
    the producer-side activation that feeds :func:`~.conv_igemm.conv3_igemm`."""
    N, Hs, Ws, Cin = x.shape
    if inmode == "up2":
        H, W = Hs * 2, Ws * 2
    elif inmode == "pool2":
        H, W = Hs // 2, Ws // 2
    else:
        H, W = Hs, Ws
    if not x.is_cuda:
        y = fused_conv2d_ref(x, pc, x2, scale, shift, relu, residual, inmode, out_nchw_f32, cout_valid,
                             act_dtype=torch.bfloat16 if x.dtype == torch.bfloat16 else None,
                             post_relu=post_relu and post_scale is None and post_shift is None, no_bias=no_bias)
        if post_scale is not None or post_shift is not None:
            yf = y.to(torch.bfloat16).float()
            if post_scale is not None:
                yf = yf * post_scale.to(yf.device)
            if post_shift is not None:
                ps = post_shift.to(yf.device)
                yf = yf + (ps[:, None, None, :] if ps.dim() == 2 else ps)
            if post_relu:
                yf = torch.relu(yf)
            y = yf.to(y.dtype)
        if out is not None:
            out.copy_(y)
            return out
        return y
    assert x.dtype == torch.bfloat16 and x.is_contiguous(), "fused_conv2d expects contiguous NHWC bf16"
    assert Cin == pc.cin_pad, f"input channels {Cin} != packed cin {pc.cin_pad}"
    if pc.wp.device != x.device:
        pc.to(x.device)
    cout_valid = cout_valid or pc.cout
    if out_nchw_f32:
        assert out is None
        out = torch.empty(N, cout_valid, H, W, device=x.device, dtype=torch.float32)
        cout_store = pc.cout_pad
    else:
        assert pc.cout % 4 == 0
        if out is None:
            out = torch.empty(N, H, W, pc.cout, device=x.device, dtype=torch.bfloat16)
        else:
            assert out.shape == (N, H, W, pc.cout) and out.dtype == torch.bfloat16 and out.is_contiguous()
        cout_store = pc.cout
    if x2 is not None:
        assert x2.shape == (N, H, W, Cin) and x2.dtype == torch.bfloat16 and x2.is_contiguous()
    if residual is not None:
        assert residual.shape == (N, H, W, pc.cout) and residual.dtype == torch.bfloat16 and residual.is_contiguous()
    # per-image affines ([N, Cin], GroupNorm scale / style shift) may be row-strided views (e.g. column
    # slices of one stacked style GEMM output): rows are read as float4 runs at n * row_stride + c
    pscale_ns = _affine_stride(scale, N, Cin)
    pshift_ns = _affine_stride(shift, N, Cin)
    qshift_ns = _affine_stride(post_shift, N, pc.cout)
    if post_scale is not None:
        assert post_scale.dtype == torch.float32 and post_scale.is_contiguous() and post_scale.numel() == pc.cout
    _native.call(
        "be_conv2d_nhwc",
        _native.ptr(x), _native.ptr(x2), _native.ptr(scale), _native.ptr(shift), pshift_ns, pscale_ns,
        int(bool(relu)) | (2 if post_relu else 0),
        _native.ptr(pc.wp), _native.ptr(None if no_bias else pc.bias), _native.ptr(residual), _native.ptr(out),
        N, H, W, Hs, Ws, Cin, cout_store, cout_valid, pc.ks, pc.ck, pc.tco, INMODES[inmode], int(out_nchw_f32),
        int(nw or choose_nw(pc, H, W, inmode, x2 is not None)), _native.ptr(post_scale), _native.ptr(post_shift),
        qshift_ns, _native.stream(x.device),
    )
    return out


def depth_to_space2(y: torch.Tensor, c: int) -> torch.Tensor:
    """[N, H, W, 4 c] (channel (2 dy + dx) * c + k) -> [N, 2H, 2W, c] NHWC (a copy)."""
    N, H, W, _ = y.shape
    return y.view(N, H, W, 2, 2, c).permute(0, 1, 3, 2, 4, 5).reshape(N, 2 * H, 2 * W, c)


def fused_conv2d_concat(xa: torch.Tensor, xb: torch.Tensor, pc: PackedConv, *, post_relu: bool = False,
                        nw: int | None = None, xb_d2s: bool = False) -> torch.Tensor:
    """3x3 conv (+ bias, + ReLU) of the channel concatenation [xa, xb] of two NHWC tensors
    ([N, H, W, Ca] and [N, H, W, Cb], ``pc`` packed for Ca + Cb input channels) without materialising
    it: ``be_conv2d_concat`` (INMODE 4) picks each 8-channel group's source in the halo loader.  Same
    K order and accumulation as :func:`fused_conv2d` on ``torch.cat([xa, xb], -1)``.  ``xb_d2s``: xb is
    [N, H/2, W/2, 4 Cb], a 2x2 transposed conv's sub-pixel channels before the depth-to-space shuffle
    (INMODE 6 reads it in place)."""
    N, H, W, Ca = xa.shape
    Cb = xb.shape[-1] // 4 if xb_d2s else xb.shape[-1]
    if xb_d2s:
        assert xb.shape[:3] == (N, H // 2, W // 2) and H % 2 == 0 and W % 2 == 0
    else:
        assert xb.shape[:3] == (N, H, W)
    assert pc.ks == 3 and pc.cin_pad == Ca + Cb
    if not xa.is_cuda:
        xbf = depth_to_space2(xb, Cb) if xb_d2s else xb
        return fused_conv2d(torch.cat([xa, xbf], -1), pc, post_relu=post_relu)
    assert xa.dtype == xb.dtype == torch.bfloat16 and xa.is_contiguous() and xb.is_contiguous()
    assert Ca % 8 == 0 and Cb % 8 == 0 and pc.cout % 4 == 0
    if pc.wp.device != xa.device:
        pc.to(xa.device)
    out = torch.empty(N, H, W, pc.cout, device=xa.device, dtype=torch.bfloat16)
    _native.call("be_conv2d_concat", _native.ptr(xa), _native.ptr(xb), _native.ptr(pc.wp), _native.ptr(pc.bias),
                 _native.ptr(out), N, H, W, Ca, Cb, pc.cout, pc.ck, pc.tco, int(bool(post_relu)),
                 int(nw or choose_nw(pc, H, W)), int(bool(xb_d2s)), _native.stream(xa.device))
    return out
