"""Fused residual half-block: two pre-activation 3x3 convs, intermediate kept in LDS
(HIP kernel ``csrc/kernels/conv_pair.hip``).

``conv_pair`` computes::

    h   = relu( (convA(actA(inxform(x))) + biasA [+ x2]) * sB + tB )
    out = convB(h) + biasB [+ convP(actP(x)) + biasP] [+ res | + up2(res)]

with ``actA(v) = relu(v * sA + tA)``, ``actP(v) = v * sP + tP``.  ``tA``/``tB`` may be per-image
``[N, C]`` rows (the folded style vector of cellpose ``batchconvstyle``).  Two calls make one Cellpose
CPnet residual block (``resdown``/``resup``, reached by the reference through
cellpose==3.1.1.2, ``/root/reference/apps/model-runner/runtime_deployment.py:19``).

The kernel never writes ``h`` to HBM; it rounds it to bf16 ONCE after actB (the per-layer path
rounds the raw conv output and then the activation), so :func:`conv_pair_ref` mirrors exactly that.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn.functional as F

from . import _native
from .conv import INMODES, PackedConv, _act_ref, _affine_stride

#: (Cin, CM, inmode, x2, proj, res) combinations the kernel is instantiated for (CPnet levels 0/1)
SUPPORTED = {
    (8, 32, "none", False, True, "none"),
    (32, 32, "none", False, False, "full"),
    (64, 32, "up2", True, False, "up2"),
    (32, 64, "pool2", False, False, "full"),
    (64, 64, "none", False, False, "full"),
    (128, 64, "up2", True, False, "up2"),
}
RESMODES = {"none": 0, "full": 1, "up2": 2}


@dataclass
class PairSpec:
    """Weights + folded affines of one fused half-block.

    ``tb`` is actB's shift with convA's bias folded in (``tB + sB * biasA``) when it is shared; for a
    per-image shift the caller folds it into the style GEMM constants instead (``tb`` then None).
    ``bias`` is convB's bias plus the projection's bias."""

    pa: PackedConv
    pb: PackedConv
    sa: torch.Tensor
    ta: torch.Tensor | None
    sb: torch.Tensor
    tb: torch.Tensor | None
    bias: torch.Tensor
    inmode: str = "none"
    pp: PackedConv | None = None
    sp: torch.Tensor | None = None
    tp: torch.Tensor | None = None

    @property
    def cm(self) -> int:
        return self.pb.cout

    @property
    def cin(self) -> int:
        return self.pa.cin_pad

    def supports(self, has_x2: bool, res: str) -> bool:
        return (self.cin, self.cm, self.inmode, has_x2, self.pp is not None, res) in SUPPORTED


def fold_bias(shift: torch.Tensor, scale: torch.Tensor, bias: torch.Tensor | None) -> torch.Tensor:
    """``t + s * b``: a conv bias pushed through the next pre-activation affine."""
    if bias is None:
        return shift.clone()
    n = bias.numel()
    out = shift.clone()
    out[..., :n] = out[..., :n] + scale[:n] * bias.to(shift.device)
    return out


def _out_hw(x: torch.Tensor, inmode: str) -> tuple[int, int]:
    Hs, Ws = x.shape[1], x.shape[2]
    if inmode == "up2":
        return 2 * Hs, 2 * Ws
    if inmode == "pool2":
        return Hs // 2, Ws // 2
    return Hs, Ws


def conv_pair_ref(x, spec: PairSpec, *, ta=None, tb=None, x2=None, res=None, res_mode="none"):
    """fp32 PyTorch oracle with the kernel's two bf16 rounding points (activated input, h)."""
    ta = spec.ta if ta is None else ta
    tb = spec.tb if tb is None else tb
    xf = x.float()
    a = _act_ref(xf, None, spec.sa, ta, True, spec.inmode).to(torch.bfloat16).float()
    wa = spec.pa.w.to(a.device)
    if wa.shape[1] < a.shape[1]:
        wa = F.pad(wa, (0, 0, 0, 0, 0, a.shape[1] - wa.shape[1]))
    hA = F.conv2d(a, wa.to(torch.bfloat16).float(), None, padding=1)
    if x2 is not None:
        hA = hA + x2.float().permute(0, 3, 1, 2)
    C = hA.shape[1]
    sb = spec.sb[:C].view(1, C, 1, 1)
    tbv = tb.view(-1, tb.shape[-1], 1, 1)[:, :C] if tb.dim() == 2 else tb[:C].view(1, C, 1, 1)
    h = torch.relu(hA * sb + tbv).to(torch.bfloat16).float()
    y = F.conv2d(h, spec.pb.w.to(h.device).to(torch.bfloat16).float(), None, padding=1)
    if spec.pp is not None:
        p = _act_ref(xf, None, spec.sp, spec.tp, False, spec.inmode).to(torch.bfloat16).float()
        wp = spec.pp.w.to(p.device)
        if wp.shape[1] < p.shape[1]:
            wp = F.pad(wp, (0, 0, 0, 0, 0, p.shape[1] - wp.shape[1]))
        y = y + F.conv2d(p, wp.to(torch.bfloat16).float(), None)
    y = y + spec.bias.to(y.device).view(1, -1, 1, 1)
    y = y.permute(0, 2, 3, 1)
    if res is not None:
        r = res.float()
        if res_mode == "up2":
            r = r.repeat_interleave(2, 1).repeat_interleave(2, 2)
        y = y + r
    return y.to(x.dtype).contiguous()


def conv_pair(x: torch.Tensor, spec: PairSpec, *, ta=None, tb=None, x2=None, res=None, res_mode: str = "none",
              out: torch.Tensor | None = None) -> torch.Tensor:
    """Run the fused half-block on NHWC bf16 ``x`` [N, Hs, Ws, Cin]; returns [N, H, W, CM] bf16.
    ``ta``/``tb`` override the spec's shifts (per-image [N, C] rows, convA bias already folded into
    ``tb``); ``res_mode`` is "full" (``res`` at output resolution) or "up2" (``res`` at half)."""
    ta = spec.ta if ta is None else ta
    tb = spec.tb if tb is None else tb
    assert ta is not None and tb is not None, "conv_pair needs actA / actB shifts"
    if res is None:
        res_mode = "none"
    if not x.is_cuda:
        y = conv_pair_ref(x, spec, ta=ta, tb=tb, x2=x2, res=res, res_mode=res_mode)
        if out is not None:
            out.copy_(y)
            return out
        return y
    N, Hs, Ws, Cin = x.shape
    H, W = _out_hw(x, spec.inmode)
    CM = spec.cm
    assert x.dtype == torch.bfloat16 and x.is_contiguous(), "conv_pair expects contiguous NHWC bf16"
    assert Cin == spec.cin, f"input channels {Cin} != packed {spec.cin}"
    if not spec.supports(x2 is not None, res_mode):
        raise ValueError(f"conv_pair: unsupported configuration {(Cin, CM, spec.inmode, x2 is not None, spec.pp is not None, res_mode)}")
    if x2 is not None:
        assert x2.shape == (N, H, W, CM) and x2.dtype == torch.bfloat16 and x2.is_contiguous()
    if res_mode == "full":
        assert res.shape == (N, H, W, CM) and res.dtype == torch.bfloat16 and res.is_contiguous()
    elif res_mode == "up2":
        assert res.shape == (N, H // 2, W // 2, CM) and res.dtype == torch.bfloat16 and res.is_contiguous()
    if out is None:
        out = torch.empty(N, H, W, CM, device=x.device, dtype=torch.bfloat16)
    else:
        assert out.shape == (N, H, W, CM) and out.dtype == torch.bfloat16 and out.is_contiguous()
        assert out.data_ptr() != x.data_ptr(), "conv_pair cannot run in place"
    ta_ns = _affine_stride(ta, N, Cin)
    tb_ns = _affine_stride(tb, N, CM)
    pp = spec.pp
    rc = _native.call(
        "be_conv_pair",
        _native.ptr(x), _native.ptr(x2), _native.ptr(spec.sa), _native.ptr(ta), ta_ns, _native.ptr(spec.sb),
        _native.ptr(tb), tb_ns, _native.ptr(spec.sp), _native.ptr(spec.tp), _native.ptr(spec.pa.wp),
        _native.ptr(spec.pb.wp), _native.ptr(None if pp is None else pp.wp), _native.ptr(spec.bias),
        _native.ptr(res), _native.ptr(out), N, H, W, Hs, Ws, Cin, CM, INMODES[spec.inmode], int(pp is not None),
        RESMODES[res_mode], _native.stream(x.device),
    )
    return out


@dataclass
class HeadSpec:
    """The network's output layer (``relu(v * s + t)`` then a 1x1 conv with bias; eval BN folded)
    fused into the epilogue of the final 32-channel half-block (kernel ``be_conv_pair_head``).
    ``wh``: bf16 [16, 32], rows = output channels (zero past ``nh``), k axis permuted to the
    accumulator layout (lane group kq holds channels 4kq..4kq+3 and 16+4kq..16+4kq+3)."""

    s: torch.Tensor
    t: torch.Tensor
    w: torch.Tensor      # fp32 [nh, 32] original weights (reference path)
    b: torch.Tensor      # fp32 [16] bias, zero padded
    nh: int
    wh: torch.Tensor | None = None

    @staticmethod
    def k_order() -> list[int]:
        return [(kq * 4 + j) if j < 4 else (16 + kq * 4 + j - 4) for kq in range(4) for j in range(8)]

    @classmethod
    def build(cls, scale: torch.Tensor, shift: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None):
        nh, cin = weight.shape[0], weight.shape[1]
        assert cin <= 32 and nh <= 16 and weight.shape[2:] == (1, 1)
        dev = weight.device
        w = torch.zeros(nh, 32, device=dev)
        w[:, :cin] = weight.detach().float().reshape(nh, cin)
        b = torch.zeros(16, device=dev)
        if bias is not None:
            b[:nh] = bias.detach().float()
        s = torch.zeros(32, device=dev)
        t = torch.zeros(32, device=dev)
        s[: scale.numel()] = scale.float()
        t[: shift.numel()] = shift.float()
        wp = torch.zeros(16, 32, device=dev)
        wp[:nh] = w[:, cls.k_order()]
        return cls(s=s.contiguous(), t=t.contiguous(), w=w, b=b.contiguous(), nh=nh,
                   wh=wp.to(torch.bfloat16).contiguous())


def head_ref(xout: torch.Tensor, head: HeadSpec) -> torch.Tensor:
    """fp32 oracle of the fused head from the block output ``xout`` (NHWC bf16): the activated input is
    rounded to bf16 as the kernel's MFMA operand is."""
    a = torch.relu(xout.float() * head.s.to(xout.device) + head.t.to(xout.device))
    w = head.w.to(a.device)
    if xout.dtype == torch.bfloat16:  # the GPU path's rounding points (CPU fp32 runs stay fp32)
        a = a.to(torch.bfloat16).float()
        w = w.to(torch.bfloat16).float()
    y = torch.einsum("nhwc,oc->nohw", a, w) + head.b[: head.nh].to(a.device).view(1, -1, 1, 1)
    return y.contiguous()


def conv_pair_head(x: torch.Tensor, spec: PairSpec, head: HeadSpec, *, ta=None, tb=None, res=None) -> torch.Tensor:
    """Final up half-block (32 -> 32 channels, ``+ res`` at full resolution) with the output layer fused:
    returns fp32 NCHW [N, nh, H, W]; the block's own 32-channel output never reaches HBM."""
    ta = spec.ta if ta is None else ta
    tb = spec.tb if tb is None else tb
    assert ta is not None and tb is not None and res is not None
    if not x.is_cuda:
        return head_ref(conv_pair_ref(x, spec, ta=ta, tb=tb, res=res, res_mode="full"), head)
    N, H, W, Cin = x.shape
    assert spec.cin == 32 and spec.cm == 32 and spec.inmode == "none" and spec.pp is None, "head fusion: 32->32 only"
    assert x.dtype == torch.bfloat16 and x.is_contiguous() and Cin == 32
    assert res.shape == (N, H, W, 32) and res.dtype == torch.bfloat16 and res.is_contiguous()
    hout = torch.empty(N, head.nh, H, W, device=x.device, dtype=torch.float32)
    _native.call(
        "be_conv_pair_head",
        _native.ptr(x), _native.ptr(spec.sa), _native.ptr(ta), _affine_stride(ta, N, Cin), _native.ptr(spec.sb),
        _native.ptr(tb), _affine_stride(tb, N, 32), _native.ptr(spec.pa.wp), _native.ptr(spec.pb.wp),
        _native.ptr(spec.bias), _native.ptr(res), _native.ptr(head.s), _native.ptr(head.t), _native.ptr(head.wh),
        _native.ptr(head.b), _native.ptr(hout), head.nh, N, H, W, _native.stream(x.device),
    )
    return hout
