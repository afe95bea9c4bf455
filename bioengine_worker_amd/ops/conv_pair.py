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
