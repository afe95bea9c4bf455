"""3x3 conv as a linear-tile implicit GEMM (HIP kernel ``csrc/kernels/conv_igemm.hip``).

``conv3_igemm(x, pk)`` computes, on an ALREADY ACTIVATED NHWC bf16 input::

    out  = conv3x3(x) + bias [+ residual]                 (optional, bf16 NHWC)
    aout = relu?( out * ascale[c] + ashift[n, c] )        (optional: the consumer's pre-activation)

The producer-side ``aout`` is how the Cellpose CPnet engine feeds these kernels: every deep conv's
BN + ReLU (+ style shift) is applied once by the conv that produced its input, so the kernel itself
stages both operands HBM -> LDS by DMA with no per-element work on the way in (SURVEY.md §2.5 K1;
the reference's cellpose ``batchconv`` = BatchNorm2d -> ReLU -> Conv2d, reached through
``apps/model-runner/runtime_deployment.py:19``).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn.functional as F

from . import _native


@dataclass
class IgemmConv:
    """3x3 weights packed in the kernel's LDS image order: [Cout/bnc][Cin/16][9][bnc/32][2][32][8]."""

    w: torch.Tensor            # fp32 [Cout, Cin, 3, 3]
    bias: torch.Tensor | None  # fp32 [Cout]
    cin: int
    cout: int
    bn: int
    wp: torch.Tensor | None = None

    @property
    def bnc(self) -> int:
        """Output channels per block (bn 65 is the 512 x 64, 8-wave A/B variant of bn 64)."""
        return 128 if self.bn % 1000 == 128 else 64

    @classmethod
    def from_weight(cls, weight: torch.Tensor, bias: torch.Tensor | None = None, bn: int | None = None) -> "IgemmConv":
        """``bn``: 64 (default; 256 px x 64 ch on 4 waves, two blocks per CU), 128 (256 x 128, 8 waves)
        or 65 (512 x 64, 8 waves); + 1000 = three LDS stages (DMA two chunks ahead)."""
        cout, cin, kh, kw = weight.shape
        assert kh == 3 and kw == 3 and cin % 16 == 0 and cout % 64 == 0, "3x3, Cin % 16 == 0, Cout % 64 == 0"
        bn = bn or 64
        assert bn in (64, 65, 128, 1065, 1128) and cout % (128 if bn % 1000 == 128 else 64) == 0
        pk = cls(w=weight.detach().float(), bias=None if bias is None else bias.detach().float().contiguous(),
                 cin=cin, cout=cout, bn=bn)
        pk.wp = pk.pack(pk.w)
        return pk

    def pack(self, w: torch.Tensor) -> torch.Tensor:
        co, ci, bn = self.cout, self.cin, self.bnc
        # [co_blk, f, co32, c16, h, j, t]
        t = w.reshape(co // bn, bn // 32, 32, ci // 16, 2, 8, 9)
        # -> [co_blk, c16, t, f, h, co32, j]
        t = t.permute(0, 3, 6, 1, 4, 2, 5)
        return t.contiguous().to(torch.bfloat16).reshape(-1)

    def to(self, device) -> "IgemmConv":
        self.w = self.w.to(device)
        if self.bias is not None:
            self.bias = self.bias.to(device)
        self.wp = self.wp.to(device)
        return self


def supported(N: int, H: int, W: int, cout: int, bn: int) -> bool:
    """Whether the kernel's halo for this image geometry fits its LDS budget."""
    return _native.hip().be_conv3_igemm_lds(N, H, W, cout, bn) > 0


def conv3_igemm_ref(x, pk: IgemmConv, residual=None, ascale=None, ashift=None, arelu=True, post_relu=False):
    """fp32 reference of the same op (bf16 operands, fp32 accumulation); returns (out, aout)."""
    xt = x.float().permute(0, 3, 1, 2)
    y = F.conv2d(xt, pk.w.to(torch.bfloat16).float().to(x.device), None, padding=1).permute(0, 2, 3, 1)
    if pk.bias is not None:
        y = y + pk.bias.to(y.device)
    if residual is not None:
        y = y + residual.float()
    if post_relu:
        y = torch.relu(y)
    out = y.to(torch.bfloat16)
    aout = None
    if ascale is not None or ashift is not None:
        a = out.float()
        if ascale is not None:
            a = a * ascale.to(a.device)
        if ashift is not None:
            sh = ashift.to(a.device)
            a = a + (sh[:, None, None, :] if sh.dim() == 2 else sh)
        if arelu:
            a = torch.relu(a)
        aout = a.to(torch.bfloat16)
    return out, aout


def conv3_igemm(x: torch.Tensor, pk: IgemmConv, *, residual=None, want_out: bool = True, ascale=None, ashift=None,
                arelu: bool = True, post_relu: bool = False, out=None, aout=None):
    """Returns ``(out, aout)``; ``out`` is None when ``want_out`` is False, ``aout`` None without an
    activation (``ascale`` / ``ashift``).  ``ashift`` may be [Cout] or a row-strided [N, Cout] view."""
    N, H, W, C = x.shape
    assert C == pk.cin
    if not x.is_cuda:
        o, a = conv3_igemm_ref(x, pk, residual, ascale, ashift, arelu, post_relu)
        return (o if want_out else None), a
    assert x.dtype == torch.bfloat16 and x.is_contiguous()
    if pk.wp.device != x.device:
        pk.to(x.device)
    if want_out and out is None:
        out = torch.empty(N, H, W, pk.cout, device=x.device, dtype=torch.bfloat16)
    act = ascale is not None or ashift is not None
    if act and aout is None:
        aout = torch.empty(N, H, W, pk.cout, device=x.device, dtype=torch.bfloat16)
    if residual is not None:
        assert residual.shape == (N, H, W, pk.cout) and residual.dtype == torch.bfloat16 and residual.is_contiguous()
    at_ns = 0
    if ashift is not None:
        assert ashift.dtype == torch.float32
        if ashift.dim() == 2:
            assert ashift.shape == (N, pk.cout) and ashift.stride(1) == 1
            at_ns = ashift.stride(0) if N > 1 else pk.cout
            assert at_ns % 4 == 0 and ashift.data_ptr() % 16 == 0
        else:
            assert ashift.is_contiguous() and ashift.numel() == pk.cout
    if ascale is not None:
        assert ascale.dtype == torch.float32 and ascale.is_contiguous() and ascale.numel() == pk.cout
    _native.call("be_conv3_igemm", _native.ptr(x), _native.ptr(pk.wp), _native.ptr(pk.bias), _native.ptr(residual),
                 _native.ptr(out if want_out else None), _native.ptr(aout if act else None), _native.ptr(ascale),
                 _native.ptr(ashift), at_ns, int(bool(arelu)), int(bool(post_relu)), N, H, W, pk.cin, pk.cout, pk.bn,
                 _native.stream(x.device))
    return (out if want_out else None), (aout if act else None)
