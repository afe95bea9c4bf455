"""MI355X graph pass for arbitrary PyTorch image models.

``optimize_for_mi355x(model)``:

1. folds every ``BatchNorm2d`` (eval statistics) that directly follows a ``Conv2d`` in an
   ``nn.Sequential`` into that conv's weights and bias;
2. replaces every eligible ``Conv2d`` (1x1 or 3x3, stride 1, dilation 1, groups 1, "same" padding
   with zeros) by :class:`HipConv2d`, absorbing a directly following ``ReLU`` into the kernel's
   output epilogue (``post_relu``);
3. casts the model to bf16 and runs activations channels-last (NHWC in memory), which is the
   fused conv kernel's native layout — a channels-last NCHW-shaped tensor *is* an NHWC buffer, so
   the remaining torch ops (pooling, upsampling, concatenation, transposed convs) consume the
   kernel's outputs without copies.

4. does the same for 3-D models: ``Conv3d`` (1x1x1 / 3x3x3, stride 1, "same" zero padding)
   + ``BatchNorm3d`` + ``ReLU`` become :class:`HipConv3d` (``ops/conv3d.py``: depth-tap
   decomposition onto the same MFMA kernel), activations run ``channels_last_3d`` (NDHWC).

Convolutions that do not match (strided, dilated, grouped, 5x5, ...) stay on MIOpen.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.conv import PackedConv, fused_conv2d
from ..ops.conv3d import PackedConv3d, fused_conv3d


def _eligible(c: nn.Module) -> bool:
    return (isinstance(c, nn.Conv2d) and type(c) is nn.Conv2d and c.kernel_size in ((1, 1), (3, 3))
            and c.stride == (1, 1) and c.dilation == (1, 1) and c.groups == 1 and c.padding_mode == "zeros"
            and c.padding == ((c.kernel_size[0] // 2, c.kernel_size[1] // 2)))


def _eligible3d(c: nn.Module) -> bool:
    return (type(c) is nn.Conv3d and c.kernel_size in ((1, 1, 1), (3, 3, 3)) and c.stride == (1, 1, 1)
            and c.dilation == (1, 1, 1) and c.groups == 1 and c.padding_mode == "zeros"
            and c.padding == tuple(k // 2 for k in c.kernel_size) and c.out_channels % 4 == 0)


_CONV = (nn.Conv2d, nn.Conv3d)
_BN = {nn.Conv2d: nn.BatchNorm2d, nn.Conv3d: nn.BatchNorm3d}


def fold_bn(conv, bn):
    """Fold eval BatchNorm{2,3}d statistics into the preceding Conv{2,3}d (new conv with bias)."""
    w = conv.weight.detach().float()
    b = conv.bias.detach().float() if conv.bias is not None else torch.zeros(w.shape[0], device=w.device)
    rstd = torch.rsqrt(bn.running_var.float() + bn.eps)
    g = bn.weight.detach().float() if bn.weight is not None else torch.ones_like(rstd)
    beta = bn.bias.detach().float() if bn.bias is not None else torch.zeros_like(rstd)
    new = type(conv)(conv.in_channels, conv.out_channels, conv.kernel_size, conv.stride, conv.padding, conv.dilation,
                     conv.groups, True, conv.padding_mode).to(w.device)
    with torch.no_grad():
        new.weight.copy_(w * (g * rstd).view(-1, *([1] * (w.dim() - 1))))
        new.bias.copy_((b - bn.running_mean.float()) * g * rstd + beta)
    return new


class HipConv2d(nn.Module):
    """Conv2d (+ folded BN)(+ ReLU) on the fused NHWC MFMA conv kernel."""

    def __init__(self, conv: nn.Conv2d, post_relu: bool = False):
        super().__init__()
        self.cin, self.cout = conv.in_channels, conv.out_channels
        self.post_relu = post_relu
        self.nchw_out = self.cout % 4 != 0
        self.pc = PackedConv.from_weight(conv.weight.detach().float(),
                                         None if conv.bias is None else conv.bias.detach().float(),
                                         cout_pad_to=16 if self.nchw_out else None)
        self._dev = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not x.is_cuda:  # CPU: reference math (bf16-rounded like the kernel)
            y = F.conv2d(x.float(), self.pc.w.to(x.device), None if self.pc.bias is None else self.pc.bias.to(x.device),
                         padding=self.pc.ks // 2)
            y = torch.relu(y) if self.post_relu else y
            return y.to(x.dtype)
        if self._dev != x.device:
            self.pc.to(x.device)
            self._dev = x.device
        N, C, H, W = x.shape
        xh = x.to(torch.bfloat16).permute(0, 2, 3, 1)
        if C != self.pc.cin_pad:
            xh = F.pad(xh, (0, self.pc.cin_pad - C))
        xh = xh.contiguous()
        if self.nchw_out:
            return fused_conv2d(xh, self.pc, out_nchw_f32=True, cout_valid=self.cout, post_relu=self.post_relu)
        y = fused_conv2d(xh, self.pc, post_relu=self.post_relu)  # [N, H, W, Cout] bf16
        return y.permute(0, 3, 1, 2)  # channels-last view, no copy

    def extra_repr(self) -> str:
        return f"{self.cin}, {self.cout}, k={self.pc.ks}, post_relu={self.post_relu}"


class HipConv3d(nn.Module):
    """Conv3d (+ folded BN)(+ ReLU) on the fused NHWC MFMA conv kernel (depth-tap decomposition)."""

    def __init__(self, conv: nn.Conv3d, post_relu: bool = False):
        super().__init__()
        self.cin, self.cout = conv.in_channels, conv.out_channels
        self.post_relu = post_relu
        self.pc = PackedConv3d(conv.weight.detach().float(), None if conv.bias is None else conv.bias.detach().float())
        self._dev = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not x.is_cuda:  # CPU: fp32 reference math in the input dtype
            y = F.conv3d(x.float(), self.pc.w.to(x.device),
                         None if self.pc.bias is None else self.pc.bias.to(x.device), padding=self.pc.ks // 2)
            y = torch.relu(y) if self.post_relu else y
            return y.to(x.dtype)
        if self._dev != x.device:
            self.pc.to(x.device)
            self._dev = x.device
        C = x.shape[1]
        xh = x.to(torch.bfloat16).permute(0, 2, 3, 4, 1)  # NDHWC (a view for channels_last_3d inputs)
        if C != self.pc.cin_pad:
            xh = F.pad(xh, (0, self.pc.cin_pad - C))
        y = fused_conv3d(xh.contiguous(), self.pc, post_relu=self.post_relu)  # [N, D, H, W, Cout]
        return y.permute(0, 4, 1, 2, 3)  # channels_last_3d view, no copy

    def extra_repr(self) -> str:
        return f"{self.cin}, {self.cout}, k={self.pc.ks}, post_relu={self.post_relu}"


def _hip_conv(conv, post_relu: bool = False):
    return HipConv3d(conv, post_relu) if isinstance(conv, nn.Conv3d) else HipConv2d(conv, post_relu)


def _ok(conv) -> bool:
    return _eligible3d(conv) if isinstance(conv, nn.Conv3d) else _eligible(conv)


def _rewrite(mod: nn.Module, stats: dict) -> None:
    for name, child in list(mod.named_children()):
        if isinstance(child, nn.Sequential):
            items = list(child._modules.items())
            i = 0
            while i < len(items):
                k, m = items[i]
                if type(m) in _CONV:
                    conv = m
                    j = i + 1
                    if j < len(items) and isinstance(items[j][1], _BN[type(m)]) and not items[j][1].training:
                        conv = fold_bn(conv, items[j][1])
                        child._modules[items[j][0]] = nn.Identity()
                        stats["bn_folded"] += 1
                        j += 1
                    relu = j < len(items) and isinstance(items[j][1], nn.ReLU)
                    if _ok(conv):
                        child._modules[k] = _hip_conv(conv, post_relu=relu)
                        stats["convs"] += 1
                        if relu:
                            child._modules[items[j][0]] = nn.Identity()
                            stats["relu_fused"] += 1
                    else:
                        child._modules[k] = conv
                        stats["skipped"] += 1
                    i = j + (1 if relu and _ok(conv) else 0)
                    continue
                _rewrite(m, stats)
                i += 1
        elif type(child) in _CONV and _ok(child):
            setattr(mod, name, _hip_conv(child))
            stats["convs"] += 1
        elif isinstance(child, _CONV):
            stats["skipped"] += 1
        else:
            _rewrite(child, stats)


def optimize_for_mi355x(model: nn.Module, device=None) -> tuple[nn.Module, dict]:
    """In-place graph pass (model must be in eval mode).  Returns (model, stats)."""
    model.eval()
    stats = {"convs": 0, "bn_folded": 0, "relu_fused": 0, "skipped": 0}
    _rewrite(model, stats)
    if device is not None:
        model.to(device)
    model.to(torch.bfloat16)
    return model, stats
