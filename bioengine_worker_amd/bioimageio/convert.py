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

Convolutions that do not match (strided, dilated, grouped, 3-D, 5x5, ...) stay on MIOpen.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.conv import PackedConv, fused_conv2d


def _eligible(c: nn.Module) -> bool:
    return (isinstance(c, nn.Conv2d) and type(c) is nn.Conv2d and c.kernel_size in ((1, 1), (3, 3))
            and c.stride == (1, 1) and c.dilation == (1, 1) and c.groups == 1 and c.padding_mode == "zeros"
            and c.padding == ((c.kernel_size[0] // 2, c.kernel_size[1] // 2)))


def fold_bn(conv: nn.Conv2d, bn: nn.BatchNorm2d) -> nn.Conv2d:
    w = conv.weight.detach().float()
    b = conv.bias.detach().float() if conv.bias is not None else torch.zeros(w.shape[0], device=w.device)
    rstd = torch.rsqrt(bn.running_var.float() + bn.eps)
    g = bn.weight.detach().float() if bn.weight is not None else torch.ones_like(rstd)
    beta = bn.bias.detach().float() if bn.bias is not None else torch.zeros_like(rstd)
    new = nn.Conv2d(conv.in_channels, conv.out_channels, conv.kernel_size, conv.stride, conv.padding, conv.dilation,
                    conv.groups, True, conv.padding_mode).to(w.device)
    with torch.no_grad():
        new.weight.copy_(w * (g * rstd)[:, None, None, None])
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


def _rewrite(mod: nn.Module, stats: dict) -> None:
    for name, child in list(mod.named_children()):
        if isinstance(child, nn.Sequential):
            items = list(child._modules.items())
            i = 0
            while i < len(items):
                k, m = items[i]
                if isinstance(m, nn.Conv2d):
                    conv = m
                    j = i + 1
                    if j < len(items) and isinstance(items[j][1], nn.BatchNorm2d) and not items[j][1].training:
                        conv = fold_bn(conv, items[j][1])
                        child._modules[items[j][0]] = nn.Identity()
                        stats["bn_folded"] += 1
                        j += 1
                    relu = j < len(items) and isinstance(items[j][1], nn.ReLU)
                    if _eligible(conv):
                        child._modules[k] = HipConv2d(conv, post_relu=relu)
                        stats["convs"] += 1
                        if relu:
                            child._modules[items[j][0]] = nn.Identity()
                            stats["relu_fused"] += 1
                    else:
                        child._modules[k] = conv
                        stats["skipped"] += 1
                    i = j + (1 if relu and _eligible(conv) else 0)
                    continue
                _rewrite(m, stats)
                i += 1
        elif _eligible(child):
            setattr(mod, name, HipConv2d(child))
            stats["convs"] += 1
        elif isinstance(child, nn.Conv2d):
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
