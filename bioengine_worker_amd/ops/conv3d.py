"""3-D convolution (1x1x1 / 3x3x3, stride 1, "same" zero padding) on the fused NHWC MFMA conv kernel.

BioImage.IO 3-D U-Nets (PlantSeg / 3D-UNet family; the model runner's 3-D path, SURVEY.md §2.5 K16,
and the fibsem volume workloads) are stacks of Conv3d(k=3) + BN + ReLU.  On MI355X they run on
the same hand-written implicit-GEMM kernel as the 2-D layers (``csrc/kernels/conv2d_nhwc.hip``),
with the depth axis decomposed into its three taps:

    out[z] = conv2d(x[z-1], W[:, :, 0]) + conv2d(x[z], W[:, :, 1]) + conv2d(x[z+1], W[:, :, 2]) + b

* activations are NDHWC bf16 (PyTorch ``channels_last_3d``): a run of z-slices of one sample is a
  contiguous [D', H, W, C] batch for the 2-D kernel, so each tap is ONE launch over all its slices;
* the centre tap writes ``out`` (with the bias), the two outer taps accumulate into it through the
  kernel's residual epilogue in place (their z-ranges are shifted by one slice, which is the zero
  padding at the volume faces), and the last tap applies the fused post-ReLU;
* 1x1x1 convs are a single 2-D 1x1 launch over all N*D slices.

Each output is rounded to bf16 between taps (the partial sums are bf16, like the activations), so
the numerics test allows three bf16 roundings.  CPU tensors run ``F.conv3d`` (the fp32 oracle).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .conv import PackedConv, fused_conv2d


class PackedConv3d:
    """A Conv3d weight [Cout, Cin, k, k, k] split into k PackedConv 2-D taps (z-major)."""

    def __init__(self, weight: torch.Tensor, bias: torch.Tensor | None = None, cout_pad_to: int | None = None):
        cout, cin, kd, kh, kw = weight.shape
        assert kd == kh == kw and kd in (1, 3), "only 1x1x1 / 3x3x3 convs"
        self.ks = kd
        self.w = weight.detach().float()
        self.bias = None if bias is None else bias.detach().float()
        self.cin, self.cout = cin, cout
        self.taps = [PackedConv.from_weight(self.w[:, :, dz], self.bias if dz == kd // 2 else None,
                                            cout_pad_to=cout_pad_to) for dz in range(kd)]
        self.cin_pad = self.taps[0].cin_pad

    def to(self, device) -> "PackedConv3d":
        for t in self.taps:
            t.to(device)
        self.w = self.w.to(device)
        if self.bias is not None:
            self.bias = self.bias.to(device)
        return self


def conv3d_ref(x: torch.Tensor, pc: PackedConv3d, post_relu: bool = False) -> torch.Tensor:
    """NDHWC reference: bf16-rounded operands, fp32 math, result in x's dtype."""
    xc = x.float().permute(0, 4, 1, 2, 3)
    w = pc.w.to(x.device)
    if w.shape[1] < xc.shape[1]:
        w = F.pad(w, (0, 0, 0, 0, 0, 0, 0, xc.shape[1] - w.shape[1]))
    if x.dtype == torch.bfloat16:
        w = w.to(torch.bfloat16).float()
    y = F.conv3d(xc, w, None if pc.bias is None else pc.bias.to(x.device), padding=pc.ks // 2)
    if post_relu:
        y = torch.relu(y)
    return y.permute(0, 2, 3, 4, 1).to(x.dtype).contiguous()


def fused_conv3d(x: torch.Tensor, pc: PackedConv3d, post_relu: bool = False) -> torch.Tensor:
    """x: NDHWC [N, D, H, W, Cin_pad] (bf16 contiguous on GPU) -> NDHWC [N, D, H, W, Cout]."""
    if not x.is_cuda:
        return conv3d_ref(x, pc, post_relu)
    N, D, H, W, C = x.shape
    assert C == pc.cin_pad and x.dtype == torch.bfloat16 and x.is_contiguous()
    if pc.ks == 1:
        y = fused_conv2d(x.view(N * D, H, W, C), pc.taps[0], post_relu=post_relu)
        return y.view(N, D, H, W, pc.cout)
    out = torch.empty(N, D, H, W, pc.cout, device=x.device, dtype=torch.bfloat16)
    below, centre, above = pc.taps
    for n in range(N):
        xn, on = x[n], out[n]
        fused_conv2d(xn, centre, out=on, post_relu=post_relu and D == 1)
        if D == 1:
            continue
        # out[z] += conv(x[z-1], W0) for z >= 1 ; out[z] += conv(x[z+1], W2) for z <= D-2
        fused_conv2d(xn[:-1], below, residual=on[1:], out=on[1:], no_bias=True)
        fused_conv2d(xn[1:], above, residual=on[:-1], out=on[:-1], no_bias=True, post_relu=post_relu)
        if post_relu:
            on[-1].relu_()  # the last slice has no z+1 tap: its ReLU is the only pass left
    return out
