"""3-D convolution (1x1x1 / 3x3x3, stride 1, "same" zero padding) on the framework's MFMA kernels.

3x3x3 convs run as ONE launch of the LDS-staged 2-D conv kernel over the N*D slices with the three
depth taps stacked on K (``be_conv3d_ztaps`` in ``csrc/kernels/conv2d_nhwc.hip``, INMODE 3: stacked
channel dz*Cin + c is channel c of slice z+dz-1, zero outside the volume): fp32 accumulation across all
27 taps, one bf16 rounding, bias + ReLU in the epilogue, and each input voxel staged ~3x per output
tile instead of gathered 27x from L2.  ``BE_CONV3D=igemm`` selects the one-launch implicit GEMM
(``be_conv3d_mt`` in ``gemm_mt.hip``, the round-5 default, also the fallback when the stacked layout
does not apply, e.g. a 1-channel input); the older three-launch depth-tap decomposition below
(``BE_CONV3D=taps``) is kept as an A/B path.

Depth-tap decomposition (A/B path):

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

import os

from . import _native
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
        # NARROW (default): a 16-channel layer keeps 16 input channels instead of being padded to 32 --
        # no padded copy of the activation in front of every such conv, fewer MFMA K steps, and the
        # 1-channel stem takes the z-tap path too: 683 vs 555 M voxel/s (profiles/r06/em3d/
        # narrow_ck16_ab_s18.txt; BE_CONV3D_NARROW=0: the padded layout, A/B)
        narrow = os.environ.get("BE_CONV3D_NARROW", "1") != "0"
        self.taps = [PackedConv.from_weight(self.w[:, :, dz], self.bias if dz == kd // 2 else None,
                                            cout_pad_to=cout_pad_to, exact_cin=narrow) for dz in range(kd)]
        self.cin_pad = self.taps[0].cin_pad
        if kd == 3:
            # implicit-GEMM weights [Cout][kpad], k = (9 dz + 3 dy + dx) * cin_pad + c, zero-padded to 64
            w = self.w.permute(0, 2, 3, 4, 1)  # [Cout, 3, 3, 3, Cin]
            w = F.pad(w, (0, self.cin_pad - cin)).reshape(cout, 27 * self.cin_pad)
            self.kpad = (27 * self.cin_pad + 63) // 64 * 64
            self.w_mt = F.pad(w, (0, self.kpad - 27 * self.cin_pad)).to(torch.bfloat16).contiguous()
            self.b_mt = (self.bias if self.bias is not None else torch.zeros(cout)).float().contiguous()
            # z-tap stacked 2-D weights for be_conv3d_ztaps: W'[co][dz * cin_pad + c][ky][kx]
            wz = F.pad(self.w, (0, 0, 0, 0, 0, 0, 0, self.cin_pad - cin)).permute(0, 2, 1, 3, 4)
            # 16-channel K chunks for the 16-channel layers (5 instead of 6 K steps per 16 channels, half
            # the chunk iterations): 707-710 vs 683-684 M voxel/s on the 3-D line's 64 x 2048^2 slab
            # (profiles/r06/em3d/narrow_ck16_ab_s18.txt); BE_CONV3D_CK16=0: 8-channel chunks (A/B)
            ck16 = os.environ.get("BE_CONV3D_CK16", "1") == "1"
            self.ztap = PackedConv.from_weight(wz.reshape(cout, 3 * self.cin_pad, 3, 3), self.bias,
                                               cin_pad=3 * self.cin_pad, exact_cin=narrow, ck16=ck16)

    def to(self, device) -> "PackedConv3d":
        for t in self.taps:
            t.to(device)
        if self.ks == 3:
            self.w_mt, self.b_mt = self.w_mt.to(device), self.b_mt.to(device)
            self.ztap.to(device)
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
    # ztaps (default): one launch of the LDS-staged 2-D kernel with the depth taps stacked on K --
    # 492 vs 351 M voxel/s for the one-launch implicit GEMM on the 3-D EM line (profiles/r06/em3d/
    # conv3d_path_ab_s8.txt): the narrow 3-D U-Net layers were bound by the igemm's 27x per-tap L2
    # gather.  igemm / taps: the previous default / the three-launch decomposition (A/B)
    mode = os.environ.get("BE_CONV3D", "ztaps")
    taps_maxcin = int(os.environ.get("BE_CONV3D_TAPS_MAXCIN", "0"))  # A/B: narrow layers on the taps path
    if mode == "ztaps" and pc.cout % 4 == 0 and pc.ztap.cin_pad == 3 * C and C % pc.ztap.ck == 0:
        out = torch.empty(N, D, H, W, pc.cout, device=x.device, dtype=torch.bfloat16)
        zt = pc.ztap
        _native.call("be_conv3d_ztaps", _native.ptr(x), _native.ptr(zt.wp), _native.ptr(zt.bias), _native.ptr(out),
                     N, D, H, W, C, pc.cout, zt.ck, zt.tco, int(post_relu), 4, _native.stream(x.device))
        return out
    if mode != "taps" and pc.cout % 4 == 0 and C > taps_maxcin:
        out = torch.empty(N, D, H, W, pc.cout, device=x.device, dtype=torch.bfloat16)
        cfg = 5 if pc.cout <= 32 else (6 if pc.cout <= 64 else 4)
        _native.call("be_conv3d_mt", _native.ptr(x), _native.ptr(pc.w_mt), _native.ptr(pc.b_mt), _native.ptr(out),
                     N, D, H, W, C, pc.cout, pc.kpad, int(post_relu), cfg, _native.stream(x.device))
        return out
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


def fused_conv3d_concat(xa: torch.Tensor, xb: torch.Tensor, pc: PackedConv3d, post_relu: bool = False) -> torch.Tensor:
    """3x3x3 conv of the channel concatenation [xa, xb] of two NDHWC volumes without materialising it
    (``be_conv3d_ztaps_concat``, INMODE 5); same K order and accumulation as :func:`fused_conv3d` on
    ``torch.cat([xa, xb], -1)`` along the z-tap path."""
    N, D, H, W, Ca = xa.shape
    Cb = xb.shape[-1]
    assert xb.shape[:4] == (N, D, H, W) and pc.ks == 3 and pc.cin_pad == Ca + Cb
    if not xa.is_cuda:
        return fused_conv3d(torch.cat([xa, xb], -1), pc, post_relu)
    zt = pc.ztap
    assert xa.dtype == xb.dtype == torch.bfloat16 and xa.is_contiguous() and xb.is_contiguous()
    assert Ca % 8 == 0 and Cb % 8 == 0 and (Ca + Cb) % zt.ck == 0 and pc.cout % 4 == 0
    out = torch.empty(N, D, H, W, pc.cout, device=xa.device, dtype=torch.bfloat16)
    _native.call("be_conv3d_ztaps_concat", _native.ptr(xa), _native.ptr(xb), _native.ptr(zt.wp), _native.ptr(zt.bias),
                 _native.ptr(out), N, D, H, W, Ca, Cb, pc.cout, zt.ck, zt.tco, int(post_relu), 4,
                 _native.stream(xa.device))
    return out


def concat3d_fusible(pc: PackedConv3d, ca: int, cb: int) -> bool:
    """Whether :func:`fused_conv3d_concat` takes this conv over a [ca | cb]-channel concatenation."""
    return (os.environ.get("BE_CONV3D", "ztaps") == "ztaps" and pc.ks == 3 and pc.cout % 4 == 0
            and pc.cin_pad == ca + cb and pc.ztap.cin_pad == 3 * (ca + cb) and (ca + cb) % pc.ztap.ck == 0
            and ca % 8 == 0 and cb % 8 == 0)


def maxpool3d_ndhwc(x: torch.Tensor) -> torch.Tensor:
    """MaxPool3d(2) (floor mode) of NDHWC [N, D, H, W, C] -> [N, D/2, H/2, W/2, C] (``vol3d.hip``)."""
    N, D, H, W, C = x.shape
    if not x.is_cuda:
        y = F.max_pool3d(x.permute(0, 4, 1, 2, 3).float(), 2)
        return y.permute(0, 2, 3, 4, 1).to(x.dtype).contiguous()
    assert x.dtype == torch.bfloat16 and x.is_contiguous() and C % 8 == 0
    out = torch.empty(N, D // 2, H // 2, W // 2, C, device=x.device, dtype=x.dtype)
    _native.call("be_maxpool3d_ndhwc", _native.ptr(x), _native.ptr(out), N, D, H, W, C, _native.stream(x.device))
    return out


def depth2space3d(y: torch.Tensor, cout: int) -> torch.Tensor:
    """[N, D, H, W, 8 cout] (channel (4 dz + 2 dy + dx) * cout + c) -> [N, 2D, 2H, 2W, cout]."""
    N, D, H, W, C8 = y.shape
    assert C8 == 8 * cout
    if not y.is_cuda or cout % 8:
        return (y.view(N, D, H, W, 2, 2, 2, cout).permute(0, 1, 4, 2, 5, 3, 6, 7)
                .reshape(N, 2 * D, 2 * H, 2 * W, cout).contiguous())
    assert y.dtype == torch.bfloat16 and y.is_contiguous()
    out = torch.empty(N, 2 * D, 2 * H, 2 * W, cout, device=y.device, dtype=y.dtype)
    _native.call("be_depth2space3d", _native.ptr(y), _native.ptr(out), N, D, H, W, cout, _native.stream(y.device))
    return out
