"""Bilinear resize (HIP ``be_resize_bilinear``, ``csrc/kernels/imageproc.hip``) for the Cellpose
diameter rescaling: the image is resized to the model's diameter before the network and the flows
back to the input size after it (reference cellpose ``transforms.resize_image``).
Same convention as ``F.interpolate(mode="bilinear", align_corners=False)``, which is the CPU path."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _native


def resize_bilinear(x: torch.Tensor, size: tuple[int, int]) -> torch.Tensor:
    """x [..., H, W] float -> [..., oh, ow] fp32."""
    oh, ow = int(size[0]), int(size[1])
    if not x.is_cuda:
        lead = x.shape[:-2]
        y = F.interpolate(x.float().reshape(-1, 1, *x.shape[-2:]), size=(oh, ow), mode="bilinear", align_corners=False)
        return y.reshape(*lead, oh, ow)
    xc = x.float().contiguous()
    ih, iw = xc.shape[-2:]
    planes = xc.numel() // (ih * iw) if xc.numel() else 0
    out = torch.empty(*xc.shape[:-2], oh, ow, dtype=torch.float32, device=x.device)
    _native.call("be_resize_bilinear", _native.ptr(xc), _native.ptr(out), planes, ih, iw, oh, ow,
                 _native.stream(x.device))
    return out
