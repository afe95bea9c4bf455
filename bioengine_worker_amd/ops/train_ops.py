"""Training ops: fused AdamW over flat buffers, fused Cellpose segmentation loss, affine augmentation.

GPU tensors run the HIP kernels (``csrc/kernels/{adamw,seg_loss,augment}.hip``); CPU tensors run the
PyTorch reference of the same math (oracle for tests).
"""
from __future__ import annotations

import math

import torch

from . import _native


# ------------------------------------------------------------------ AdamW

def adamw_flat_(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, *, lr: float, step: int,
                betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, grad_scale: float = 1.0,
                p_bf16: torch.Tensor | None = None) -> None:
    """In-place AdamW (decoupled weight decay, torch.optim.AdamW semantics) on flat fp32 buffers."""
    b1, b2 = betas
    if p.is_cuda:
        _native.call("be_adamw_flat", _native.ptr(p), _native.ptr(g), _native.ptr(m), _native.ptr(v),
                     _native.ptr(p_bf16), p.numel(), float(lr), float(b1), float(b2), float(eps), float(weight_decay),
                     int(step), float(grad_scale), _native.stream(p.device))
        return
    gg = g * grad_scale
    p.mul_(1 - lr * weight_decay)
    m.mul_(b1).add_(gg, alpha=1 - b1)
    v.mul_(b2).addcmul_(gg, gg, value=1 - b2)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)
    if p_bf16 is not None:
        p_bf16.copy_(p.to(torch.bfloat16))


def sumsq(x: torch.Tensor) -> torch.Tensor:
    if x.is_cuda:
        out = torch.zeros(1, device=x.device, dtype=torch.float32)
        _native.call("be_sumsq", _native.ptr(x), x.numel(), _native.ptr(out), _native.stream(x.device))
        return out[0]
    return (x.float() ** 2).sum()


# ------------------------------------------------------------------ segmentation loss

def seg_loss_ref(y: torch.Tensor, lbl: torch.Tensor) -> torch.Tensor:
    y = y.float()
    veci = 5.0 * lbl[:, 1:3]
    loss = torch.nn.functional.mse_loss(y[:, :2], veci) / 2.0
    loss2 = torch.nn.functional.binary_cross_entropy_with_logits(y[:, 2], (lbl[:, 0] > 0.5).float())
    return loss + loss2


class _SegLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, lbl):
        B, _, H, W = y.shape
        yc = y.contiguous()
        lc = lbl.float().contiguous()
        loss = torch.zeros(1, device=y.device, dtype=torch.float32)
        grad = torch.empty_like(yc)
        _native.call("be_seg_loss", _native.ptr(yc), int(yc.dtype == torch.bfloat16), _native.ptr(lc), B, H * W,
                     _native.ptr(loss), _native.ptr(grad), _native.stream(y.device))
        ctx.save_for_backward(grad)
        return loss[0]

    @staticmethod
    def backward(ctx, go):
        (grad,) = ctx.saved_tensors
        return grad * go.to(grad.dtype), None


def seg_loss_and_grad(y: torch.Tensor, lbl: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """(loss, dLoss/dy) in one fused HIP launch (the autograd-free training engine's loss)."""
    B, _, H, W = y.shape
    yc = y.contiguous()
    lc = lbl.float().contiguous()
    loss = torch.zeros(1, device=y.device, dtype=torch.float32)
    grad = torch.empty_like(yc)
    _native.call("be_seg_loss", _native.ptr(yc), int(yc.dtype == torch.bfloat16), _native.ptr(lc), B, H * W,
                 _native.ptr(loss), _native.ptr(grad), _native.stream(y.device))
    return loss[0], grad


def seg_loss(y: torch.Tensor, lbl: torch.Tensor) -> torch.Tensor:
    """Cellpose ``_loss_fn_seg``: MSE(y[:, :2], 5*lbl[:, 1:3])/2 + BCEWithLogits(y[:, 2], lbl[:, 0] > .5)."""
    if y.is_cuda:
        assert y.shape[1] == 3 and lbl.shape[1] >= 3
        return _SegLoss.apply(y, lbl)
    return seg_loss_ref(y, lbl)


# ------------------------------------------------------------------ augmentation

def random_affine_params(B: int, H: int, W: int, xy=(224, 224), scale_range: float = 1.0, rescale=None,
                         do_flip: bool = True, rotate: bool = True, generator: torch.Generator | None = None):
    """cellpose random_rotate_and_resize parameters -> (aff [B, 8] inverse maps, flip [B], scale [B])."""
    g = generator
    scale_range = max(0.0, min(2.0, float(scale_range)))
    aff = torch.zeros(B, 8)
    flip = torch.zeros(B, dtype=torch.int32)
    scales = torch.zeros(B)
    for n in range(B):
        fl = bool(torch.rand(1, generator=g).item() > 0.5) and do_flip
        theta = float(torch.rand(1, generator=g).item()) * math.pi * 2 if rotate else 0.0
        sc = (1 - scale_range / 2) + scale_range * float(torch.rand(1, generator=g).item())
        if rescale is not None:
            sc *= 1.0 / float(rescale[n])
        dxy = torch.clamp(torch.tensor([W * sc - xy[1], H * sc - xy[0]]), min=0)
        dxy = (torch.rand(2, generator=g) - 0.5) * dxy
        cc = torch.tensor([W / 2.0, H / 2.0])
        cc1 = cc - torch.tensor([W - xy[1], H - xy[0]]) / 2.0 + dxy
        # forward map: dst = cc1 + sc * R(theta) (src - cc);  R columns (cos t, sin t), (-sin t, cos t)
        c, s = math.cos(theta), math.sin(theta)
        Mf = torch.tensor([[sc * c, -sc * s], [sc * s, sc * c]])  # dst - cc1 = Mf @ (src - cc)
        Minv = torch.linalg.inv(Mf)
        t = cc - Minv @ cc1
        aff[n, :6] = torch.tensor([Minv[0, 0], Minv[0, 1], t[0], Minv[1, 0], Minv[1, 1], t[1]])
        aff[n, 6] = math.cos(-theta)
        aff[n, 7] = math.sin(-theta)
        flip[n] = int(fl)
        scales[n] = sc
    return aff, flip, scales


def affine_warp(img: torch.Tensor, lbl: torch.Tensor | None, aff: torch.Tensor, flip: torch.Tensor, oh: int, ow: int):
    """img [B, C, H, W], lbl [B, CL, H, W] (cellprob/instances, flowY, flowX, ...) -> warped crops."""
    B, C, H, W = img.shape
    if img.is_cuda:
        imgc = img.float().contiguous()
        out_img = torch.empty(B, C, oh, ow, device=img.device)
        lc = lbl.float().contiguous() if lbl is not None else None
        CL = lbl.shape[1] if lbl is not None else 0
        out_lbl = torch.empty(B, CL, oh, ow, device=img.device) if lbl is not None else None
        a = aff.to(img.device, torch.float32).contiguous()
        f = flip.to(img.device, torch.int32).contiguous()
        _native.call("be_affine_warp", _native.ptr(imgc), C, _native.ptr(lc), CL, B, H, W, _native.ptr(a), _native.ptr(f),
                     oh, ow, _native.ptr(out_img), _native.ptr(out_lbl), _native.stream(img.device))
        return out_img, out_lbl
    return affine_warp_ref(img, lbl, aff, flip, oh, ow)


def affine_warp_ref(img, lbl, aff, flip, oh, ow):
    B, C, H, W = img.shape
    ys, xs = torch.meshgrid(torch.arange(oh, dtype=torch.float32), torch.arange(ow, dtype=torch.float32), indexing="ij")

    def bil(src, sy, sx):
        y0 = torch.floor(sy)
        x0 = torch.floor(sx)
        wy, wx = sy - y0, sx - x0
        y0, x0 = y0.long(), x0.long()
        out = torch.zeros_like(sy)
        for dy, dx, w in ((0, 0, (1 - wy) * (1 - wx)), (0, 1, (1 - wy) * wx), (1, 0, wy * (1 - wx)), (1, 1, wy * wx)):
            yy, xx = y0 + dy, x0 + dx
            ok = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
            out += torch.where(ok, src[yy.clamp(0, H - 1), xx.clamp(0, W - 1)], torch.zeros_like(sy)) * w
        return out

    oi = torch.zeros(B, C, oh, ow)
    ol = torch.zeros(B, lbl.shape[1], oh, ow) if lbl is not None else None
    for b in range(B):
        A = aff[b]
        sx = A[0] * xs + A[1] * ys + A[2]
        sy = A[3] * xs + A[4] * ys + A[5]
        if int(flip[b]):
            sx = (W - 1) - sx
        for c in range(C):
            oi[b, c] = bil(img[b, c].float(), sy, sx)
        if lbl is not None:
            ny, nx = torch.round(sy).long(), torch.round(sx).long()
            ok = (ny >= 0) & (ny < H) & (nx >= 0) & (nx < W)
            ol[b, 0] = torch.where(ok, lbl[b, 0][ny.clamp(0, H - 1), nx.clamp(0, W - 1)], torch.zeros_like(sy))
            if lbl.shape[1] >= 3:
                v2 = bil(lbl[b, 1].float(), sy, sx)
                v1 = bil(lbl[b, 2].float(), sy, sx)
                if int(flip[b]):
                    v1 = -v1
                cs, sn = A[6], A[7]
                ol[b, 1] = -v1 * sn + v2 * cs
                ol[b, 2] = v1 * cs + v2 * sn
    return oi, ol
