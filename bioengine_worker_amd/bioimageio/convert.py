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
   decomposition onto the same MFMA kernel), activations run ``channels_last_3d`` (NDHWC);
5. ``GroupNorm`` / ``InstanceNorm2d`` (+ ``ReLU``) in front of an eligible conv run in that
   conv's input prologue (:class:`HipNormConv2d`, per-image affine from fp32 statistics);
6. ``ConvTranspose2d(k=2, s=2)`` becomes a 1x1 MFMA conv + depth-to-space
   (:class:`HipConvTranspose2x2`) and ``Conv2d(k=2, s=2)`` space-to-depth + a 1x1 MFMA conv
   (:class:`HipConvStride2x2`); in 3-D, ``ConvTranspose3d(k=2, s=2)`` becomes a 1x1x1 MFMA conv to
   8*Cout + the ``vol3d.hip`` depth-to-space scatter (:class:`HipConvTranspose3x2`) and
   ``MaxPool3d(2)`` the ``vol3d.hip`` NDHWC pooling kernel (:class:`HipMaxPool3d`), so a 3-D U-Net
   runs no library convolution;
7. 2-D models run their forward under a deferred-fusion scope (:class:`DeferredFusion`): a
   ``torch.cat`` along channels of two channels-last bf16 tensors and a ``MaxPool2d(2)``
   (:class:`HipMaxPool2d`) return an unfilled placeholder, and the :class:`HipConv2d` that consumes
   it reads the sources directly (``be_conv2d_concat`` / the 2x2 max-pool halo loader), so the U-Net
   decoder's skip concatenation and the encoder's pooling never make a copy.  Any other consumer of
   a placeholder sees it filled first (the scope intercepts every torch call while it is pending),
   so the rewrite cannot change a model's results.  ``BE_UNET_LAZY=0`` turns it off.

TorchScript-only weights go through :mod:`.ts_convert` (frozen graph rewrite).  Convolutions that
do not match (3x3 strided, dilated, grouped, 5x5, ...) stay on MIOpen.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

import collections
import os
import threading
import weakref

from torch.overrides import TorchFunctionMode

from ..ops.conv import PackedConv, depth_to_space2, fused_conv2d, fused_conv2d_concat
from ..ops.conv3d import (PackedConv3d, concat3d_fusible, depth2space3d, fused_conv3d, fused_conv3d_concat,
                          maxpool3d_ndhwc)


def _eligible(c: nn.Module) -> bool:
    return (isinstance(c, nn.Conv2d) and type(c) is nn.Conv2d and c.kernel_size in ((1, 1), (3, 3))
            and c.stride == (1, 1) and c.dilation == (1, 1) and c.groups == 1 and c.padding_mode == "zeros"
            and c.padding == ((c.kernel_size[0] // 2, c.kernel_size[1] // 2)))


def _eligible3d(c: nn.Module) -> bool:
    # 3x3x3 needs Cout % 4 (implicit-GEMM tiles); a 1x1x1 with a ragged Cout (a segmentation head)
    # runs the 2-D kernel's fp32 NCHW-output epilogue instead
    return (type(c) is nn.Conv3d and c.kernel_size in ((1, 1, 1), (3, 3, 3)) and c.stride == (1, 1, 1)
            and c.dilation == (1, 1, 1) and c.groups == 1 and c.padding_mode == "zeros"
            and c.padding == tuple(k // 2 for k in c.kernel_size)
            and (c.out_channels % 4 == 0 or c.kernel_size == (1, 1, 1)))


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
        # first, before ANY tensor access (which would make the scope fill a placeholder): is x a
        # deferred cat / max-pool this conv can read from its sources?
        scope = getattr(_tls, "scope", None)
        if scope is not None and scope.pending and not self.nchw_out:
            ent = scope.take(x, self._fusible)
            if ent is not None:
                src = ent[2]
                if src.is_cuda and self._dev != src.device:
                    self.pc.to(src.device)
                    self._dev = src.device
                if ent[1] == "cat_d2s":  # the up-conv's sub-pixel output, read before its shuffle
                    y = fused_conv2d_concat(ent[2].permute(0, 2, 3, 1), ent[3], self.pc, post_relu=self.post_relu,
                                            xb_d2s=True)
                elif ent[1] == "cat":
                    y = fused_conv2d_concat(ent[2].permute(0, 2, 3, 1), ent[3].permute(0, 2, 3, 1), self.pc,
                                            post_relu=self.post_relu)
                else:
                    y = fused_conv2d(src.permute(0, 2, 3, 1), self.pc, inmode="pool2", post_relu=self.post_relu)
                return y.permute(0, 3, 1, 2)
        if not x.is_cuda:  # CPU: reference math (bf16-rounded like the kernel)
            y = F.conv2d(x.float(), self.pc.w.to(x.device), None if self.pc.bias is None else self.pc.bias.to(x.device),
                         padding=self.pc.ks // 2)
            y = torch.relu(y) if self.post_relu else y
            y = y.to(x.dtype)
            # the GPU path's layout, for the deferral tests (a scope exists on CPU only with ALLOW_CPU)
            return y.contiguous(memory_format=torch.channels_last) if scope is not None else y
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

    def _fusible(self, ent: tuple) -> bool:
        if ent[1] == "cat":
            return self.pc.ks == 3 and self.pc.cin_pad == ent[2].shape[1] + ent[3].shape[1]
        if ent[1] == "cat_d2s":
            return self.pc.ks == 3 and self.pc.cin_pad == ent[2].shape[1] + ent[4]
        if ent[1] == "pool":
            return self.pc.cin_pad == ent[2].shape[1]  # any kernel size: the loader pools 2x2
        return False

    def extra_repr(self) -> str:
        return f"{self.cin}, {self.cout}, k={self.pc.ks}, post_relu={self.post_relu}"


# ---- deferred cat / max-pool fusion (item 7 of the module docstring) ------------------------------
_tls = threading.local()
#: BE_UNET_LAZY=0: no deferred fusion (A/B)
LAZY = os.environ.get("BE_UNET_LAZY", "1") != "0"


# tensor metadata reads: they never need a placeholder's data, so they do not fill it
_META = {torch.Tensor.shape.__get__, torch.Tensor.dtype.__get__, torch.Tensor.device.__get__,
         torch.Tensor.is_cuda.__get__, torch.Tensor.requires_grad.__get__, torch.Tensor.ndim.__get__,
         torch.Tensor.layout.__get__, torch.Tensor.dim, torch.Tensor.size, torch.Tensor.stride,
         torch.Tensor.is_contiguous, torch.Tensor.numel}


def _nhwc_dense(t: torch.Tensor) -> bool:
    """Channels-last dense (an NHWC / NDHWC buffer viewed as NCHW / NCDHW)."""
    if t.dim() == 4:
        return t.permute(0, 2, 3, 1).is_contiguous()
    return t.dim() == 5 and t.permute(0, 2, 3, 4, 1).is_contiguous()


class DeferredFusion(TorchFunctionMode):
    """Scope of one model forward.  ``torch.cat([a, b], dim=1)`` of two channels-last bf16 tensors
    (channels % 8 == 0) and :class:`HipMaxPool2d` return an unfilled channels-last placeholder and
    record its sources; a :class:`HipConv2d` that receives a placeholder reads the sources itself.
    The placeholder stays pending (held weakly): any other torch call that touches it fills it
    first, an in-place write to one of its sources fills it before the write, and leaving the scope
    fills every placeholder still alive (returned, or kept by the model).  The mode sees every torch
    function call made while it is active, so results are those of the eager model; a placeholder
    that only a HIP conv ever read is freed unfilled -- the copy that is saved.  Nothing is deferred
    when a source requires grad."""

    #: tests only: defer on CPU tensors too (the consumers then run their reference math)
    ALLOW_CPU = False

    def __init__(self):
        super().__init__()
        self.pending: dict[int, tuple] = {}  # id(placeholder) -> (weakref(placeholder), kind, *sources)
        self.deferred = 0
        self.filled = 0
        self.filled_kinds: collections.Counter = collections.Counter()

    def _ok_src(self, t: torch.Tensor) -> bool:
        return ((t.is_cuda or self.ALLOW_CPU) and t.dtype == torch.bfloat16 and not t.requires_grad
                and _nhwc_dense(t) and not self._is_pending(t))

    def _is_pending(self, t) -> bool:
        ent = self.pending.get(id(t))
        return ent is not None and ent[0]() is t

    def _kind(self, t) -> str | None:
        ent = self.pending.get(id(t))
        return ent[1] if ent is not None and ent[0]() is t else None

    def source_d2s(self, t) -> tuple | None:
        """(y, c) if ``t`` is a pending 2x2 depth-to-space placeholder of y [N, H, W, 4c]."""
        ent = self.pending.get(id(t))
        return ent[2:] if ent is not None and ent[0]() is t and ent[1] == "d2s" else None

    def defer_d2s(self, y: torch.Tensor, c: int) -> torch.Tensor | None:
        """Placeholder for the depth-to-space of y [N, H, W, 4c] (NHWC bf16), [N, c, 2H, 2W] channels-last."""
        if not ((y.is_cuda or self.ALLOW_CPU) and y.dtype == torch.bfloat16 and y.is_contiguous()
                and not y.requires_grad and c % 8 == 0):
            return None
        N, H, W, _ = y.shape
        ph = torch.empty((N, c, 2 * H, 2 * W), dtype=y.dtype, device=y.device, memory_format=torch.channels_last)
        return self._add(ph, "d2s", y, c)

    def _add(self, ph: torch.Tensor, kind: str, *srcs) -> torch.Tensor:
        self.pending[id(ph)] = (weakref.ref(ph), kind, *srcs)
        self.deferred += 1
        return ph

    def defer_pool(self, x: torch.Tensor) -> torch.Tensor | None:
        if not (x.dim() == 4 and self._ok_src(x) and x.shape[2] >= 2 and x.shape[3] >= 2):
            return None
        N, C, H, W = x.shape
        ph = torch.empty((N, C, H // 2, W // 2), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        return self._add(ph, "pool", x)

    def _defer_cat(self, args, kwargs) -> torch.Tensor | None:
        if "out" in kwargs or not args:
            return None
        ts = args[0]
        dim = args[1] if len(args) > 1 else kwargs.get("dim", 0)
        if not isinstance(ts, (list, tuple)) or len(ts) != 2 or dim not in (1, -3, -4):
            return None
        a, b = ts
        if not (isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor) and a.dim() == b.dim()
                and a.dim() in (4, 5) and dim in (1, 1 - a.dim())):
            return None
        b_ok = self._ok_src(b) or (a.dim() == 4 and self._kind(b) == "d2s")
        if not (self._ok_src(a) and b_ok and a.device == b.device and a.shape[0] == b.shape[0]
                and a.shape[2:] == b.shape[2:] and a.shape[1] % 8 == 0 and b.shape[1] % 8 == 0):
            return None
        shape = (a.shape[0], a.shape[1] + b.shape[1]) + tuple(a.shape[2:])
        fmt = torch.channels_last if a.dim() == 4 else torch.channels_last_3d
        ph = torch.empty(shape, dtype=a.dtype, device=a.device, memory_format=fmt)
        d2s = self.source_d2s(b)
        if d2s is not None:  # hold the up-conv's sub-pixel output, not its (unfilled) placeholder
            return self._add(ph, "cat_d2s", a, d2s[0], d2s[1])
        return self._add(ph, "cat", a, b)

    def take(self, x: torch.Tensor, fusible) -> tuple | None:
        """(placeholder, kind, *sources) if ``x`` is a pending placeholder and ``fusible`` accepts it.
        The entry stays pending: the placeholder is filled if anything else touches it later."""
        ent = self.pending.get(id(x))
        if ent is None or ent[0]() is not x:
            return None
        ent = (x,) + ent[1:]
        return ent if fusible(ent) else None

    def _fill_key(self, key: int) -> None:
        wr, kind, *srcs = self.pending.pop(key)
        ph = wr()
        if ph is None:
            return
        if kind == "cat":
            torch.cat(srcs, dim=1, out=ph)
        elif kind == "cat_d2s":
            torch.cat([srcs[0], depth_to_space2(srcs[1], srcs[2]).permute(0, 3, 1, 2)], dim=1, out=ph)
        elif kind == "d2s":
            ph.permute(0, 2, 3, 1).copy_(depth_to_space2(srcs[0], srcs[1]))
        else:
            ph.copy_(F.max_pool2d(srcs[0], 2))
        self.filled += 1
        self.filled_kinds[kind] += 1

    def _fill_in(self, obj) -> None:
        if isinstance(obj, torch.Tensor):
            if self._is_pending(obj):
                self._fill_key(id(obj))
        elif isinstance(obj, (list, tuple)):
            for o in obj:
                self._fill_in(o)
        elif isinstance(obj, dict):
            for o in obj.values():
                self._fill_in(o)

    @staticmethod
    def _written(func, args, kwargs) -> list:
        name = getattr(func, "__name__", "")
        out = []
        if args and isinstance(args[0], torch.Tensor) and (
                (name.endswith("_") and not name.endswith("__")) or name == "__setitem__"
                or (name.startswith("__i") and name.endswith("__"))):
            out.append(args[0])
        o = kwargs.get("out")
        if isinstance(o, torch.Tensor):
            out.append(o)
        elif isinstance(o, (list, tuple)):
            out.extend(t for t in o if isinstance(t, torch.Tensor))
        return out

    def _fill_readers_of(self, written: list) -> None:
        """Fill every pending placeholder with a source in the storage ``written`` is about to change."""
        ptrs = {t.untyped_storage().data_ptr() for t in written}
        for key, ent in list(self.pending.items()):
            if key in self.pending and any(isinstance(s, torch.Tensor) and s.untyped_storage().data_ptr() in ptrs
                                           for s in ent[2:]):
                self._fill_key(key)

    def flush(self) -> None:
        # newest first: a consumer entry (a cat) holds its deferred sources; dropping it first lets a
        # source that nothing else kept die unfilled
        for key in reversed(list(self.pending)):
            if key in self.pending:
                self._fill_key(key)

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func is torch.cat:
            ph = self._defer_cat(args, kwargs)
            if ph is not None:
                return ph
        if self.pending and func not in _META:
            self._fill_in(args)
            self._fill_in(kwargs)
            written = self._written(func, args, kwargs)
            if written and self.pending:
                self._fill_readers_of(written)
        return func(*args, **kwargs)


class HipMaxPool2d(nn.Module):
    """``MaxPool2d(2)``: inside a :class:`DeferredFusion` scope a placeholder the next HIP conv pools
    in its halo loader (inmode ``pool2``); elsewhere ``F.max_pool2d``."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        scope = getattr(_tls, "scope", None)
        if scope is not None:
            ph = scope.defer_pool(x)
            if ph is not None:
                return ph
        return F.max_pool2d(x, 2)


def _mp2_ok(m) -> bool:
    two = lambda v: v == 2 or v == (2, 2)  # noqa: E731
    return (type(m) is nn.MaxPool2d and two(m.kernel_size) and two(m.stride if m.stride is not None else 2)
            and m.padding in (0, (0, 0)) and m.dilation in (1, (1, 1)) and not m.ceil_mode
            and not m.return_indices)


def _install_deferred_fusion(model: nn.Module) -> None:
    orig = model.forward

    def forward(*args, **kwargs):
        x = args[0] if args else None
        if not (isinstance(x, torch.Tensor) and (x.is_cuda or DeferredFusion.ALLOW_CPU)) or not LAZY:
            return orig(*args, **kwargs)
        prev = getattr(_tls, "scope", None)
        scope = DeferredFusion()
        _tls.scope = scope
        try:
            with scope:
                out = orig(*args, **kwargs)
                scope.flush()
        finally:
            _tls.scope = prev
        model._be_fusion_stats = (scope.deferred, scope.filled)
        model._be_fusion_filled = dict(scope.filled_kinds)
        return out

    model.forward = forward


class HipConv3d(nn.Module):
    """Conv3d (+ folded BN)(+ ReLU) on the fused NHWC MFMA conv kernel (depth-tap decomposition)."""

    def __init__(self, conv: nn.Conv3d, post_relu: bool = False):
        super().__init__()
        self.cin, self.cout = conv.in_channels, conv.out_channels
        self.post_relu = post_relu
        self.nchw_out = self.cout % 4 != 0  # 1x1x1 head: fp32 NCDHW straight from the epilogue
        self.pc = PackedConv3d(conv.weight.detach().float(), None if conv.bias is None else conv.bias.detach().float(),
                               cout_pad_to=16 if self.nchw_out else None)
        self._dev = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        scope = getattr(_tls, "scope", None)  # a deferred cat: checked before any tensor access (see HipConv2d)
        if scope is not None and scope.pending and not self.nchw_out:
            ent = scope.take(x, lambda e: e[1] == "cat" and concat3d_fusible(self.pc, e[2].shape[1], e[3].shape[1]))
            if ent is not None:
                a, b = (t.permute(0, 2, 3, 4, 1) for t in ent[2:])
                if a.is_cuda and self._dev != a.device:
                    self.pc.to(a.device)
                    self._dev = a.device
                return fused_conv3d_concat(a, b, self.pc, post_relu=self.post_relu).permute(0, 4, 1, 2, 3)
        if not x.is_cuda:  # CPU: fp32 reference math in the input dtype
            y = F.conv3d(x.float(), self.pc.w.to(x.device),
                         None if self.pc.bias is None else self.pc.bias.to(x.device), padding=self.pc.ks // 2)
            y = torch.relu(y) if self.post_relu else y
            y = y.to(x.dtype)
            return y.contiguous(memory_format=torch.channels_last_3d) if scope is not None else y
        if self._dev != x.device:
            self.pc.to(x.device)
            self._dev = x.device
        N, C, D, H, W = x.shape
        xh = x.to(torch.bfloat16).permute(0, 2, 3, 4, 1)  # NDHWC (a view for channels_last_3d inputs)
        if C != self.pc.cin_pad:
            xh = F.pad(xh, (0, self.pc.cin_pad - C))
        if self.nchw_out:  # [N*D, Cout, H, W] fp32 -> NCDHW view
            y = fused_conv2d(xh.contiguous().view(N * D, H, W, self.pc.cin_pad), self.pc.taps[0], out_nchw_f32=True,
                             cout_valid=self.cout, post_relu=self.post_relu)
            return y.view(N, D, self.cout, H, W).permute(0, 2, 1, 3, 4)
        y = fused_conv3d(xh.contiguous(), self.pc, post_relu=self.post_relu)  # [N, D, H, W, Cout]
        return y.permute(0, 4, 1, 2, 3)  # channels_last_3d view, no copy

    def extra_repr(self) -> str:
        return f"{self.cin}, {self.cout}, k={self.pc.ks}, post_relu={self.post_relu}"


def _group_affine(yh: torch.Tensor, groups: int, weight, bias, eps: float):
    """Per-image, per-channel (scale, shift) [N, C] that apply GroupNorm to the NHWC tensor ``yh``
    (statistics in fp32): what the next conv's prologue consumes instead of a normalised copy."""
    N, H, W, C = yh.shape
    var, mean = torch.var_mean(yh.float().view(N, H * W, groups, C // groups), dim=(1, 3), unbiased=False)
    rstd = torch.rsqrt(var + eps)  # [N, G]
    rstd_c = rstd.repeat_interleave(C // groups, dim=1)
    mean_c = mean.repeat_interleave(C // groups, dim=1)
    g = weight.float().view(1, C) if weight is not None else torch.ones(1, C, device=yh.device)
    b = bias.float().view(1, C) if bias is not None else torch.zeros(1, C, device=yh.device)
    scale = (rstd_c * g).contiguous()
    return scale, (b - mean_c * scale).contiguous()


def _norm_params(norm: nn.Module):
    if isinstance(norm, nn.GroupNorm):
        return norm.num_groups, norm.weight, norm.bias, norm.eps
    return norm.num_features, norm.weight, norm.bias, norm.eps  # InstanceNorm2d: one group per channel


def _instance_norm_ok(m: nn.Module) -> bool:
    return isinstance(m, nn.InstanceNorm2d) and not m.track_running_stats


class HipNormConv2d(nn.Module):
    """GroupNorm / InstanceNorm (+ ReLU) of the incoming activation fused into the PROLOGUE of the
    following conv: the statistics are reduced from the producer's NHWC output and the per-image
    affine + ReLU are applied while the conv stages its input tiles in LDS (the same per-image
    prologue the GroupNorm training engine uses), so the normalised tensor never exists."""

    def __init__(self, norm: nn.Module, relu: bool, conv: nn.Conv2d, post_relu: bool = False):
        super().__init__()
        self.groups, w, b, self.eps = _norm_params(norm)
        self.register_buffer("gn_weight", None if w is None else w.detach().float().clone())
        self.register_buffer("gn_bias", None if b is None else b.detach().float().clone())
        self.relu = relu
        self.conv = HipConv2d(conv, post_relu)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not x.is_cuda:
            w = None if self.gn_weight is None else self.gn_weight.to(x.device).float()
            b = None if self.gn_bias is None else self.gn_bias.to(x.device).float()
            h = F.group_norm(x.float(), self.groups, w, b, self.eps)
            return self.conv((torch.relu(h) if self.relu else h).to(x.dtype))
        hc = self.conv
        if hc._dev != x.device:
            hc.pc.to(x.device)
            hc._dev = x.device
        N, C, H, W = x.shape
        xh = x.to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()
        scale, shift = _group_affine(xh, self.groups, self.gn_weight, self.gn_bias, self.eps)
        if C != hc.pc.cin_pad:
            xh = F.pad(xh, (0, hc.pc.cin_pad - C))
            scale = F.pad(scale, (0, hc.pc.cin_pad - C))
            shift = F.pad(shift, (0, hc.pc.cin_pad - C))
        if hc.nchw_out:
            return fused_conv2d(xh, hc.pc, scale=scale, shift=shift, relu=self.relu, out_nchw_f32=True,
                                cout_valid=hc.cout, post_relu=hc.post_relu)
        y = fused_conv2d(xh, hc.pc, scale=scale, shift=shift, relu=self.relu, post_relu=hc.post_relu)
        return y.permute(0, 3, 1, 2)


class HipConvTranspose2x2(nn.Module):
    """ConvTranspose2d(k=2, stride=2) as a 1x1 MFMA conv to 4*Cout channels (one per output
    sub-pixel) followed by a depth-to-space shuffle: each output pixel (2y+dy, 2x+dx) is
    W[:, :, dy, dx]^T x[y, x] + b."""

    def __init__(self, ct: nn.ConvTranspose2d):
        super().__init__()
        w = ct.weight.detach().float()  # [Cin, Cout, 2, 2]
        self.cin, self.cout = w.shape[0], w.shape[1]
        w1 = w.permute(2, 3, 1, 0).reshape(4 * self.cout, self.cin, 1, 1)  # row (dy*2+dx)*Cout + co
        b1 = None if ct.bias is None else ct.bias.detach().float().repeat(4)
        self.ref = ct
        self.pc = PackedConv.from_weight(w1, b1)
        self._dev = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        scope = getattr(_tls, "scope", None)  # (on CPU only in tests: DeferredFusion.ALLOW_CPU)
        if not x.is_cuda and scope is None:
            return self.ref.to(x.device).float()(x.float()).to(x.dtype)
        if self._dev != x.device:
            self.pc.to(x.device)
            self._dev = x.device
        N, C, H, W = x.shape
        xh = x.to(torch.bfloat16).permute(0, 2, 3, 1)
        if C != self.pc.cin_pad:
            xh = F.pad(xh, (0, self.pc.cin_pad - C))
        y = fused_conv2d(xh.contiguous(), self.pc)  # [N, H, W, 4*Cout]
        if scope is not None:  # a decoder concatenation can read the sub-pixel layout in place
            ph = scope.defer_d2s(y, self.cout)
            if ph is not None:
                return ph
        return depth_to_space2(y, self.cout).permute(0, 3, 1, 2)

    def extra_repr(self) -> str:
        return f"{self.cin}, {self.cout}, k=2, s=2 (1x1 MFMA + depth-to-space)"


class HipConvTranspose3x2(nn.Module):
    """ConvTranspose3d(k=2, stride=2) as a 1x1x1 MFMA conv to 8*Cout channels (one per output
    sub-voxel) followed by the depth-to-space scatter of ``vol3d.hip``: each output voxel
    (2z+dz, 2y+dy, 2x+dx) is W[:, :, dz, dy, dx]^T x[z, y, x] + b."""

    def __init__(self, ct: nn.ConvTranspose3d):
        super().__init__()
        w = ct.weight.detach().float()  # [Cin, Cout, 2, 2, 2]
        self.cin, self.cout = w.shape[0], w.shape[1]
        w1 = w.permute(2, 3, 4, 1, 0).reshape(8 * self.cout, self.cin, 1, 1)  # row (4dz+2dy+dx)*Cout + co
        b1 = None if ct.bias is None else ct.bias.detach().float().repeat(8)
        self.__dict__["ref"] = ct  # CPU oracle only: not a registered submodule (no library op in the tree)
        self.pc = PackedConv.from_weight(w1, b1)
        self._dev = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not x.is_cuda:
            return self.ref.to(x.device).float()(x.float()).to(x.dtype)
        if self._dev != x.device:
            self.pc.to(x.device)
            self._dev = x.device
        N, C, D, H, W = x.shape
        xh = x.to(torch.bfloat16).permute(0, 2, 3, 4, 1)
        if C != self.pc.cin_pad:
            xh = F.pad(xh, (0, self.pc.cin_pad - C))
        y = fused_conv2d(xh.contiguous().view(N * D, H, W, self.pc.cin_pad), self.pc)  # [N*D, H, W, 8*Cout]
        out = depth2space3d(y.view(N, D, H, W, 8 * self.cout), self.cout)  # [N, 2D, 2H, 2W, Cout]
        return out.permute(0, 4, 1, 2, 3)

    def extra_repr(self) -> str:
        return f"{self.cin}, {self.cout}, k=2, s=2 (1x1x1 MFMA + depth-to-space)"


class HipMaxPool3d(nn.Module):
    """MaxPool3d(2) on NDHWC bf16 (``vol3d.hip``): one 16-byte load per 8 channels per window voxel."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not x.is_cuda or x.shape[1] % 8:
            return F.max_pool3d(x, 2)
        y = maxpool3d_ndhwc(x.to(torch.bfloat16).permute(0, 2, 3, 4, 1).contiguous())
        return y.permute(0, 4, 1, 2, 3)


def _ct3_ok(m) -> bool:
    return (type(m) is nn.ConvTranspose3d and m.kernel_size == (2, 2, 2) and m.stride == (2, 2, 2)
            and m.padding == (0, 0, 0) and m.output_padding == (0, 0, 0) and m.dilation == (1, 1, 1)
            and m.groups == 1)


def _mp3_ok(m) -> bool:
    def two(v):
        return v in (2, (2, 2, 2))

    return (type(m) is nn.MaxPool3d and two(m.kernel_size) and two(m.stride if m.stride is not None else 2)
            and m.padding in (0, (0, 0, 0)) and m.dilation in (1, (1, 1, 1)) and not m.ceil_mode
            and not m.return_indices)


class HipConvStride2x2(nn.Module):
    """Conv2d(k=2, stride=2) (strided-conv downsampling) as space-to-depth + a 1x1 MFMA conv over
    4*Cin channels: out[y, x] = sum_{dy,dx} W[:, :, dy, dx] x[2y+dy, 2x+dx]."""

    def __init__(self, conv: nn.Conv2d, post_relu: bool = False):
        super().__init__()
        w = conv.weight.detach().float()  # [Cout, Cin, 2, 2]
        self.cin, self.cout = w.shape[1], w.shape[0]
        w1 = w.permute(0, 2, 3, 1).reshape(self.cout, 4 * self.cin, 1, 1)  # col (dy*2+dx)*Cin + ci
        self.post_relu = post_relu
        self.ref = conv
        self.nchw_out = self.cout % 4 != 0
        self.pc = PackedConv.from_weight(w1, None if conv.bias is None else conv.bias.detach().float(),
                                         cout_pad_to=16 if self.nchw_out else None)
        self._dev = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not x.is_cuda:
            y = self.ref.to(x.device).float()(x.float())
            return (torch.relu(y) if self.post_relu else y).to(x.dtype)
        if self._dev != x.device:
            self.pc.to(x.device)
            self._dev = x.device
        N, C, H, W = x.shape
        xh = x.to(torch.bfloat16).permute(0, 2, 3, 1)[:, : H // 2 * 2, : W // 2 * 2]
        xs = xh.reshape(N, H // 2, 2, W // 2, 2, C).permute(0, 1, 3, 2, 4, 5).reshape(N, H // 2, W // 2, 4 * C)
        if 4 * C != self.pc.cin_pad:
            xs = F.pad(xs, (0, self.pc.cin_pad - 4 * C))
        xs = xs.contiguous()
        if self.nchw_out:
            return fused_conv2d(xs, self.pc, out_nchw_f32=True, cout_valid=self.cout, post_relu=self.post_relu)
        return fused_conv2d(xs, self.pc, post_relu=self.post_relu).permute(0, 3, 1, 2)


def _ct2x2_ok(m) -> bool:
    return (type(m) is nn.ConvTranspose2d and m.kernel_size == (2, 2) and m.stride == (2, 2) and m.padding == (0, 0)
            and m.output_padding == (0, 0) and m.dilation == (1, 1) and m.groups == 1)


def _s2_ok(m) -> bool:
    return (type(m) is nn.Conv2d and m.kernel_size == (2, 2) and m.stride == (2, 2) and m.padding == (0, 0)
            and m.dilation == (1, 1) and m.groups == 1)


def _hip_conv(conv, post_relu: bool = False):
    return HipConv3d(conv, post_relu) if isinstance(conv, nn.Conv3d) else HipConv2d(conv, post_relu)


def _ok(conv) -> bool:
    return _eligible3d(conv) if isinstance(conv, nn.Conv3d) else _eligible(conv)


def _is_norm(m) -> bool:
    return isinstance(m, nn.GroupNorm) or _instance_norm_ok(m)


def _rewrite(mod: nn.Module, stats: dict) -> None:
    for name, child in list(mod.named_children()):
        if isinstance(child, nn.Sequential):
            items = list(child._modules.items())
            i = 0
            while i < len(items):
                k, m = items[i]
                # [GroupNorm|InstanceNorm, (ReLU), Conv] -> the norm runs in the conv's prologue
                if _is_norm(m):
                    j = i + 1
                    relu = j < len(items) and isinstance(items[j][1], nn.ReLU)
                    j += 1 if relu else 0
                    nxt = items[j][1] if j < len(items) else None
                    if type(nxt) is nn.Conv2d and _eligible(nxt):
                        post = j + 1 < len(items) and isinstance(items[j + 1][1], nn.ReLU)
                        child._modules[k] = HipNormConv2d(m, relu, nxt, post_relu=post)
                        if relu:
                            child._modules[items[i + 1][0]] = nn.Identity()
                        child._modules[items[j][0]] = nn.Identity()
                        if post:
                            child._modules[items[j + 1][0]] = nn.Identity()
                            stats["relu_fused"] += 1
                        stats["norm_fused"] += 1
                        stats["convs"] += 1
                        i = j + 1 + (1 if post else 0)
                        continue
                    stats["norm_unfused"] += 1
                    i += 1
                    continue
                if _ct2x2_ok(m):
                    child._modules[k] = HipConvTranspose2x2(m)
                    stats["conv_transpose"] += 1
                    i += 1
                    continue
                if _ct3_ok(m):
                    child._modules[k] = HipConvTranspose3x2(m)
                    stats["conv_transpose"] += 1
                    i += 1
                    continue
                if _mp3_ok(m):
                    child._modules[k] = HipMaxPool3d()
                    stats["pool3d"] += 1
                    i += 1
                    continue
                if _mp2_ok(m):
                    child._modules[k] = HipMaxPool2d()
                    stats["pool2d"] += 1
                    i += 1
                    continue
                if _s2_ok(m):
                    relu = i + 1 < len(items) and isinstance(items[i + 1][1], nn.ReLU)
                    child._modules[k] = HipConvStride2x2(m, post_relu=relu)
                    if relu:
                        child._modules[items[i + 1][0]] = nn.Identity()
                    stats["strided"] += 1
                    i += 2 if relu else 1
                    continue
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
        elif _ct2x2_ok(child):
            setattr(mod, name, HipConvTranspose2x2(child))
            stats["conv_transpose"] += 1
        elif _ct3_ok(child):
            setattr(mod, name, HipConvTranspose3x2(child))
            stats["conv_transpose"] += 1
        elif _mp3_ok(child):
            setattr(mod, name, HipMaxPool3d())
            stats["pool3d"] += 1
        elif _mp2_ok(child):
            setattr(mod, name, HipMaxPool2d())
            stats["pool2d"] += 1
        elif _s2_ok(child):
            setattr(mod, name, HipConvStride2x2(child))
            stats["strided"] += 1
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
    stats = {"convs": 0, "bn_folded": 0, "relu_fused": 0, "skipped": 0, "norm_fused": 0, "norm_unfused": 0,
             "conv_transpose": 0, "strided": 0, "pool3d": 0, "pool2d": 0}
    _rewrite(model, stats)
    if any(isinstance(m, (HipConv2d, HipConv3d)) for m in model.modules()):
        _install_deferred_fusion(model)
    if device is not None:
        model.to(device)
    model.to(torch.bfloat16)
    return model, stats
