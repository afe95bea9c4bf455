"""ONNX graph executor on PyTorch-ROCm with the MI355X conv fusions (model-runner
weights format "onnx").

The reference hands ONNX weights to onnxruntime (``/root/reference/apps/model-runner/
runtime_deployment.py:22``; format selection ``entry_deployment.py:1884-1887``).  Here the graph from
:mod:`.onnx_proto` is compiled once into a flat list of steps (one closure per node, attributes
resolved up front) and run eagerly: shape arithmetic (Shape / Gather / Concat / Reshape chains) stays
in CPU int64 tensors so it never syncs the GPU, float initializers are module buffers (so ``.to`` moves
and casts them), and with ``optimize=True`` the same fusions as :mod:`.convert` are applied on the
dataflow graph instead of on ``nn.Sequential`` order:

* Conv -> BatchNormalization (constant statistics) folded, -> Relu absorbed into the epilogue, onto
  the fused NHWC MFMA conv (1x1 / 3x3 "same", stride 1; 3-D 1x1x1 / 3x3x3);
* InstanceNormalization / GroupNormalization (-> Relu) -> Conv: statistics + affine in the conv's
  prologue (:class:`.convert.HipNormConv2d`);
* ConvTranspose(k=2, s=2) as 1x1 MFMA + depth-to-space; Conv(k=2, s=2) as space-to-depth + 1x1.

A fused link is only taken when the intermediate tensor has exactly one consumer and is not a
graph output.  Everything else runs as the equivalent torch op.
"""
from __future__ import annotations

import math
from pathlib import Path

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import onnx_proto as P

# operands from this input index on are shape/scale data: kept as CPU fp32/int64, never cast or moved
_META_FROM = {"Resize": 1, "Upsample": 1, "Clip": 1, "Pad": 1, "Range": 0, "ConstantOfShape": 0, "Reshape": 1,
              "Slice": 1, "Expand": 1, "Tile": 1, "Squeeze": 1, "Unsqueeze": 1, "Split": 1, "TopK": 1}
_INT_DT = (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool)


def _ints(v) -> list[int]:
    if v is None:
        return []
    if torch.is_tensor(v):
        return [int(x) for x in v.reshape(-1).tolist()]
    return [int(x) for x in v]


def _scalar(v):
    return None if v is None else (v.reshape(-1)[0].item() if torch.is_tensor(v) else v)


def _on(a: torch.Tensor, ref: torch.Tensor) -> torch.Tensor:
    return a if a.device == ref.device else a.to(ref.device)


def _bin(fn):
    def f(a, b):
        if a.device != b.device:  # CPU shape/int constants meeting device activations
            if a.dim() == 0 or a.device.type == "cpu":
                a = a.to(b.device)
            else:
                b = b.to(a.device)
        return [fn(a, b)]
    return f


def _div(a, b):
    if a.dtype in _INT_DT and b.dtype in _INT_DT:
        return torch.div(a, b, rounding_mode="trunc")
    return a / b


def _pad_cfg(pads: list[int], nd: int) -> list[int]:
    """ONNX [b1..bn, e1..en] over the last ``nd`` dims -> F.pad order (last dim first)."""
    cfg = []
    for i in reversed(range(nd)):
        cfg += [pads[i], pads[i + nd]]
    return cfg


def _same_pads(shape, k, s, d, mode) -> list[int]:
    nd = len(k)
    b, e = [0] * nd, [0] * nd
    for i in range(nd):
        L = shape[i]
        tot = max(0, (math.ceil(L / s[i]) - 1) * s[i] + (k[i] - 1) * d[i] + 1 - L)
        lo = tot // 2 if mode == "SAME_UPPER" else tot - tot // 2
        b[i], e[i] = lo, tot - lo
    return b + e


def _conv_geom(a, w_shape, x_shape=None):
    nd = len(w_shape) - 2
    k = list(a.get("kernel_shape") or w_shape[2:])
    s = list(a.get("strides") or [1] * nd)
    d = list(a.get("dilations") or [1] * nd)
    auto = a.get("auto_pad", "NOTSET")
    if auto in ("SAME_UPPER", "SAME_LOWER"):
        pads = _same_pads(x_shape[2:], k, s, d, auto) if x_shape is not None else None
    elif auto == "VALID":
        pads = [0] * (2 * nd)
    else:
        pads = list(a.get("pads") or [0] * (2 * nd))
    return nd, k, s, d, pads


_CONV = {1: F.conv1d, 2: F.conv2d, 3: F.conv3d}
_CONVT = {1: F.conv_transpose1d, 2: F.conv_transpose2d, 3: F.conv_transpose3d}
_MAXP = {1: F.max_pool1d, 2: F.max_pool2d, 3: F.max_pool3d}
_AVGP = {1: F.avg_pool1d, 2: F.avg_pool2d, 3: F.avg_pool3d}


# ----------------------------------------------------------------------------- op compilers
def _op_conv(n, opset):
    a = n.attrs
    g = int(a.get("group", 1))

    def f(x, w, b=None):
        nd, k, s, d, pads = _conv_geom(a, list(w.shape), list(x.shape))
        if pads[:nd] == pads[nd:]:
            return [_CONV[nd](x, w, b, s, pads[:nd], d, g)]
        return [_CONV[nd](F.pad(x, _pad_cfg(pads, nd)), w, b, s, 0, d, g)]
    return f


def _op_conv_transpose(n, opset):
    a = n.attrs
    g = int(a.get("group", 1))

    def f(x, w, b=None):
        nd = w.dim() - 2
        s = list(a.get("strides") or [1] * nd)
        d = list(a.get("dilations") or [1] * nd)
        op = list(a.get("output_padding") or [0] * nd)
        k = list(a.get("kernel_shape") or w.shape[2:])
        pads = list(a.get("pads") or [0] * (2 * nd))
        if a.get("output_shape"):
            outs = list(a["output_shape"])[-nd:]
            tot = [s[i] * (x.shape[2 + i] - 1) + op[i] + ((k[i] - 1) * d[i] + 1) - outs[i] for i in range(nd)]
            upper = a.get("auto_pad", "SAME_UPPER") != "SAME_LOWER"
            pads = [t // 2 if upper else t - t // 2 for t in tot] + [t - (t // 2 if upper else t - t // 2) for t in tot]
        if pads[:nd] == pads[nd:]:
            return [_CONVT[nd](x, w, b, s, pads[:nd], op, g, d)]
        y = _CONVT[nd](x, w, b, s, 0, op, g, d)
        sl = [slice(None), slice(None)] + [slice(pads[i], y.shape[2 + i] - pads[i + nd]) for i in range(nd)]
        return [y[tuple(sl)]]
    return f


def _op_pool(n, opset, kind):
    a = n.attrs

    def f(x):
        nd = x.dim() - 2
        k = list(a["kernel_shape"])
        s = list(a.get("strides") or [1] * nd)
        d = list(a.get("dilations") or [1] * nd)
        auto = a.get("auto_pad", "NOTSET")
        pads = (_same_pads(x.shape[2:], k, s, d, auto) if auto in ("SAME_UPPER", "SAME_LOWER")
                else list(a.get("pads") or [0] * (2 * nd)))
        ceil = bool(a.get("ceil_mode", 0))
        sym = pads[:nd] == pads[nd:] and all(pads[i] <= k[i] // 2 for i in range(nd))
        if kind == "max":
            if sym:
                return [_MAXP[nd](x, k, s, pads[:nd], d, ceil)]
            xp = F.pad(x, _pad_cfg(pads, nd), value=float("-inf"))
            return [_MAXP[nd](xp, k, s, 0, d, ceil)]
        cip = bool(a.get("count_include_pad", 0))
        if sym and not ceil:
            return [_AVGP[nd](x, k, s, pads[:nd], ceil, cip)]
        xp = F.pad(x, _pad_cfg(pads, nd))
        y = _AVGP[nd](xp, k, s, 0, ceil, True)
        if cip:
            return [y]
        m = F.pad(torch.ones_like(x[:1, :1]), _pad_cfg(pads, nd))
        return [y / _AVGP[nd](m, k, s, 0, ceil, True)]
    return f


def _op_resize(n, opset):
    a = n.attrs
    upsample = n.op_type == "Upsample"
    mode = a.get("mode", "nearest")
    mode = {"bilinear": "linear", "trilinear": "linear"}.get(mode, mode)
    ctm = "asymmetric" if (upsample or opset < 11) else a.get("coordinate_transformation_mode", "half_pixel")
    nmode = "floor" if (upsample or opset < 11) else a.get("nearest_mode", "round_prefer_floor")

    def f(x, *rest):
        scales, sizes = None, None
        if upsample:
            scales = a.get("scales") if opset < 9 else (rest[0] if rest else None)
        elif opset < 11:
            scales = rest[0] if rest else None
        else:
            scales = rest[1] if len(rest) > 1 else None
            sizes = rest[2] if len(rest) > 2 else None
        scales = [float(v) for v in (scales.reshape(-1).tolist() if torch.is_tensor(scales) else (scales or []))]
        sizes = _ints(sizes)
        nd = x.dim() - 2
        if sizes:
            out = sizes[-nd:]
            sc = [out[i] / x.shape[2 + i] for i in range(nd)]
        else:
            if scales[:2] not in ([1.0, 1.0], []) and len(scales) == x.dim():
                raise NotImplementedError("Resize over batch/channel axes")
            sc = scales[-nd:]
            out = [int(math.floor(x.shape[2 + i] * sc[i])) for i in range(nd)]
        if mode == "nearest" and ctm == "asymmetric" and nmode == "floor" and not sizes:
            return [F.interpolate(x, scale_factor=sc, mode="nearest", recompute_scale_factor=False)]
        if mode == "linear" and nd in (1, 2, 3) and ctm in ("half_pixel", "pytorch_half_pixel", "align_corners"):
            im = {1: "linear", 2: "bilinear", 3: "trilinear"}[nd]
            if ctm == "align_corners":
                return [F.interpolate(x, size=out, mode=im, align_corners=True)]
            if ctm == "half_pixel" or all(o > 1 for o in out):
                kw = dict(size=out) if sizes else dict(scale_factor=sc, recompute_scale_factor=False)
                return [F.interpolate(x, mode=im, align_corners=False, **kw)]
        if mode == "cubic" and nd == 2 and ctm in ("half_pixel", "align_corners") and a.get("cubic_coeff_a", -0.75) == -0.75:
            if ctm == "align_corners":
                return [F.interpolate(x, size=out, mode="bicubic", align_corners=True)]
            kw = dict(size=out) if sizes else dict(scale_factor=sc, recompute_scale_factor=False)
            return [F.interpolate(x, mode="bicubic", align_corners=False, **kw)]
        if mode == "cubic":
            raise NotImplementedError(f"Resize cubic with {ctm}")
        # generic separable path (exact ONNX coordinate transforms)
        y = x
        for i in range(nd):
            L, O, s = x.shape[2 + i], out[i], sc[i]
            o = torch.arange(O, dtype=torch.float64)
            if ctm == "half_pixel":
                src = (o + 0.5) / s - 0.5
            elif ctm == "pytorch_half_pixel":
                src = (o + 0.5) / s - 0.5 if O > 1 else torch.zeros_like(o)
            elif ctm == "align_corners":
                src = o * (L - 1) / (O - 1) if O > 1 else torch.zeros_like(o)
            elif ctm == "tf_half_pixel_for_nn":
                src = (o + 0.5) / s
            else:
                src = o / s
            dim = 2 + i
            if mode == "nearest":
                idx = {"round_prefer_floor": torch.ceil(src - 0.5), "round_prefer_ceil": torch.floor(src + 0.5),
                       "floor": torch.floor(src), "ceil": torch.ceil(src)}[nmode]
                idx = idx.clamp(0, L - 1).long().to(x.device)
                y = y.index_select(dim, idx)
            else:
                src = src.clamp(0, L - 1)
                i0 = src.floor().long()
                i1 = (i0 + 1).clamp(max=L - 1)
                wt = (src - i0).to(x.dtype).to(x.device)
                shp = [1] * y.dim()
                shp[dim] = O
                wt = wt.view(shp)
                y = y.index_select(dim, i0.to(x.device)) * (1 - wt) + y.index_select(dim, i1.to(x.device)) * wt
        return [y]
    return f


def _axes_arg(n, opset, rest, since):
    if opset >= since:
        return _ints(rest[0]) if rest and rest[0] is not None else None
    v = n.attrs.get("axes")
    return list(v) if v is not None else None


def _op_reduce(n, opset, fn, since):
    keep = bool(n.attrs.get("keepdims", 1))
    noop = bool(n.attrs.get("noop_with_empty_axes", 0))

    def f(x, *rest):
        axes = _axes_arg(n, opset, rest, since)
        if not axes:
            if noop:
                return [x]
            axes = list(range(x.dim()))
        return [fn(x, axes, keep)]
    return f


def _reduce_max(x, ax, k):
    return torch.amax(x, dim=ax, keepdim=k)


def _reduce_min(x, ax, k):
    return torch.amin(x, dim=ax, keepdim=k)


def _reduce_prod(x, ax, k):
    for d in sorted([a % x.dim() for a in ax], reverse=True):
        x = torch.prod(x, dim=d, keepdim=k)
    return x


def _op_softmax(n, opset, fn):
    axis = n.attrs.get("axis", 1 if opset < 13 else -1)

    def f(x):
        if opset >= 13:
            return [fn(x, dim=axis)]
        ax = axis % x.dim()
        shp = x.shape
        y = fn(x.reshape(int(math.prod(shp[:ax])), -1), dim=1)
        return [y.reshape(shp)]
    return f


def _op_slice(n, opset):
    def f(x, *rest):
        if opset < 10:
            starts, ends = list(n.attrs["starts"]), list(n.attrs["ends"])
            axes = list(n.attrs.get("axes") or range(len(starts)))
            steps = [1] * len(starts)
        else:
            starts, ends = _ints(rest[0]), _ints(rest[1])
            axes = _ints(rest[2]) if len(rest) > 2 and rest[2] is not None else list(range(len(starts)))
            steps = _ints(rest[3]) if len(rest) > 3 and rest[3] is not None else [1] * len(starts)
        sl = [slice(None)] * x.dim()
        rev = []
        for st, en, ax, sp in zip(starts, ends, axes, steps):
            ax %= x.dim()
            L = x.shape[ax]
            b, e, s = slice(st, en, sp).indices(L)
            if s > 0:
                sl[ax] = slice(b, e, s)
            else:
                rev.append((ax, torch.arange(b, e, s)))
        y = x[tuple(sl)]
        for ax, idx in rev:
            y = y.index_select(ax, idx.to(y.device))
        return [y]
    return f


def _op_pad(n, opset):
    mode = {"constant": "constant", "reflect": "reflect", "edge": "replicate", "wrap": "circular"}[n.attrs.get("mode", "constant")]

    def f(x, *rest):
        if opset < 11:
            pads, val, axes = list(n.attrs["pads"]), float(n.attrs.get("value", 0.0)), None
        else:
            pads = _ints(rest[0])
            val = _scalar(rest[1]) if len(rest) > 1 and rest[1] is not None else 0
            axes = _ints(rest[2]) if len(rest) > 2 and rest[2] is not None else None
        r = x.dim()
        if axes is not None:
            full = [0] * (2 * r)
            k = len(axes)
            for j, ax in enumerate(axes):
                full[ax % r], full[ax % r + r] = pads[j], pads[j + k]
            pads = full
        first = next((i for i in range(r) if pads[i] or pads[i + r]), r)
        nd = r - first
        if nd == 0:
            return [x]
        cfg = []
        for i in reversed(range(first, r)):
            cfg += [pads[i], pads[i + r]]
        if mode == "constant":
            return [F.pad(x, cfg, value=val)]
        lead = x.shape[:first]
        y = x.reshape(1, -1, *x.shape[first:]) if first != 2 or r < 3 else x
        y = F.pad(y, cfg, mode=mode)
        return [y.reshape(*lead, *y.shape[-nd:]) if y is not x else y]
    return f


def _op_reshape(n, opset):
    allowzero = bool(n.attrs.get("allowzero", 0))

    def f(x, shape=None):
        shp = _ints(shape) if opset >= 5 else list(n.attrs["shape"])
        if not allowzero:
            shp = [x.shape[i] if v == 0 else v for i, v in enumerate(shp)]
        return [x.reshape(shp)]
    return f


def _op_squeeze(n, opset, un):
    def f(x, axes=None):
        ax = _ints(axes) if opset >= 13 and axes is not None else list(n.attrs.get("axes") or [])
        if un:
            r = x.dim() + len(ax)
            for a_ in sorted(a % r for a in ax):
                x = x.unsqueeze(a_)
            return [x]
        if not ax:
            return [x.squeeze()]
        for a_ in sorted((a % x.dim() for a in ax), reverse=True):
            x = x.squeeze(a_)
        return [x]
    return f


def _op_split(n, opset):
    axis = n.attrs.get("axis", 0)
    nout = len(n.outputs)

    def f(x, split=None):
        sp = _ints(split) if opset >= 13 and split is not None else list(n.attrs.get("split") or [])
        if not sp:
            L = x.shape[axis]
            c = math.ceil(L / nout)
            sp = [c] * (nout - 1) + [L - c * (nout - 1)]
        return list(torch.split(x, sp, dim=axis))
    return f


def _op_gather(n, opset):
    axis = n.attrs.get("axis", 0)

    def f(x, idx):
        ax = axis % x.dim()
        idx = _on(idx.long(), x)
        idx = torch.where(idx < 0, idx + x.shape[ax], idx)
        y = x.index_select(ax, idx.reshape(-1))
        return [y.reshape(tuple(x.shape[:ax]) + tuple(idx.shape) + tuple(x.shape[ax + 1:]))]
    return f


def _op_cast(n, opset):
    dt = P._TORCH[n.attrs["to"]]
    return lambda x: [x.to(dt)]


def _op_constant(n, opset, base):
    a = n.attrs
    if "value" in a:
        v = P.tensor_to_torch(a["value"], base)
    elif "value_float" in a:
        v = torch.tensor(float(a["value_float"]))
    elif "value_floats" in a:
        v = torch.tensor(list(a["value_floats"]), dtype=torch.float32)
    elif "value_int" in a:
        v = torch.tensor(int(a["value_int"]))
    elif "value_ints" in a:
        v = torch.tensor(list(a["value_ints"]), dtype=torch.int64)
    else:
        raise NotImplementedError(f"Constant with {list(a)}")
    return v


def _op_shape(n, opset):
    start, end = n.attrs.get("start", 0), n.attrs.get("end")

    def f(x):
        return [torch.tensor(list(x.shape)[start:end], dtype=torch.int64)]
    return f


def _op_gemm(n, opset):
    a = n.attrs
    alpha, beta = float(a.get("alpha", 1.0)), float(a.get("beta", 1.0))
    ta, tb = int(a.get("transA", 0)), int(a.get("transB", 0))

    def f(A, B, C=None):
        A = A.t() if ta else A
        B = B.t() if tb else B
        y = A @ B
        if alpha != 1.0:
            y = y * alpha
        if C is not None:
            y = y + (C * beta if beta != 1.0 else C)
        return [y]
    return f


def _op_clip(n, opset):
    def f(x, lo=None, hi=None):
        if opset < 11:
            lo, hi = n.attrs.get("min"), n.attrs.get("max")
        lo, hi = _scalar(lo), _scalar(hi)
        return [torch.clamp(x, lo, hi)]
    return f


def _op_norm(n, opset, kind):
    eps = float(n.attrs.get("epsilon", 1e-5))

    def f(x, scale=None, bias=None, mean=None, var=None):
        if kind == "bn":
            return [F.batch_norm(x, mean, var, scale, bias, False, 0.0, eps)]
        if kind == "in":
            return [F.instance_norm(x, weight=scale, bias=bias, eps=eps)]
        if kind == "gn":
            G = int(n.attrs["num_groups"])
            C = x.shape[1]
            if scale is not None and scale.numel() == G and G != C:  # opset 18: per-group affine
                scale, bias = scale.repeat_interleave(C // G), bias.repeat_interleave(C // G)
            return [F.group_norm(x, G, scale, bias, eps)]
        axis = n.attrs.get("axis", -1) % x.dim()
        return [F.layer_norm(x, x.shape[axis:], scale, bias, eps)]
    return f


def _op_depth_space(n, opset, d2s):
    bs = int(n.attrs["blocksize"])
    mode = n.attrs.get("mode", "DCR")

    def f(x):
        N, C, H, W = x.shape
        if d2s:
            if mode == "CRD":
                return [F.pixel_shuffle(x, bs)]
            y = x.reshape(N, bs, bs, C // (bs * bs), H, W).permute(0, 3, 4, 1, 5, 2)
            return [y.reshape(N, C // (bs * bs), H * bs, W * bs)]
        y = x.reshape(N, C, H // bs, bs, W // bs, bs).permute(0, 3, 5, 1, 2, 4)
        return [y.reshape(N, C * bs * bs, H // bs, W // bs)]
    return f


def _variadic(fn):
    def f(*xs):
        y = xs[0]
        for t in xs[1:]:
            y = fn(y, _on(t, y))
        return [y]
    return f


def _op_expand(n, opset):
    def f(x, shape):
        shp = torch.broadcast_shapes(tuple(x.shape), tuple(_ints(shape)))
        return [x.expand(shp)]
    return f


def _op_arg(n, opset, fn):
    axis, keep = n.attrs.get("axis", 0), bool(n.attrs.get("keepdims", 1))
    last = bool(n.attrs.get("select_last_index", 0))

    def f(x):
        if last:
            L = x.shape[axis]
            return [L - 1 - fn(x.flip(axis), dim=axis, keepdim=keep)]
        return [fn(x, dim=axis, keepdim=keep)]
    return f


def _unary(fn):
    return lambda n, opset: (lambda x: [fn(x)])


_UNARY = {
    "Relu": torch.relu, "Sigmoid": torch.sigmoid, "Tanh": torch.tanh, "Exp": torch.exp, "Log": torch.log,
    "Sqrt": torch.sqrt, "Abs": torch.abs, "Neg": torch.neg, "Reciprocal": torch.reciprocal, "Floor": torch.floor,
    "Ceil": torch.ceil, "Round": torch.round, "Erf": torch.erf, "Sin": torch.sin, "Cos": torch.cos,
    "Not": torch.logical_not, "Softplus": F.softplus, "Softsign": F.softsign, "Mish": F.mish,
    "HardSwish": F.hardswish, "IsNaN": torch.isnan, "Sign": torch.sign, "Identity": lambda x: x,
}
_BINARY = {
    "Add": torch.add, "Sub": torch.sub, "Mul": torch.mul, "Div": _div, "Pow": torch.pow, "MatMul": torch.matmul,
    "Equal": torch.eq, "Greater": torch.gt, "Less": torch.lt, "GreaterOrEqual": torch.ge, "LessOrEqual": torch.le,
    "And": torch.logical_and, "Or": torch.logical_or, "Xor": torch.logical_xor,
    "Mod": torch.remainder, "PRelu": lambda x, s: torch.where(x >= 0, x, x * s),
}


def compile_node(n, opset: int, base=None):
    """Return ``f(*inputs) -> list[outputs]`` for one NodeProto (attributes resolved now)."""
    t, a = n.op_type, n.attrs
    if n.domain not in ("", "ai.onnx"):
        raise NotImplementedError(f"ONNX op {n.domain}::{t}")
    if t in _UNARY:
        return _unary(_UNARY[t])(n, opset)
    if t in _BINARY:
        return _bin(_BINARY[t])
    simple = {
        "Conv": _op_conv, "ConvTranspose": _op_conv_transpose, "Resize": _op_resize, "Upsample": _op_resize,
        "Slice": _op_slice, "Pad": _op_pad, "Reshape": _op_reshape, "Split": _op_split, "Gather": _op_gather,
        "Cast": _op_cast, "Shape": _op_shape, "Gemm": _op_gemm, "Clip": _op_clip, "Expand": _op_expand,
    }
    if t in simple:
        return simple[t](n, opset)
    if t in ("MaxPool", "AveragePool"):
        return _op_pool(n, opset, "max" if t == "MaxPool" else "avg")
    if t in ("GlobalAveragePool", "GlobalMaxPool"):
        red = torch.mean if t == "GlobalAveragePool" else torch.amax
        return lambda x: [red(x, dim=tuple(range(2, x.dim())), keepdim=True)]
    if t in ("Squeeze", "Unsqueeze"):
        return _op_squeeze(n, opset, t == "Unsqueeze")
    if t == "Flatten":
        ax = a.get("axis", 1)
        return lambda x: [x.reshape(int(math.prod(x.shape[:ax % max(x.dim(), 1)] if ax else [1])), -1)]
    if t == "Transpose":
        perm = a.get("perm")
        return lambda x: [x.permute(*(perm or reversed(range(x.dim()))))]
    if t == "Concat":
        ax = a["axis"]

        def cat(*xs):
            dev = next((x.device for x in xs if x.device.type != "cpu"), xs[0].device)
            return [torch.cat([x.to(dev) for x in xs], dim=ax)]
        return cat
    if t == "Dropout":
        return lambda x, *r: [x, torch.ones_like(x, dtype=torch.bool)][:len(n.outputs)]
    if t == "ConstantOfShape":
        v = P.tensor_to_torch(a["value"], base) if "value" in a else torch.zeros(1)
        return lambda shape: [torch.full(_ints(shape), v.reshape(-1)[0].item(), dtype=v.dtype)]
    if t == "Size":
        return lambda x: [torch.tensor(x.numel(), dtype=torch.int64)]
    if t == "BatchNormalization":
        return _op_norm(n, opset, "bn")
    if t == "InstanceNormalization":
        return _op_norm(n, opset, "in")
    if t == "GroupNormalization":
        return _op_norm(n, opset, "gn")
    if t == "LayerNormalization":
        return _op_norm(n, opset, "ln")
    if t in ("Softmax", "LogSoftmax"):
        return _op_softmax(n, opset, F.softmax if t == "Softmax" else F.log_softmax)
    if t == "LeakyRelu":
        al = float(a.get("alpha", 0.01))
        return lambda x: [F.leaky_relu(x, al)]
    if t == "Elu":
        al = float(a.get("alpha", 1.0))
        return lambda x: [F.elu(x, al)]
    if t == "Selu":
        al, gm = float(a.get("alpha", 1.67326319217681884765625)), float(a.get("gamma", 1.05070102214813232421875))
        return lambda x: [gm * torch.where(x > 0, x, al * (torch.exp(x) - 1))]
    if t == "HardSigmoid":
        al, be = float(a.get("alpha", 0.2)), float(a.get("beta", 0.5))
        return lambda x: [torch.clamp(al * x + be, 0, 1)]
    if t == "Gelu":
        ap = a.get("approximate", "none")
        return lambda x: [F.gelu(x, approximate=ap)]
    if t in ("Sum", "Max", "Min", "Mean"):
        fn = {"Sum": torch.add, "Max": torch.maximum, "Min": torch.minimum, "Mean": torch.add}[t]
        g = _variadic(fn)
        return (lambda *xs: [g(*xs)[0] / len(xs)]) if t == "Mean" else g
    if t == "Where":
        return lambda c, x, y: [torch.where(_on(c, x), x, _on(y, x))]
    if t == "ReduceMean":
        return _op_reduce(n, opset, lambda x, ax, k: torch.mean(x, dim=ax, keepdim=k), 18)
    if t == "ReduceSum":
        return _op_reduce(n, opset, lambda x, ax, k: torch.sum(x, dim=ax, keepdim=k), 13)
    if t == "ReduceMax":
        return _op_reduce(n, opset, _reduce_max, 18)
    if t == "ReduceMin":
        return _op_reduce(n, opset, _reduce_min, 18)
    if t == "ReduceProd":
        return _op_reduce(n, opset, _reduce_prod, 18)
    if t == "ReduceL2":
        return _op_reduce(n, opset, lambda x, ax, k: torch.sqrt(torch.sum(x * x, dim=ax, keepdim=k)), 18)
    if t == "ReduceSumSquare":
        return _op_reduce(n, opset, lambda x, ax, k: torch.sum(x * x, dim=ax, keepdim=k), 18)
    if t in ("ArgMax", "ArgMin"):
        return _op_arg(n, opset, torch.argmax if t == "ArgMax" else torch.argmin)
    if t in ("DepthToSpace", "SpaceToDepth"):
        return _op_depth_space(n, opset, t == "DepthToSpace")
    if t == "Tile":
        return lambda x, rep: [x.repeat(*_ints(rep))]
    if t == "Range":
        return lambda s, e, d: [torch.arange(_scalar(s), _scalar(e), _scalar(d), dtype=s.dtype)]
    if t == "Einsum":
        eq = a["equation"]
        return lambda *xs: [torch.einsum(eq, *xs)]
    raise NotImplementedError(f"ONNX op {t} (opset {opset}) is not supported by the MI355X runtime")


# ----------------------------------------------------------------------------- fusion
def _eligible_geom(a, w):
    """(nd, kernel, strides, dilations, symmetric pads or None) of a constant-weight conv."""
    nd, k, s, d, pads = _conv_geom(a, list(w.shape))
    if a.get("auto_pad", "NOTSET") in ("SAME_UPPER", "SAME_LOWER"):
        pads = ([x // 2 for x in k] * 2 if all(x % 2 == 1 for x in k) and set(s) == {1} and set(d) == {1}
                else None)
    return nd, k, s, d, (pads if pads is not None and pads[:nd] == pads[nd:] else None)


class _ConvSpec:
    """A Conv/ConvTranspose with constant weights, as the nn module convert.py's Hip* classes take."""

    @staticmethod
    def conv(w, b, nd, k, s, d, pads, groups=1):
        cls = {2: nn.Conv2d, 3: nn.Conv3d}[nd]
        m = cls(w.shape[1] * groups, w.shape[0], k, s, [p for p in pads[:nd]], d, groups, b is not None)
        with torch.no_grad():
            m.weight.copy_(w.float())
            if b is not None:
                m.bias.copy_(b.float())
        return m.eval()


class OnnxModule(nn.Module):
    """An ONNX graph as a torch module; ``forward(*inputs)`` in graph-input order."""

    def __init__(self, model: "P.Model", optimize: bool = False, base_dir=None):
        super().__init__()
        g = model.graph
        self.opset = model.opset.get("", model.opset.get("ai.onnx", 13))
        self.base_dir = base_dir
        consts: dict[str, torch.Tensor] = {}
        for t in g.initializers:
            consts[t.name] = P.tensor_to_torch(t, base_dir)
        self.input_names = [vi.name for vi in g.inputs if vi.name not in consts]
        self.output_names = [vi.name for vi in g.outputs]
        nodes = []
        for n in g.nodes:  # fold Constant nodes into the constant table
            if n.op_type == "Constant" and n.domain in ("", "ai.onnx"):
                consts[n.outputs[0]] = _op_constant(n, self.opset, base_dir)
            else:
                nodes.append(n)
        self.stats = {"nodes": len(nodes), "convs": 0, "bn_folded": 0, "relu_fused": 0, "norm_fused": 0,
                      "conv_transpose": 0, "strided": 0, "skipped": 0}
        self.fused = nn.ModuleList()
        steps = self._fuse(nodes, consts) if optimize else [(n, None) for n in nodes]
        # float constants become buffers (moved/cast by .to); integer ones stay CPU shape data
        self._const_cpu: dict[str, torch.Tensor] = {}
        self._buf_of: dict[str, str] = {}
        used = {i for n, _ in steps for i in n.inputs} | set(self.output_names)
        meta = {x for n, _ in steps for j, x in enumerate(n.inputs) if j >= _META_FROM.get(n.op_type, 99)}
        for name, v in consts.items():
            if name not in used:
                continue
            if v.is_floating_point() and name not in meta:
                key = f"c{len(self._buf_of)}"
                self.register_buffer(key, v, persistent=False)
                self._buf_of[name] = key
            else:
                self._const_cpu[name] = v
        self._steps = []
        for n, mod in steps:
            fn = mod if mod is not None else compile_node(n, self.opset, base_dir)
            self._steps.append((n.op_type, fn, list(n.inputs), list(n.outputs)))
        # drop activations after their last use (keeps peak memory at the live set)
        last = {}
        for i, (_, _, ins, _) in enumerate(self._steps):
            for x in ins:
                last[x] = i
        self._free = [[x for x in ins if last.get(x) == i and x not in self.output_names]
                      for i, (_, _, ins, _) in enumerate(self._steps)]

    @classmethod
    def from_file(cls, path, optimize: bool = False) -> "OnnxModule":
        m = P.load_model(path)
        return cls(m, optimize=optimize, base_dir=str(Path(path).parent))

    # ------------------------------------------------------------------ fusion pass
    def _fuse(self, nodes, consts):
        consumers: dict[str, list[int]] = {}
        for i, n in enumerate(nodes):
            for x in n.inputs:
                consumers.setdefault(x, []).append(i)
        outs = set(self.output_names)

        def sole(name):
            c = consumers.get(name, [])
            return nodes[c[0]] if len(c) == 1 and name not in outs else None

        def const(name):
            return consts.get(name) if name else None

        from .convert import (HipConv2d, HipConv3d, HipConvStride2x2, HipConvTranspose2x2, HipNormConv2d,
                              _eligible, _eligible3d, fold_bn)

        dead: set[int] = set()
        out: list = []
        idx = {id(n): i for i, n in enumerate(nodes)}
        for i, n in enumerate(nodes):
            if i in dead:
                continue
            st = self.stats
            if n.op_type == "Conv" and const(n.inputs[1]) is not None and int(n.attrs.get("group", 1)) == 1:
                w = const(n.inputs[1])
                b = const(n.inputs[2]) if len(n.inputs) > 2 else None
                if len(n.inputs) > 2 and n.inputs[2] and b is None:
                    out.append((n, None))
                    continue
                nd, k, s, d, pads = _eligible_geom(n.attrs, w)
                if nd not in (2, 3) or pads is None:
                    out.append((n, None))
                    st["skipped"] += 1
                    continue
                chain, y = [], n.outputs[0]
                conv = _ConvSpec.conv(w, b, nd, k, s, d, pads)
                nx = sole(y)
                if (nx is not None and nx.op_type == "BatchNormalization" and len(nx.outputs) == 1
                        and all(const(x) is not None for x in nx.inputs[1:5])):
                    bn = (nn.BatchNorm2d if nd == 2 else nn.BatchNorm3d)(w.shape[0], eps=float(nx.attrs.get("epsilon", 1e-5)))
                    with torch.no_grad():
                        bn.weight.copy_(const(nx.inputs[1]).float())
                        bn.bias.copy_(const(nx.inputs[2]).float())
                        bn.running_mean.copy_(const(nx.inputs[3]).float())
                        bn.running_var.copy_(const(nx.inputs[4]).float())
                    conv = fold_bn(conv, bn.eval())
                    chain.append(nx)
                    y = nx.outputs[0]
                    st["bn_folded"] += 1
                    nx = sole(y)
                relu = nx is not None and nx.op_type == "Relu"
                s2 = nd == 2 and k == [2, 2] and s == [2, 2] and d == [1, 1] and pads == [0, 0, 0, 0]
                ok = _eligible(conv) if nd == 2 else _eligible3d(conv)
                if not (ok or s2):
                    if chain:  # keep the BN fold even when the conv stays on MIOpen
                        mod = _TorchConv(conv)
                        self.fused.append(mod)
                        out.append((_synthetic("Conv", [n.inputs[0]], [y]), mod))
                        dead.update(idx[id(c)] for c in chain)
                    else:
                        out.append((n, None))
                    st["skipped"] += 1
                    continue
                if relu:
                    chain.append(nx)
                    y = nx.outputs[0]
                    st["relu_fused"] += 1
                if s2:
                    mod = HipConvStride2x2(conv, post_relu=relu)
                    st["strided"] += 1
                else:
                    mod = (HipConv2d if nd == 2 else HipConv3d)(conv, post_relu=relu)
                    st["convs"] += 1
                self.fused.append(mod)
                dead.update(idx[id(c)] for c in chain)
                out.append((_synthetic("HipConv", [n.inputs[0]], [y]), mod))
                continue
            if n.op_type in ("InstanceNormalization", "GroupNormalization") and all(const(x) is not None for x in n.inputs[1:3]):
                chain, y = [], n.outputs[0]
                nx = sole(y)
                relu = nx is not None and nx.op_type == "Relu"
                if relu:
                    chain.append(nx)
                    y = nx.outputs[0]
                    nx = sole(y)
                if (nx is not None and nx.op_type == "Conv" and nx.inputs[0] == y and const(nx.inputs[1]) is not None
                        and const(nx.inputs[1]).dim() == 4 and int(nx.attrs.get("group", 1)) == 1):
                    w = const(nx.inputs[1])
                    b = const(nx.inputs[2]) if len(nx.inputs) > 2 and nx.inputs[2] else None
                    _, k, s, d, pads = _eligible_geom(nx.attrs, w)
                    conv = _ConvSpec.conv(w, b, 2, k, s, d, pads) if pads is not None else None
                    if conv is not None and _eligible(conv):
                        C = w.shape[1]
                        G = C if n.op_type == "InstanceNormalization" else int(n.attrs["num_groups"])
                        sc, bi = const(n.inputs[1]).float(), const(n.inputs[2]).float()
                        if sc.numel() == G and G != C:
                            sc, bi = sc.repeat_interleave(C // G), bi.repeat_interleave(C // G)
                        norm = nn.GroupNorm(G, C, eps=float(n.attrs.get("epsilon", 1e-5)))
                        with torch.no_grad():
                            norm.weight.copy_(sc)
                            norm.bias.copy_(bi)
                        chain.append(nx)
                        y = nx.outputs[0]
                        nx2 = sole(y)
                        post = nx2 is not None and nx2.op_type == "Relu"
                        if post:
                            chain.append(nx2)
                            y = nx2.outputs[0]
                            st["relu_fused"] += 1
                        mod = HipNormConv2d(norm, relu, conv, post_relu=post)
                        self.fused.append(mod)
                        dead.update(idx[id(c)] for c in chain)
                        out.append((_synthetic("HipNormConv", [n.inputs[0]], [y]), mod))
                        st["norm_fused"] += 1
                        st["convs"] += 1
                        continue
                out.append((n, None))
                continue
            if n.op_type == "ConvTranspose" and const(n.inputs[1]) is not None:
                w = const(n.inputs[1])
                b = const(n.inputs[2]) if len(n.inputs) > 2 and n.inputs[2] else None
                a = n.attrs
                if (w.dim() == 4 and list(w.shape[2:]) == [2, 2] and list(a.get("strides") or [1, 1]) == [2, 2]
                        and not any(a.get("pads") or []) and not any(a.get("output_padding") or [])
                        and list(a.get("dilations") or [1, 1]) == [1, 1] and int(a.get("group", 1)) == 1
                        and not a.get("output_shape")):
                    ct = nn.ConvTranspose2d(w.shape[0], w.shape[1], 2, 2, bias=b is not None)
                    with torch.no_grad():
                        ct.weight.copy_(w.float())
                        if b is not None:
                            ct.bias.copy_(b.float())
                    mod = HipConvTranspose2x2(ct.eval())
                    self.fused.append(mod)
                    out.append((_synthetic("HipConvTranspose", [n.inputs[0]], [n.outputs[0]]), mod))
                    st["conv_transpose"] += 1
                    continue
            out.append((n, None))
        return out

    # ------------------------------------------------------------------ run
    def forward(self, *xs):
        env: dict[str, torch.Tensor] = {}
        for name, x in zip(self.input_names, xs):
            env[name] = x
        for name, key in self._buf_of.items():
            env[name] = getattr(self, key)
        env.update(self._const_cpu)
        for (op, fn, ins, outs), free in zip(self._steps, self._free):
            args = [env[x] if x else None for x in ins]
            while args and args[-1] is None:
                args.pop()
            res = fn(*args) if not isinstance(fn, nn.Module) else [fn(args[0])]
            for name, v in zip(outs, res):
                if name:
                    env[name] = v
            for x in free:
                if x in env and x not in self._buf_of and x not in self._const_cpu:
                    del env[x]
        ys = [env[o] for o in self.output_names]
        return ys[0] if len(ys) == 1 else tuple(ys)


class _TorchConv(nn.Module):
    """A BN-folded conv that stays on MIOpen (shape not eligible for the MFMA kernel)."""

    def __init__(self, conv):
        super().__init__()
        self.conv = conv

    def forward(self, x):
        return self.conv(x.to(self.conv.weight.dtype))


def _synthetic(op, ins, outs):
    return P.Node(op, list(ins), list(outs))
