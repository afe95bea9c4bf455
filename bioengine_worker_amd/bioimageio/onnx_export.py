"""PyTorch -> ONNX export without the ``onnx`` package (``torch.onnx.export`` needs it and it is not in
this image): the module is traced with ``torch.fx`` and every node is written as the equivalent ONNX
op through :class:`.onnx_proto.GraphBuilder`.

Used to add an ``onnx`` weights entry to packages this framework writes (the reference's model runner
accepts all four bioimage.io weight formats, ``/root/reference/apps/model-runner/entry_deployment.py:
1884-1887``) and as the independent producer for the ONNX runtime's tests.  Covers the layers of
bioimage.io-style CNNs (conv / transposed conv / norms / pooling / resampling / activations, concat
and elementwise arithmetic); anything else raises with the layer's name.
"""
from __future__ import annotations

import operator

import torch
import torch.fx as fx
import torch.nn as nn
import torch.nn.functional as F

from .onnx_proto import GraphBuilder

_ACT = {nn.ReLU: "Relu", nn.Sigmoid: "Sigmoid", nn.Tanh: "Tanh", nn.Identity: "Identity", nn.Dropout: "Identity",
        nn.Softplus: "Softplus", nn.ELU: "Elu", nn.LeakyReLU: "LeakyRelu", nn.GELU: "Gelu"}
_FN = {torch.relu: "Relu", F.relu: "Relu", torch.sigmoid: "Sigmoid", torch.tanh: "Tanh", torch.exp: "Exp",
       operator.add: "Add", torch.add: "Add", operator.mul: "Mul", torch.mul: "Mul", operator.sub: "Sub",
       operator.truediv: "Div"}


def export_onnx(model: nn.Module, path, input_name: str = "input", output_name: str = "output",
                spatial_dims: int = 2) -> dict:
    """Write ``model`` (eval mode) as an ONNX file; returns {"opset": ..., "nodes": ...}."""
    model = model.eval()
    gm = fx.symbolic_trace(model)
    mods = dict(gm.named_modules())
    uses_gn = any(isinstance(m, nn.GroupNorm) for m in mods.values())
    b = GraphBuilder("bioengine_export", opset=21 if uses_gn else 17)
    names: dict[fx.Node, str] = {}
    counter = [0]

    def init(prefix, t):
        counter[0] += 1
        return b.init(f"{prefix}_{counter[0]}", t.detach().float().cpu())

    def arg(a):
        if isinstance(a, fx.Node):
            return names[a]
        return init("const", torch.tensor(float(a)))

    for n in gm.graph.nodes:
        if n.op == "placeholder":
            shape = ["N", "C"] + [f"d{i}" for i in range(spatial_dims)]
            names[n] = b.input(input_name, shape)
            continue
        if n.op == "output":
            src = n.args[0]
            b.node("Identity", [names[src]], [output_name])
            b.output(output_name)
            continue
        if n.op == "call_module":
            m = mods[n.target]
            x = names[n.args[0]]
            tag = n.target.replace(".", "_")
            if isinstance(m, (nn.Conv2d, nn.Conv3d)):
                if m.padding_mode != "zeros" or isinstance(m.padding, str):
                    raise NotImplementedError(f"{n.target}: padding {m.padding!r}/{m.padding_mode}")
                ins = [x, init(f"{tag}_w", m.weight)] + ([init(f"{tag}_b", m.bias)] if m.bias is not None else [])
                names[n] = b.node("Conv", ins, kernel_shape=list(m.kernel_size), strides=list(m.stride),
                                  dilations=list(m.dilation), group=m.groups, pads=list(m.padding) * 2)
            elif isinstance(m, (nn.ConvTranspose2d, nn.ConvTranspose3d)):
                ins = [x, init(f"{tag}_w", m.weight)] + ([init(f"{tag}_b", m.bias)] if m.bias is not None else [])
                names[n] = b.node("ConvTranspose", ins, kernel_shape=list(m.kernel_size), strides=list(m.stride),
                                  dilations=list(m.dilation), group=m.groups, pads=list(m.padding) * 2,
                                  output_padding=list(m.output_padding))
            elif isinstance(m, (nn.BatchNorm2d, nn.BatchNorm3d)):
                C = m.num_features
                w = m.weight if m.weight is not None else torch.ones(C)
                bb = m.bias if m.bias is not None else torch.zeros(C)
                names[n] = b.node("BatchNormalization", [x, init(f"{tag}_g", w), init(f"{tag}_b", bb),
                                                         init(f"{tag}_m", m.running_mean), init(f"{tag}_v", m.running_var)],
                                  epsilon=float(m.eps))
            elif isinstance(m, (nn.InstanceNorm2d, nn.InstanceNorm3d)):
                C = m.num_features
                w = m.weight if m.weight is not None else torch.ones(C)
                bb = m.bias if m.bias is not None else torch.zeros(C)
                names[n] = b.node("InstanceNormalization", [x, init(f"{tag}_g", w), init(f"{tag}_b", bb)],
                                  epsilon=float(m.eps))
            elif isinstance(m, nn.GroupNorm):  # opset 21: per-channel scale / bias
                C = m.num_channels
                w = m.weight if m.weight is not None else torch.ones(C)
                bb = m.bias if m.bias is not None else torch.zeros(C)
                names[n] = b.node("GroupNormalization", [x, init(f"{tag}_g", w), init(f"{tag}_b", bb)],
                                  num_groups=m.num_groups, epsilon=float(m.eps))
            elif isinstance(m, (nn.MaxPool2d, nn.MaxPool3d, nn.AvgPool2d, nn.AvgPool3d)):
                nd = 2 if isinstance(m, (nn.MaxPool2d, nn.AvgPool2d)) else 3

                def tup(v):
                    return list(v) if isinstance(v, (tuple, list)) else [v] * nd
                k = tup(m.kernel_size)
                s = tup(m.stride if m.stride is not None else m.kernel_size)
                p = tup(m.padding)
                kw = dict(kernel_shape=k, strides=s, pads=p * 2, ceil_mode=int(m.ceil_mode))
                if isinstance(m, (nn.MaxPool2d, nn.MaxPool3d)):
                    names[n] = b.node("MaxPool", [x], dilations=tup(m.dilation), **kw)
                else:
                    names[n] = b.node("AveragePool", [x], count_include_pad=int(m.count_include_pad), **kw)
            elif isinstance(m, nn.Upsample):
                sf = m.scale_factor
                if sf is None:
                    raise NotImplementedError(f"{n.target}: Upsample(size=...)")
                sf = list(sf) if isinstance(sf, (tuple, list)) else [sf] * spatial_dims
                scales = init(f"{tag}_scales", torch.tensor([1.0, 1.0] + [float(v) for v in sf]))
                mode = "nearest" if m.mode == "nearest" else "linear"
                ctm = "asymmetric" if mode == "nearest" else ("align_corners" if m.align_corners else "half_pixel")
                names[n] = b.node("Resize", [x, "", scales], mode=mode, coordinate_transformation_mode=ctm,
                                  nearest_mode="floor")
            elif isinstance(m, nn.Softmax):
                names[n] = b.node("Softmax", [x], axis=m.dim if m.dim is not None else 1)
            elif type(m) in _ACT:
                kw = {}
                if isinstance(m, nn.LeakyReLU):
                    kw["alpha"] = float(m.negative_slope)
                elif isinstance(m, nn.ELU):
                    kw["alpha"] = float(m.alpha)
                elif isinstance(m, nn.GELU):
                    kw["approximate"] = m.approximate
                names[n] = b.node(_ACT[type(m)], [x], **kw)
            else:
                raise NotImplementedError(f"ONNX export: layer {n.target} ({type(m).__name__})")
            continue
        if n.op == "call_function":
            if n.target in (torch.cat, torch.concat):
                xs = n.args[0]
                dim = n.kwargs.get("dim", n.args[1] if len(n.args) > 1 else 0)
                names[n] = b.node("Concat", [names[a] for a in xs], axis=int(dim))
            elif n.target in _FN:
                names[n] = b.node(_FN[n.target], [arg(a) for a in n.args])
            elif n.target is F.interpolate:
                sf = n.kwargs.get("scale_factor")
                mode = n.kwargs.get("mode", "nearest")
                if sf is None:
                    raise NotImplementedError("F.interpolate(size=...) export")
                sf = list(sf) if isinstance(sf, (tuple, list)) else [sf] * spatial_dims
                scales = init("interp_scales", torch.tensor([1.0, 1.0] + [float(v) for v in sf]))
                ac = bool(n.kwargs.get("align_corners"))
                names[n] = b.node("Resize", [names[n.args[0]], "", scales],
                                  mode="nearest" if mode == "nearest" else "linear",
                                  coordinate_transformation_mode="asymmetric" if mode == "nearest" else (
                                      "align_corners" if ac else "half_pixel"), nearest_mode="floor")
            else:
                raise NotImplementedError(f"ONNX export: function {n.target}")
            continue
        raise NotImplementedError(f"ONNX export: fx op {n.op} {n.target}")
    b.save(path)
    return {"opset": b.opset, "nodes": len(b._nodes)}
