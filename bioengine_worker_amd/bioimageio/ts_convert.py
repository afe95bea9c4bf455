"""MI355X graph pass for TorchScript-only bioimage.io weights (reference loads them with
``torch.jit.load`` and runs them as-is, ``apps/model-runner/runtime_deployment.py:187-312``).

A scripted/traced module's ``forward`` is TorchScript IR, so its submodules cannot be swapped for
Python modules the way :func:`.convert.optimize_for_mi355x` rewrites eager models.  Instead:

1. ``torch.jit.freeze`` inlines the weights as graph constants and folds every Conv→BatchNorm pair
   into the convolution (the frozen-graph conv-BN folding pass);
2. a pattern rewrite replaces ``aten::_convolution`` / ``aten::conv2d`` (and a directly following
   ``aten::relu``/``relu_``) by ``bioengine::hip_conv2d``, an operator registered with the
   dispatcher whose implementation runs eligible 2-D convolutions (1x1 / 3x3, stride 1, groups 1,
   "same" padding) on the fused NHWC MFMA conv kernel with the ReLU in its epilogue; the packed
   bf16 weights are built once per constant weight tensor and cached.  Everything else (3-D,
   strided, transposed convs) falls back to ATen inside the same operator.

Activations stay in the graph's dtype between operators (the rest of a TorchScript graph has fp32
constants), so each HIP conv converts its input to bf16 NHWC on the way in.
"""
from __future__ import annotations

import threading

import torch
import torch.nn.functional as F

_LIB = None
_LOCK = threading.Lock()
_CACHE: dict = {}
COUNTS = {"hip": 0, "fallback": 0}

_SCHEMA = ("hip_conv2d(Tensor x, Tensor w, Tensor? b, int[] stride, int[] padding, int[] dilation, bool transposed, "
           "int[] output_padding, int groups, bool relu) -> Tensor")


def _eligible(x, w, stride, padding, dilation, transposed, groups) -> bool:
    return (x.is_cuda and x.dim() == 4 and w.dim() == 4 and not transposed and groups == 1
            and w.shape[2] == w.shape[3] and w.shape[2] in (1, 3) and list(stride) == [1, 1]
            and list(dilation) == [1, 1] and list(padding) == [w.shape[2] // 2] * 2)


def _packed(w, b):
    from ..ops.conv import PackedConv

    key = (w.data_ptr(), tuple(w.shape), None if b is None else b.data_ptr())
    pc = _CACHE.get(key)
    if pc is None:
        cout = w.shape[0]
        pc = PackedConv.from_weight(w.detach().float(), None if b is None else b.detach().float(),
                                    cout_pad_to=16 if cout % 4 else None).to(w.device)
        _CACHE[key] = pc
    return pc


def _impl(x, w, b, stride, padding, dilation, transposed, output_padding, groups, relu):
    if not _eligible(x, w, stride, padding, dilation, transposed, groups):
        COUNTS["fallback"] += 1
        if transposed:
            y = F.conv_transpose2d(x, w, b, stride, padding, output_padding, groups, dilation) if x.dim() == 4 else \
                F.conv_transpose3d(x, w, b, stride, padding, output_padding, groups, dilation)
        else:
            y = (F.conv2d if x.dim() == 4 else F.conv3d)(x, w, b, stride, padding, dilation, groups)
        return torch.relu(y) if relu else y
    from ..ops.conv import fused_conv2d

    COUNTS["hip"] += 1
    pc = _packed(w, b)
    C = x.shape[1]
    xh = x.to(torch.bfloat16).permute(0, 2, 3, 1)
    if C != pc.cin_pad:
        xh = F.pad(xh, (0, pc.cin_pad - C))
    xh = xh.contiguous()
    cout = w.shape[0]
    if cout % 4:
        y = fused_conv2d(xh, pc, out_nchw_f32=True, cout_valid=cout, post_relu=relu)
        return y.to(x.dtype)
    return fused_conv2d(xh, pc, post_relu=relu).permute(0, 3, 1, 2).to(x.dtype)


def register() -> None:
    global _LIB
    with _LOCK:
        if _LIB is not None:
            return
        lib = torch.library.Library("bioengine", "DEF")
        lib.define(_SCHEMA)
        lib.impl("hip_conv2d", _impl, "CompositeExplicitAutograd")
        _LIB = lib


_ARGS13 = "%x, %w, %b, %s, %p, %d, %t, %op, %g, %b1, %b2, %b3, %b4"
_ARGS7 = "%x, %w, %b, %s, %p, %d, %g"


def _rules():
    rules = []
    for relu in ("aten::relu", "aten::relu_", None):
        tail = f"\n    %r = {relu}(%y)\n    return (%r)" if relu else "\n    return (%y)"
        flag = "1" if relu else "0"
        rules.append((f"graph({_ARGS13}):\n    %y = aten::_convolution({_ARGS13}){tail}",
                      f"graph({_ARGS13}):\n    %f : bool = prim::Constant[value={flag}]()\n"
                      f"    %r = bioengine::hip_conv2d(%x, %w, %b, %s, %p, %d, %t, %op, %g, %f)\n    return (%r)"))
        rules.append((f"graph({_ARGS7}):\n    %y = aten::conv2d({_ARGS7}){tail}",
                      f"graph({_ARGS7}):\n    %f : bool = prim::Constant[value={flag}]()\n"
                      f"    %t : bool = prim::Constant[value=0]()\n    %op : int[] = prim::Constant[value=[0, 0]]()\n"
                      f"    %r = bioengine::hip_conv2d(%x, %w, %b, %s, %p, %d, %t, %op, %g, %f)\n    return (%r)"))
    return rules


def optimize_torchscript(module: torch.jit.ScriptModule) -> tuple[torch.jit.ScriptModule, dict]:
    """Freeze + rewrite a loaded TorchScript model in place of its graph; returns (module, stats)."""
    register()
    frozen = torch.jit.freeze(module.eval())
    g = frozen.graph
    before = sum(1 for n in g.nodes() if n.kind() in ("aten::_convolution", "aten::conv2d"))
    relu_before = sum(1 for n in g.nodes() if n.kind() in ("aten::relu", "aten::relu_"))
    for pat, rep in _rules():
        torch._C._jit_pass_custom_pattern_based_rewrite_graph(pat, rep, g)
    hip = 0
    for n in g.nodes():  # transposed convolutions are rewritten too but run on ATen inside the op
        if n.kind() == "bioengine::hip_conv2d" and not n.inputsAt(6).toIValue():
            hip += 1
    relu_after = sum(1 for n in g.nodes() if n.kind() in ("aten::relu", "aten::relu_"))
    stats = {"convs": hip, "convs_in_graph": before, "relu_fused": relu_before - relu_after, "bn_folded": "freeze",
             "mode": "torchscript-rewrite"}
    return frozen, stats
