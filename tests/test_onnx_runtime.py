"""ONNX weights without onnx/onnxruntime: protobuf reader/writer round trip, op semantics against
PyTorch fp32 references, the fx exporter + executor on the package U-Nets (batch / group / instance
norm, pool / strided-conv downsampling), the fusion pass, and ONNX-only packages through the model
runner's PredictionPipeline / test_model.  (No onnx file ships in the reference; parity with
onnxruntime itself is unpinned — the oracle is the fp32 PyTorch model the file was exported from.)"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from bioengine_worker_amd.bioimageio import onnx_proto as P
from bioengine_worker_amd.bioimageio.onnx_runtime import OnnxModule
from bioengine_worker_amd.bioimageio.package import load_module, write_unet2d_package


def _run(b: P.GraphBuilder, *xs, opt=False):
    m = OnnxModule(P.parse_model(b.to_bytes()), optimize=opt)
    return m, m(*xs)


def test_proto_roundtrip_attributes_and_tensors():
    b = P.GraphBuilder("g", opset=13)
    b.input("x", ["N", 3])
    w = torch.randn(3, 4)
    b.init("w", w)
    b.init("i64", torch.tensor([-1, 5, 1 << 40]))
    b.init("h", torch.randn(5).half())
    b.node("MatMul", ["x", "w"], ["y"])
    b.node("LeakyRelu", ["y"], ["z"], alpha=0.25)
    b.node("Transpose", ["z"], ["out"], perm=[1, 0])
    b.output("out")
    m = P.parse_model(b.to_bytes())
    assert m.opset[""] == 13 and [n.op_type for n in m.graph.nodes] == ["MatMul", "LeakyRelu", "Transpose"]
    assert m.graph.nodes[1].attrs["alpha"] == pytest.approx(0.25) and m.graph.nodes[2].attrs["perm"] == [1, 0]
    assert m.graph.inputs[0].shape == ["N", 3]
    inits = {t.name: P.tensor_to_torch(t) for t in m.graph.initializers}
    assert torch.equal(inits["w"], w) and inits["i64"].tolist() == [-1, 5, 1 << 40]
    assert inits["h"].dtype == torch.float16
    x = torch.randn(2, 3)
    _, y = _run(b, x)
    assert torch.allclose(y, F.leaky_relu(x @ w, 0.25).t(), atol=1e-6)


def test_dynamic_shape_chain_and_slicing():
    """The Shape -> Gather -> Unsqueeze -> Concat -> Reshape chains exporters emit, Slice with a
    negative step, Pad (reflect), Split, Gather with negative indices, Softmax opset-11 semantics."""
    b = P.GraphBuilder("g", opset=13)
    b.input("x", ["N", "C", "H", "W"])
    b.init("zero", torch.tensor(0))
    b.init("minus1", torch.tensor([-1]))
    b.init("ax0", torch.tensor([0]))
    b.init("st", torch.tensor([-1]))
    b.init("en", torch.tensor([-(1 << 62)]))
    b.init("ax3", torch.tensor([3]))
    b.init("stp", torch.tensor([-1]))
    b.init("pads", torch.tensor([0, 0, 1, 2, 0, 0, 2, 1]))
    b.init("split", torch.tensor([1, 2]))
    b.init("gi", torch.tensor([-1, 0]))
    s = b.node("Shape", ["x"])
    n0 = b.node("Gather", [s, "zero"], axis=0)
    n0u = b.node("Unsqueeze", [n0, "ax0"])
    shp = b.node("Concat", [n0u, "minus1"], axis=0)
    b.node("Reshape", ["x", shp], ["flat"])
    b.node("Slice", ["x", "st", "en", "ax3", "stp"], ["flip"])
    b.node("Pad", ["x", "pads"], ["pad"], mode="reflect")
    b.node("Split", ["x", "split"], ["s1", "s2"], axis=1)
    b.node("Gather", ["x", "gi"], ["g"], axis=1)
    for o in ("flat", "flip", "pad", "s1", "s2", "g"):
        b.output(o)
    x = torch.randn(2, 3, 5, 6)
    _, ys = _run(b, x)
    flat, flip, pad, s1, s2, g = ys
    assert torch.equal(flat, x.reshape(2, -1)) and torch.equal(flip, x.flip(3))
    assert torch.allclose(pad, F.pad(x, (2, 1, 1, 2), mode="reflect"))
    assert torch.equal(s1, x[:, :1]) and torch.equal(s2, x[:, 1:]) and torch.equal(g, x[:, [2, 0]])

    b11 = P.GraphBuilder("g", opset=11)
    b11.input("x")
    b11.node("Softmax", ["x"], ["y"], axis=1)  # opset < 13: softmax over the flattened trailing dims
    b11.output("y")
    _, y = _run(b11, x)
    assert torch.allclose(y, torch.softmax(x.reshape(2, -1), 1).reshape(x.shape), atol=1e-6)


@pytest.mark.parametrize("mode,ctm,nearest", [
    ("nearest", "asymmetric", "floor"), ("nearest", "half_pixel", "round_prefer_floor"),
    ("linear", "half_pixel", None), ("linear", "align_corners", None), ("linear", "asymmetric", None),
    ("cubic", "half_pixel", None)])
def test_resize_modes(mode, ctm, nearest):
    x = torch.randn(1, 2, 7, 9)
    b = P.GraphBuilder("g", opset=13)
    b.input("x")
    b.init("sc", torch.tensor([1.0, 1.0, 2.0, 2.0]))
    kw = dict(mode=mode, coordinate_transformation_mode=ctm)
    if nearest:
        kw["nearest_mode"] = nearest
    b.node("Resize", ["x", "", "sc"], ["y"], **kw)
    b.output("y")
    _, y = _run(b, x)
    assert y.shape == (1, 2, 14, 18)
    if mode == "nearest":
        ref = F.interpolate(x, scale_factor=2, mode="nearest")  # integer scales: every rule picks floor(o/2)
    elif ctm == "asymmetric":  # src = o / 2, edge-clamped: separable reference
        ref = x
        for d, L in ((2, 7), (3, 9)):
            src = torch.arange(2 * L, dtype=torch.float64) / 2
            i0 = src.floor().long()
            i1 = (i0 + 1).clamp(max=L - 1)
            w = (src - i0).float().view([-1 if k == d else 1 for k in range(4)])
            ref = ref.index_select(d, i0) * (1 - w) + ref.index_select(d, i1) * w
    else:
        im = "bilinear" if mode == "linear" else "bicubic"
        ref = F.interpolate(x, scale_factor=2, mode=im, align_corners=(ctm == "align_corners"))
    assert torch.allclose(y, ref, atol=1e-5)


def test_conv_auto_pad_and_asymmetric_pads():
    x = torch.randn(1, 3, 11, 10)
    w = torch.randn(4, 3, 3, 3)
    b = P.GraphBuilder("g", opset=13)
    b.input("x")
    b.init("w", w)
    b.node("Conv", ["x", "w"], ["a"], auto_pad="SAME_UPPER", strides=[2, 2])
    b.node("Conv", ["x", "w"], ["c"], pads=[0, 1, 2, 1])
    b.node("MaxPool", ["x"], ["m"], kernel_shape=[3, 3], strides=[2, 2], pads=[0, 0, 1, 1])
    for o in "acm":
        b.output(o)
    _, (a, c, m) = _run(b, x)
    # SAME_UPPER, stride 2 on 11x10: total pad 2/1 -> begin 1/0, end 1/1
    assert torch.allclose(a, F.conv2d(F.pad(x, (0, 1, 1, 1)), w, stride=2), atol=1e-5)
    assert torch.allclose(c, F.conv2d(F.pad(x, (1, 1, 0, 2)), w), atol=1e-5)
    assert torch.allclose(m, F.max_pool2d(F.pad(x, (0, 1, 0, 1), value=float("-inf")), 3, 2))


@pytest.mark.parametrize("norm,down", [("batch", "pool"), ("group", "conv"), ("instance", "pool")])
def test_export_and_execute_unet(tmp_path, norm, down):
    """fx exporter -> file -> OnnxModule reproduces the PyTorch U-Net (fp32, CPU), unoptimised and
    with the fusion pass (its Hip* modules run their CPU reference math here)."""
    from bioengine_worker_amd.bioimageio.convert import optimize_for_mi355x
    from bioengine_worker_amd.bioimageio.onnx_export import export_onnx

    p = write_unet2d_package(tmp_path / norm, f"onnx-{norm}", test_shape=(1, 1, 64, 64), torchscript=False,
                             norm=norm, down=down, features=(8, 16, 32, 64))
    import yaml

    kw = yaml.safe_load((p / "rdf.yaml").read_text())["weights"]["pytorch_state_dict"]["architecture"]["kwargs"]
    net = load_module(p / "model.py", f"onnx_{norm}_src").UNet2d(**kw).eval()
    net.load_state_dict(torch.load(p / "weights.pt", weights_only=True))
    info = export_onnx(net, tmp_path / "m.onnx")
    x = torch.randn(2, 1, 64, 80)
    with torch.no_grad():
        ref = net(x)
        y = OnnxModule.from_file(tmp_path / "m.onnx")(x)
        assert (y - ref).abs().max() < 1e-4
        mo = OnnxModule.from_file(tmp_path / "m.onnx", optimize=True)
        yo = mo(x)
    _, st_eager = optimize_for_mi355x(load_module(p / "model.py", f"onnx_{norm}_b").UNet2d(**kw).eval())
    assert mo.stats["convs"] == st_eager["convs"] and mo.stats["conv_transpose"] == st_eager["conv_transpose"]
    # dataflow-level fusion also catches norm -> conv pairs that straddle two nn.Sequential blocks
    assert mo.stats["strided"] == st_eager["strided"] and mo.stats["norm_fused"] >= st_eager["norm_fused"]
    assert mo.stats["bn_folded"] == st_eager["bn_folded"]
    assert (yo - ref).abs().max() < 1e-3  # CPU path of the fused modules: bf16-rounded weights
    assert info["opset"] == (21 if norm == "group" else 17)


def test_onnx_only_package_through_runner(tmp_path):
    from bioengine_worker_amd.bioimageio.runner import PredictionPipeline
    from bioengine_worker_amd.bioimageio.testing import test_model

    p = write_unet2d_package(tmp_path / "o", "onnx-only", test_shape=(1, 1, 64, 64), torchscript=False,
                             state_dict=False, onnx=True, features=(8, 16, 32, 64))
    pipe = PredictionPipeline(p, device="cpu")
    assert pipe.weights_format == "onnx" and not pipe.optimized
    y = pipe.predict(np.load(p / "test_input.npy"))["probabilities"]
    assert np.abs(y - np.load(p / "test_output.npy")).max() < 1e-4
    rep = test_model(p, device="cpu") if "device" in test_model.__code__.co_varnames else test_model(p)
    assert rep["status"] == "passed", rep


def test_both_formats_prefers_state_dict_and_onnx_selectable(tmp_path):
    from bioengine_worker_amd.bioimageio.runner import PredictionPipeline

    p = write_unet2d_package(tmp_path / "b", "onnx-both", test_shape=(1, 1, 64, 64), torchscript=False, onnx=True,
                             features=(8, 16, 32, 64))
    assert PredictionPipeline(p, device="cpu").weights_format == "pytorch_state_dict"
    pipe = PredictionPipeline(p, device="cpu", weights_format="onnx")
    y = pipe.predict(np.load(p / "test_input.npy"))["probabilities"]
    assert np.abs(y - np.load(p / "test_output.npy")).max() < 1e-3


@pytest.mark.gpu
def test_onnx_package_optimized_on_gpu(gpu, tmp_path):
    """ONNX-only U-Nets on the MI355X: the fusion pass puts every eligible conv on the MFMA kernel
    (BN folded, ReLU in the epilogue, GN/IN in the prologue, k2s2 transposed/strided convs) and the
    result matches the fp32 PyTorch model's test output at the bf16 tolerance."""
    from bioengine_worker_amd.bioimageio.runner import PredictionPipeline
    from bioengine_worker_amd.bioimageio.testing import test_model

    for norm, down in (("batch", "pool"), ("group", "conv")):
        p = write_unet2d_package(tmp_path / norm, f"gpu-onnx-{norm}", test_shape=(1, 1, 128, 128), torchscript=False,
                                 state_dict=False, onnx=True, norm=norm, down=down)
        pipe = PredictionPipeline(p, device=gpu)
        assert pipe.weights_format == "onnx" and pipe.optimized
        st = pipe.convert_stats
        if norm == "batch":
            assert st["convs"] == 15 and st["relu_fused"] == 14 and st["bn_folded"] == 14
        else:
            assert st["norm_fused"] >= 7 and st["strided"] == 3 and st["conv_transpose"] == 3
        y = pipe.predict(np.load(p / "test_input.npy"))["probabilities"]
        assert np.abs(y - np.load(p / "test_output.npy")).max() < 0.05
        rep = test_model(p)
        assert rep["status"] == "passed", rep
        assert rep["details"][2]["optimized"] is True
