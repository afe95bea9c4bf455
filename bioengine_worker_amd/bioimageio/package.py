"""Self-contained bioimage.io demo model packages (offline model zoo, tests, bench).

``write_unet2d_package(dir)`` writes a complete RDF 0.5 package: ``model.py`` (a 2-D U-Net with
Conv-BN-ReLU blocks, max-pool encoder, transposed-conv decoder with skip concatenation, 1x1 head +
sigmoid — the architecture family of the zoo's nucleus-segmentation U-Nets such as
``affable-shark``), ``weights.pt`` (state dict, random init with non-trivial BN statistics),
``weights_torchscript.pt``, ``test_input.npy`` / ``test_output.npy`` (computed in fp32 on CPU),
``README.md`` and ``rdf.yaml``.
"""
from __future__ import annotations

import importlib.util
import textwrap
from pathlib import Path

import numpy as np
import torch
import yaml

from .spec import sha256_file

MODEL_SRC = textwrap.dedent('''
    import torch
    import torch.nn as nn


    def _norm(kind, c):
        if kind == "group":
            return nn.GroupNorm(min(8, c), c)
        if kind == "instance":
            return nn.InstanceNorm2d(c, affine=True)
        return nn.BatchNorm2d(c)


    def conv_block(cin, cout, norm="batch"):
        return nn.Sequential(
            nn.Conv2d(cin, cout, 3, padding=1), _norm(norm, cout), nn.ReLU(inplace=True),
            nn.Conv2d(cout, cout, 3, padding=1), _norm(norm, cout), nn.ReLU(inplace=True))


    class UNet2d(nn.Module):
        def __init__(self, in_channels=1, out_channels=2, features=(32, 64, 128, 256), final_activation="Sigmoid",
                     norm="batch", down="pool"):
            super().__init__()
            self.encoders = nn.ModuleList()
            self.downs = nn.ModuleList()
            c = in_channels
            for f in features[:-1]:
                self.encoders.append(conv_block(c, f, norm))
                # 2x2 max-pool, or a learned 2x2 stride-2 convolution
                self.downs.append(nn.MaxPool2d(2) if down == "pool" else nn.Conv2d(f, f, 2, stride=2))
                c = f
            self.base = conv_block(c, features[-1], norm)
            self.ups = nn.ModuleList()
            self.decoders = nn.ModuleList()
            c = features[-1]
            for f in reversed(features[:-1]):
                self.ups.append(nn.ConvTranspose2d(c, f, 2, stride=2))
                self.decoders.append(conv_block(2 * f, f, norm))
                c = f
            self.head = nn.Conv2d(c, out_channels, 1)
            self.act = getattr(nn, final_activation)() if final_activation else nn.Identity()

        def forward(self, x):
            skips = []
            for enc, down in zip(self.encoders, self.downs):
                x = enc(x)
                skips.append(x)
                x = down(x)
            x = self.base(x)
            for up, dec, s in zip(self.ups, self.decoders, reversed(skips)):
                x = dec(torch.cat([s, up(x)], dim=1))
            return self.act(self.head(x))
''')


MODEL3D_SRC = textwrap.dedent('''
    import torch
    import torch.nn as nn


    def conv_block(cin, cout):
        return nn.Sequential(
            nn.Conv3d(cin, cout, 3, padding=1), nn.BatchNorm3d(cout), nn.ReLU(inplace=True),
            nn.Conv3d(cout, cout, 3, padding=1), nn.BatchNorm3d(cout), nn.ReLU(inplace=True))


    class UNet3d(nn.Module):
        """3-D U-Net (PlantSeg / 3D-UNet family): Conv3d-BN-ReLU pairs, 2x max-pool, transposed-conv
        decoder with skip concatenation, 1x1x1 head + sigmoid."""

        def __init__(self, in_channels=1, out_channels=1, features=(16, 32, 64, 128), final_activation="Sigmoid"):
            super().__init__()
            self.encoders = nn.ModuleList()
            c = in_channels
            for f in features[:-1]:
                self.encoders.append(conv_block(c, f))
                c = f
            self.pool = nn.MaxPool3d(2)
            self.base = conv_block(c, features[-1])
            self.ups = nn.ModuleList()
            self.decoders = nn.ModuleList()
            c = features[-1]
            for f in reversed(features[:-1]):
                self.ups.append(nn.ConvTranspose3d(c, f, 2, stride=2))
                self.decoders.append(conv_block(2 * f, f))
                c = f
            self.head = nn.Conv3d(c, out_channels, 1)
            self.act = getattr(nn, final_activation)() if final_activation else nn.Identity()

        def forward(self, x):
            skips = []
            for enc in self.encoders:
                x = enc(x)
                skips.append(x)
                x = self.pool(x)
            x = self.base(x)
            for up, dec, s in zip(self.ups, self.decoders, reversed(skips)):
                x = dec(torch.cat([s, up(x)], dim=1))
            return self.act(self.head(x))
''')


def _randomize_bn(net: torch.nn.Module, seed: int) -> None:
    """Non-trivial eval statistics / affines so BN folding and GN/IN prologues are exercised."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for m in net.modules():
            if isinstance(m, (torch.nn.BatchNorm2d, torch.nn.BatchNorm3d)):
                m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.1)
                m.running_var.copy_(torch.rand(m.num_features, generator=g) * 0.5 + 0.75)
            if isinstance(m, (torch.nn.BatchNorm2d, torch.nn.BatchNorm3d, torch.nn.GroupNorm, torch.nn.InstanceNorm2d)) \
                    and m.weight is not None:
                m.weight.copy_(torch.rand(m.weight.shape[0], generator=g) * 0.5 + 0.75)
                m.bias.copy_(torch.randn(m.bias.shape[0], generator=g) * 0.1)


def load_module(path: Path, name: str = "bioimageio_model_src"):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def write_unet2d_package(out: str | Path, model_id: str = "demo-unet2d", in_channels: int = 1, out_channels: int = 2,
                         features=(32, 64, 128, 256), test_shape=(1, 1, 256, 256), seed: int = 0,
                         torchscript: bool = True, norm: str = "batch", down: str = "pool",
                         state_dict: bool = True, onnx: bool = False) -> Path:
    """``norm``: batch / group / instance; ``down``: pool / conv (2x2 stride-2); ``state_dict=False``
    writes a TorchScript-only package (the traced module is the only weights entry), or an ONNX-only
    one with ``onnx=True, torchscript=False``; ``onnx=True`` adds ``weights.onnx`` (own exporter)."""
    out = Path(out)
    out.mkdir(parents=True, exist_ok=True)
    (out / "model.py").write_text(MODEL_SRC)
    mod = load_module(out / "model.py", f"pkg_{model_id.replace('-', '_')}")
    kwargs = {"in_channels": in_channels, "out_channels": out_channels, "features": list(features),
              "final_activation": "Sigmoid", "norm": norm, "down": down}
    torch.manual_seed(seed)
    net = mod.UNet2d(**kwargs)
    _randomize_bn(net, seed)
    net.eval()
    torch.save(net.state_dict(), out / "weights.pt")
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:test_shape[2], 0:test_shape[3]]
    img = rng.normal(0, 0.2, test_shape).astype(np.float32)
    for _ in range(12):
        cy, cx, r = rng.uniform(20, test_shape[2] - 20), rng.uniform(20, test_shape[3] - 20), rng.uniform(6, 14)
        img[:, :, ((yy - cy) ** 2 + (xx - cx) ** 2) < r * r] += 1.0
    img = (img * 200 + 300).astype(np.float32)
    np.save(out / "test_input.npy", img)
    x = torch.from_numpy(img)
    x = (x - x.mean(dim=(2, 3), keepdim=True)) / (x.std(dim=(2, 3), keepdim=True, unbiased=False) + 1e-6)
    with torch.no_grad():
        y = net(x).numpy()
    np.save(out / "test_output.npy", y)
    weights = {"pytorch_state_dict": {
        "source": "weights.pt", "sha256": sha256_file(out / "weights.pt"),
        "architecture": {"source": "model.py", "sha256": sha256_file(out / "model.py"), "callable": "UNet2d",
                         "kwargs": kwargs},
        "pytorch_version": "2.5"}}
    if onnx:
        from .onnx_export import export_onnx

        info = export_onnx(net, out / "weights.onnx", input_name="raw", output_name="probabilities")
        weights["onnx"] = {"source": "weights.onnx", "sha256": sha256_file(out / "weights.onnx"),
                           "opset_version": info["opset"]}
        if state_dict:
            weights["onnx"]["parent"] = "pytorch_state_dict"
    if torchscript or (not state_dict and not onnx):
        ts = torch.jit.trace(net, x[:, :, :64, :64])
        ts.save(str(out / "weights_torchscript.pt"))
        weights["torchscript"] = {"source": "weights_torchscript.pt", "sha256": sha256_file(out / "weights_torchscript.pt"),
                                  "pytorch_version": "2.5"}
        if state_dict:
            weights["torchscript"]["parent"] = "pytorch_state_dict"
    if not state_dict:
        del weights["pytorch_state_dict"]
        (out / "weights.pt").unlink()
    (out / "README.md").write_text(f"# {model_id}\n\nDemo 2-D U-Net (random weights) for the MI355X model runner.\n")
    rdf = {
        "format_version": "0.5.3", "type": "model", "id": model_id, "name": f"Demo U-Net 2D ({model_id})",
        "description": "2-D U-Net nucleus segmentation demo package (random weights) for the bioengine-worker-amd model runner.",
        "authors": [{"name": "bioengine-worker-amd"}], "cite": [{"text": "Ronneberger et al. U-Net", "doi": "10.1007/978-3-319-24574-4_28"}],
        "license": "MIT", "documentation": "README.md", "tags": ["unet", "segmentation", "nuclei", "2d", "demo"],
        "inputs": [{"id": "raw", "axes": [
            {"type": "batch"}, {"type": "channel", "channel_names": [f"c{i}" for i in range(in_channels)]},
            {"type": "space", "id": "y", "size": {"min": 64, "step": 16}},
            {"type": "space", "id": "x", "size": {"min": 64, "step": 16}}],
            "test_tensor": {"source": "test_input.npy", "sha256": sha256_file(out / "test_input.npy")},
            "data": {"type": "float32"},
            "preprocessing": [{"id": "zero_mean_unit_variance", "kwargs": {"axes": ["y", "x"], "eps": 1e-6}}]}],
        "outputs": [{"id": "probabilities", "axes": [
            {"type": "batch"}, {"type": "channel", "channel_names": [f"p{i}" for i in range(out_channels)]},
            {"type": "space", "id": "y", "size": {"tensor_id": "raw", "axis_id": "y"}, "halo": 16},
            {"type": "space", "id": "x", "size": {"tensor_id": "raw", "axis_id": "x"}, "halo": 16}],
            "test_tensor": {"source": "test_output.npy", "sha256": sha256_file(out / "test_output.npy")},
            "data": {"type": "float32"}}],
        "weights": weights,
        "config": {"bioimageio": {"reproducibility_tolerance": [{"relative_tolerance": 1e-3, "absolute_tolerance": 1e-4}]}},
    }
    (out / "rdf.yaml").write_text(yaml.safe_dump(rdf, sort_keys=False))
    return out


def write_unet3d_package(out: str | Path, model_id: str = "demo-unet3d", in_channels: int = 1, out_channels: int = 1,
                         features=(16, 32, 64, 128), test_shape=(1, 1, 32, 64, 64), seed: int = 0) -> Path:
    """RDF 0.5 package of a 3-D U-Net (axes b, c, z, y, x) — the 3-D model-runner / volume path."""
    out = Path(out)
    out.mkdir(parents=True, exist_ok=True)
    (out / "model.py").write_text(MODEL3D_SRC)
    mod = load_module(out / "model.py", f"pkg3d_{model_id.replace('-', '_')}")
    kwargs = {"in_channels": in_channels, "out_channels": out_channels, "features": list(features),
              "final_activation": "Sigmoid"}
    torch.manual_seed(seed)
    net = mod.UNet3d(**kwargs)
    _randomize_bn(net, seed)
    net.eval()
    torch.save(net.state_dict(), out / "weights.pt")
    rng = np.random.default_rng(seed)
    zz, yy, xx = np.mgrid[0:test_shape[2], 0:test_shape[3], 0:test_shape[4]]
    img = rng.normal(0, 0.2, test_shape).astype(np.float32)
    for _ in range(10):
        c = [rng.uniform(4, n - 4) for n in test_shape[2:]]
        r = rng.uniform(3, 8)
        img[:, :, ((zz - c[0]) ** 2 + (yy - c[1]) ** 2 + (xx - c[2]) ** 2) < r * r] += 1.0
    img = (img * 200 + 300).astype(np.float32)
    np.save(out / "test_input.npy", img)
    x = torch.from_numpy(img)
    x = (x - x.mean(dim=(2, 3, 4), keepdim=True)) / (x.std(dim=(2, 3, 4), keepdim=True, unbiased=False) + 1e-6)
    with torch.no_grad():
        y = net(x).numpy()
    np.save(out / "test_output.npy", y)
    (out / "README.md").write_text(f"# {model_id}\n\nDemo 3-D U-Net (random weights) for the MI355X model runner.\n")
    space = lambda a: {"type": "space", "id": a, "size": {"min": 16, "step": 8}}  # noqa: E731
    same = lambda a: {"type": "space", "id": a, "size": {"tensor_id": "raw", "axis_id": a}, "halo": 4}  # noqa: E731
    rdf = {
        "format_version": "0.5.3", "type": "model", "id": model_id, "name": f"Demo U-Net 3D ({model_id})",
        "description": "3-D U-Net volume segmentation demo package (random weights) for the bioengine-worker-amd model runner.",
        "authors": [{"name": "bioengine-worker-amd"}],
        "cite": [{"text": "Cicek et al. 3D U-Net", "doi": "10.1007/978-3-319-46723-8_49"}],
        "license": "MIT", "documentation": "README.md", "tags": ["unet", "segmentation", "3d", "demo"],
        "inputs": [{"id": "raw", "axes": [
            {"type": "batch"}, {"type": "channel", "channel_names": [f"c{i}" for i in range(in_channels)]},
            space("z"), space("y"), space("x")],
            "test_tensor": {"source": "test_input.npy", "sha256": sha256_file(out / "test_input.npy")},
            "data": {"type": "float32"},
            "preprocessing": [{"id": "zero_mean_unit_variance", "kwargs": {"axes": ["z", "y", "x"], "eps": 1e-6}}]}],
        "outputs": [{"id": "probabilities", "axes": [
            {"type": "batch"}, {"type": "channel", "channel_names": [f"p{i}" for i in range(out_channels)]},
            same("z"), same("y"), same("x")],
            "test_tensor": {"source": "test_output.npy", "sha256": sha256_file(out / "test_output.npy")},
            "data": {"type": "float32"}}],
        "weights": {"pytorch_state_dict": {
            "source": "weights.pt", "sha256": sha256_file(out / "weights.pt"),
            "architecture": {"source": "model.py", "sha256": sha256_file(out / "model.py"), "callable": "UNet3d",
                             "kwargs": kwargs},
            "pytorch_version": "2.5"}},
        "config": {"bioimageio": {"reproducibility_tolerance": [{"relative_tolerance": 1e-3, "absolute_tolerance": 1e-4}]}},
    }
    (out / "rdf.yaml").write_text(yaml.safe_dump(rdf, sort_keys=False))
    return out
