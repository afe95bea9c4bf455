"""Model-runner U-Net (bioimage.io 2-D U-Net, Conv-BN-ReLU x2 blocks, features 32-256) throughput:
MI355X graph pass (fused NHWC MFMA convs, bf16 channels-last) vs the same network in PyTorch
(fp32 and bf16 channels-last on MIOpen)."""
import copy
import json
import sys
import tempfile
import time

import torch

sys.path.insert(0, ".")
from bioengine_worker_amd.bioimageio.convert import optimize_for_mi355x  # noqa: E402
from bioengine_worker_amd.bioimageio.package import load_module, write_unet2d_package, write_unet3d_package  # noqa: E402


def bench(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def main():
    dev = torch.device("cuda")
    d = write_unet2d_package(tempfile.mkdtemp() + "/u", torchscript=False, test_shape=(1, 1, 64, 64))
    mod = load_module(d / "model.py")
    net = mod.UNet2d(in_channels=1, out_channels=2, features=[32, 64, 128, 256]).eval().to(dev)
    net.load_state_dict(torch.load(d / "weights.pt", weights_only=True))
    for B, S in ((16, 512), (4, 1024)):
        x = torch.randn(B, 1, S, S, device=dev)
        with torch.no_grad():
            t32 = bench(lambda: net(x))
            nb = copy.deepcopy(net).to(torch.bfloat16).to(memory_format=torch.channels_last)
            xb = x.bfloat16().contiguous(memory_format=torch.channels_last)
            tb = bench(lambda: nb(xb))
            opt, st = optimize_for_mi355x(copy.deepcopy(net), dev)
            to = bench(lambda: opt(xb))
        print(json.dumps({"unet2d": [B, S, S], "mpix_per_s_mi355x": round(B * S * S / to / 1e6, 1),
                          "ms_mi355x": round(to * 1e3, 2), "ms_torch_fp32": round(t32 * 1e3, 2),
                          "ms_torch_bf16_cl": round(tb * 1e3, 2), "speedup_vs_fp32": round(t32 / to, 2),
                          "speedup_vs_bf16": round(tb / to, 2), "convert": st}), flush=True)

    d3 = write_unet3d_package(tempfile.mkdtemp() + "/u3", test_shape=(1, 1, 16, 32, 32))
    mod3 = load_module(d3 / "model.py", "unet3d_bench")
    net3 = mod3.UNet3d(in_channels=1, out_channels=1, features=[16, 32, 64, 128]).eval().to(dev)
    net3.load_state_dict(torch.load(d3 / "weights.pt", weights_only=True))
    for B, D, S in ((1, 64, 256), (2, 96, 160)):
        x = torch.randn(B, 1, D, S, S, device=dev)
        with torch.no_grad():
            t32 = bench(lambda: net3(x), n=5)
            nb = copy.deepcopy(net3).to(torch.bfloat16).to(memory_format=torch.channels_last_3d)
            xb = x.bfloat16().contiguous(memory_format=torch.channels_last_3d)
            tb = bench(lambda: nb(xb), n=5)
            nb3 = copy.deepcopy(net3).to(torch.bfloat16)
            xb3 = x.bfloat16()
            tb3 = bench(lambda: nb3(xb3), n=5)
            opt, st = optimize_for_mi355x(copy.deepcopy(net3), dev)
            to = bench(lambda: opt(xb), n=5)
            err = (opt(xb).float() - net3(x)).abs().max().item()
        print(json.dumps({"unet3d": [B, D, S, S], "mvox_per_s_mi355x": round(B * D * S * S / to / 1e6, 1),
                          "ms_mi355x": round(to * 1e3, 2), "ms_torch_fp32": round(t32 * 1e3, 2),
                          "ms_torch_bf16_cl3d": round(tb * 1e3, 2), "ms_torch_bf16_ncdhw": round(tb3 * 1e3, 2),
                          "speedup_vs_fp32": round(t32 / to, 2),
                          "speedup_vs_best_bf16": round(min(tb, tb3) / to, 2), "max_abs_err_vs_fp32": round(err, 4),
                          "convert": st}), flush=True)


if __name__ == "__main__":
    main()
