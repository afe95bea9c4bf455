"""Run each CPnet conv layer shape a few times (for rocprofv3 --pmc counter collection)."""
import sys

import torch

sys.path.insert(0, ".")
from bioengine_worker_amd.ops.conv import PackedConv, fused_conv2d  # noqa: E402


def main():
    dev = torch.device("cuda")
    T = 288
    layers = [("L0", 3, 32, 32, 224, "none"), ("L1", 3, 64, 64, 112, "none"), ("L2", 3, 128, 128, 56, "none"),
              ("L3", 3, 256, 256, 28, "none"), ("U0", 3, 64, 32, 224, "up2"), ("P1", 3, 32, 64, 112, "pool2")]
    for name, ks, cin, cout, H, inmode in layers:
        Hs = {"none": H, "pool2": 2 * H, "up2": H // 2}[inmode]
        x = torch.randn(T, Hs, Hs, cin, device=dev).bfloat16()
        pc = PackedConv.from_weight(torch.randn(cout, cin, ks, ks) / (cin * ks * ks) ** 0.5, torch.zeros(cout)).to(dev)
        sc, sh = torch.ones(cin, device=dev), torch.zeros(cin, device=dev)
        for _ in range(3):
            fused_conv2d(x, pc, scale=sc, shift=sh, relu=True, inmode=inmode)
        torch.cuda.synchronize()
        print(name, "done", flush=True)


if __name__ == "__main__":
    main()
