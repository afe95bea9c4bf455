"""Sweep persistent-grid size and nw for the fused conv on CPnet layer shapes (288 tiles)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from bioengine_worker_amd.ops import _native  # noqa: E402
from bioengine_worker_amd.ops.conv import PackedConv, fused_conv2d  # noqa: E402
from tools.conv_sweep import bench  # noqa: E402


def main():
    dev = torch.device("cuda")
    T = 288
    layers = [("L0 3x3 32->32", 3, 32, 32, 224, "none"), ("L1 3x3 64->64", 3, 64, 64, 112, "none"),
              ("L2 3x3 128->128", 3, 128, 128, 56, "none"), ("L3 3x3 256->256", 3, 256, 256, 28, "none"),
              ("U0 up 64->32", 3, 64, 32, 224, "up2"), ("L1 pool 32->64", 3, 32, 64, 112, "pool2"),
              ("L0 3x3 8->32", 3, 8, 32, 224, "none"), ("L2 up 256->128", 3, 256, 128, 56, "up2")]
    for name, ks, cin, cout, H, inmode in layers:
        Hs = {"none": H, "pool2": 2 * H, "up2": H // 2}[inmode]
        x = torch.randn(T, Hs, Hs, cin, device=dev).bfloat16()
        w = torch.randn(cout, cin, ks, ks) / (cin * ks * ks) ** 0.5
        pc = PackedConv.from_weight(w, torch.zeros(cout)).to(dev)
        sc, sh = torch.ones(cin, device=dev), torch.zeros(cin, device=dev)
        flops = 2.0 * T * H * H * cout * cin * ks * ks
        byts = 2.0 * (x.numel() + T * H * H * cout)
        for nw in (4, 8):
            for pb in ((0, 512, 1024, 2048) if pc.tco <= 32 else (0,)):
                _native.call("be_conv2d_set_persist", pb)
                dt = bench(lambda: fused_conv2d(x, pc, scale=sc, shift=sh, relu=True, inmode=inmode, nw=nw))
                print(json.dumps({"layer": name, "nw": nw, "persist": pb, "ms": round(dt * 1e3, 3),
                                  "TFs": round(flops / dt / 1e12, 1), "GBs": round(byts / dt / 1e9, 1)}), flush=True)
    _native.call("be_conv2d_set_persist", 0)
    from bioengine_worker_amd.models.cpnet import CPnet, CPnetEngine
    import bioengine_worker_amd.ops.conv as cv

    eng = CPnetEngine(CPnet().randomize_(0).eval(), dev)
    xin = torch.randn(T, 224, 224, 8, device=dev).bfloat16()
    for nw in (None, 4, 8):
        cv.DEFAULT_NW = nw
        dt = bench(lambda: eng(xin), n=5)
        print(json.dumps({"engine_forward_tiles": T, "nw": nw, "ms": round(dt * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
