"""Per-layer sweep of the fused conv kernel on the CPnet layer shapes at the bench's tile batch.

Prints achieved TF/s and GB/s per (layer, tco, nw) and the full-engine forward time.
Usage: python tools/conv_sweep.py [--tiles 288]
"""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from bioengine_worker_amd.ops.conv import PackedConv, fused_conv2d  # noqa: E402


def bench(fn, n=20):
    fn()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(True), torch.cuda.Event(True)
    ev0.record()
    for _ in range(n):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / n * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=288)
    a = ap.parse_args()
    dev = torch.device("cuda")
    T = a.tiles
    # (name, ks, cin, cout, H(out), inmode)
    layers = [("L0 3x3 32->32", 3, 32, 32, 224, "none"), ("L0 3x3 8->32", 3, 8, 32, 224, "none"),
              ("L1 3x3 64->64", 3, 64, 64, 112, "none"), ("L1 pool 32->64", 3, 32, 64, 112, "pool2"),
              ("L2 3x3 128->128", 3, 128, 128, 56, "none"), ("L3 3x3 256->256", 3, 256, 256, 28, "none"),
              ("U0 up 64->32", 3, 64, 32, 224, "up2"), ("L1 1x1 64->128", 1, 64, 128, 56, "pool2")]
    res = []
    for name, ks, cin, cout, H, inmode in layers:
        Hs = {"none": H, "pool2": 2 * H, "up2": H // 2}[inmode]
        x = torch.randn(T, Hs, Hs, cin, device=dev).bfloat16()
        w = torch.randn(cout, cin, ks, ks) / (cin * ks * ks) ** 0.5
        pc = PackedConv.from_weight(w, torch.zeros(cout)).to(dev)
        sc = torch.ones(cin, device=dev)
        sh = torch.zeros(cin, device=dev)
        flops = 2.0 * T * H * H * cout * cin * ks * ks
        byts = 2.0 * (x.numel() + T * H * H * cout)
        for nw in (4, 8):
            dt = bench(lambda: fused_conv2d(x, pc, scale=sc, shift=sh, relu=True, inmode=inmode, nw=nw))
            r = {"layer": name, "nw": nw, "tco": pc.tco, "ms": round(dt * 1e3, 3), "TFs": round(flops / dt / 1e12, 1),
                 "GBs": round(byts / dt / 1e9, 1)}
            res.append(r)
            print(json.dumps(r), flush=True)
    # engine forward
    from bioengine_worker_amd.models.cpnet import CPnet, CPnetEngine

    eng = CPnetEngine(CPnet().randomize_(0).eval(), dev)
    xin = torch.randn(T, 224, 224, 8, device=dev).bfloat16()
    for nw in (4, 8):
        import bioengine_worker_amd.ops.conv as cv

        cv.DEFAULT_NW = nw
        dt = bench(lambda: eng(xin), n=5)
        print(json.dumps({"engine_forward_tiles": T, "nw": nw, "ms": round(dt * 1e3, 2),
                          "ms_per_512img": round(dt * 1e3 / (T / 9), 3)}), flush=True)


if __name__ == "__main__":
    main()
