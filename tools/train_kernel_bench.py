#!/usr/bin/env python3
"""Per-kernel timing of the training kernels on the fine-tune bench's largest shapes (HIP events).

    python tools/train_kernel_bench.py [--B 8] [--H 256] [--C 32]
Prints one JSON line per kernel with us/call and effective GB/s or TFLOP/s."""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--H", type=int, default=256)
    ap.add_argument("--C", type=int, default=32)
    args = ap.parse_args()
    from bioengine_worker_amd.ops import conv as convops
    from bioengine_worker_amd.ops import conv_train as ct

    dev = torch.device("cuda", 0)
    B, H, C = args.B, args.H, args.C
    x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
    dA = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
    dx = torch.empty_like(x)
    nbytes = x.numel() * 2
    tag = {"B": B, "H": H, "C": C, "env": {k: v for k, v in os.environ.items() if k.startswith("BE_")}}

    def mk(nunits):
        units = [ct.BnUnit(gamma=torch.ones(C, device=dev), beta=torch.zeros(C, device=dev), run_mean=None,
                           run_var=None, relu=True, scale=torch.ones(C, device=dev), shift=torch.zeros(B, C, device=dev),
                           dgamma=torch.zeros(C, device=dev), dbeta=torch.zeros(C, device=dev)) for _ in range(nunits)]
        stat = torch.zeros(ct.BnSite.stat_numel(B, C), device=dev)
        tk = torch.zeros(2, dtype=torch.int32, device=dev)
        return ct.BnSite(B, C, C, units, stat, tk), stat, tk

    s, stat, tk = mk(1)

    def stats():
        stat.zero_()
        s.stats(x)

    us = timeit(stats)
    print(json.dumps({"k": "bn_stats(+zero)", "us": round(us, 1), "GBs": round(nbytes / us / 1e3, 1), **tag}))
    s.stats(x)

    def red():
        tk.zero_()
        s.bwd_reduce(x, [dA])

    us = timeit(red)
    print(json.dumps({"k": "bn_bwd_reduce", "us": round(us, 1), "GBs": round(2 * nbytes / us / 1e3, 1), **tag}))
    us = timeit(lambda: s.bwd_apply(x, [dA], dx=dx, dx_acc=True))
    print(json.dumps({"k": "bn_bwd_apply(acc)", "us": round(us, 1), "GBs": round(4 * nbytes / us / 1e3, 1), **tag}))
    dw = torch.zeros(C, C, 3, 3, device=dev)
    db = torch.zeros(C, device=dev)
    sc = torch.ones(C, device=dev)
    sh = torch.zeros(B, C, device=dev)
    for sp in (None, 64, 128, 256, 1024):
        us = timeit(lambda: ct.conv_wgrad(x, dA, ks=3, cin_valid=C, cout_valid=C, dw=dw, db=db, scale=sc, shift=sh,
                                          relu=True, splits=sp))
        fl = 2.0 * B * H * H * 9 * C * C
        print(json.dumps({"k": "wgrad3x3(+reduce)", "splits": sp or ct.wgrad_splits(B, H, H, C, C, 3), "us": round(us, 1),
                          "TFs": round(fl / us / 1e6, 1), **tag}))
    pc = convops.PackedConv.from_weight(torch.randn(C, C, 3, 3)).to(dev)
    us = timeit(lambda: convops.fused_conv2d(x, pc, scale=sc, shift=sh, relu=True))
    print(json.dumps({"k": "conv3x3 fwd", "us": round(us, 1), "TFs": round(2.0 * B * H * H * 9 * C * C / us / 1e6, 1), **tag}))


if __name__ == "__main__":
    main()
