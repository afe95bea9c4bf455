#!/usr/bin/env python3
"""Per-layer A/B: the linear-tile implicit-GEMM 3x3 conv (conv_igemm.hip) against the per-layer
pre-activation kernel (conv2d_nhwc.hip) on the headline CPnet's layer shapes (288 tiles of 224x224 =
one 32-image 512x512 batch).  HIP-event median of --reps launches, random data.  One JSON line per
(layer, kernel)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

SHAPES = [  # name, N, H, W, Cin, Cout
    ("L3 256->256 @28", 288, 28, 28, 256, 256),
    ("L2 128->128 @56", 288, 56, 56, 128, 128),
    ("L1 64->64 @112", 288, 112, 112, 64, 64),
    ("L0 32->32 @224 (bn64 pad)", 288, 224, 224, 32, 64),
]


def timeit(fn, reps):
    ts = []
    for r in range(reps + 3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        if r >= 3:
            ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--only", default="")
    ap.add_argument("--bns", default="64,128,65,1128,1065")
    ap.add_argument("--variants", default="plain,res+act")
    ap.add_argument("--no-ref", action="store_true", help="skip the per-layer reference kernel")
    a = ap.parse_args()
    from bioengine_worker_amd.ops import conv as convops
    from bioengine_worker_amd.ops import conv_igemm as ig

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for name, N, H, W, cin, cout in SHAPES:
        if a.only and a.only not in name:
            continue
        x = torch.randn(N, H, W, cin, device=dev, generator=g).to(torch.bfloat16)
        w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) / (9 * cin) ** 0.5
        b = 0.1 * torch.randn(cout, device=dev, generator=g)
        res = torch.randn(N, H, W, cout, device=dev, generator=g).to(torch.bfloat16)
        s = torch.ones(cout, device=dev)
        t = torch.zeros(cout, device=dev)
        flops = 2.0 * N * H * W * cin * cout * 9
        rows = []
        for bn in [int(v) for v in a.bns.split(",")]:
            if cout % (128 if bn % 1000 == 128 else 64) or not ig.supported(N, H, W, cout, bn):
                continue
            pk = ig.IgemmConv.from_weight(w, b, bn=bn).to(dev)
            out = torch.empty(N, H, W, cout, device=dev, dtype=torch.bfloat16)
            aout = torch.empty_like(out)
            for variant, kw in (("plain", {}), ("res+act", dict(residual=res, ascale=s, ashift=t, aout=aout))):
                if variant not in a.variants.split(","):
                    continue
                ms, mn = timeit(lambda: ig.conv3_igemm(x, pk, out=out, **kw), a.reps)
                rows.append(dict(layer=name, kernel=f"igemm bn{bn}", variant=variant, ms=round(ms, 4),
                                 min_ms=round(mn, 4), TFs=round(flops / ms / 1e9, 1)))
        if cin % 32 == 0 and not a.no_ref:
            pc = convops.PackedConv.from_weight(w, b).to(dev)
            sc = torch.ones(cin, device=dev)
            sh = torch.zeros(cin, device=dev)
            for variant, kw in (("plain", {}), ("res", dict(residual=res))):
                ms, mn = timeit(lambda: convops.fused_conv2d(x, pc, scale=sc, shift=sh, relu=True, **kw), a.reps)
                rows.append(dict(layer=name, kernel="conv2d_nhwc", variant=variant, ms=round(ms, 4), min_ms=round(mn, 4),
                                 TFs=round(flops / ms / 1e9, 1)))
        for r in rows:
            print(json.dumps(r), flush=True)
        del x, res


if __name__ == "__main__":
    main()
