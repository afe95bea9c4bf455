#!/usr/bin/env python3
"""Ping-pong GEMM (csrc/kernels/gemm_pp.hip) A/B, HIP-event median of --reps launches, random data.

* GEMM: the CPSAM ViT-L training forward shapes at batch 8 (M = 8,192 tokens) and square 4096 /
  8192, against PyTorch's hipBLASLt call and the in-house two-barrier kernel (gemm_bf16 cfg 0).
* CONV: the headline CPnet's deep 3x3 layers (288 tiles of 224^2 = one 32-image 512^2 batch)
  against the per-layer pre-activation kernel (conv2d_nhwc) and the round-4 igemm kernel.
One JSON line per (case, impl)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


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
    return ts[len(ts) // 2]


def emit(**kw):
    print(json.dumps(kw), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cfgs", default="0,1,2")
    ap.add_argument("--what", default="gemm,conv")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    from bioengine_worker_amd.ops import gemm_bf16 as gb
    from bioengine_worker_amd.ops import gemm_pp as pp

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    cfgs = [int(c) for c in a.cfgs.split(",")]
    if "gemm" in a.what:
        cases = [("qkv b8", 8192, 3072, 1024), ("proj b8", 8192, 1024, 1024), ("lin1 b8", 8192, 4096, 1024),
                 ("lin2 b8", 8192, 1024, 4096), ("sq4096", 4096, 4096, 4096), ("sq8192", 8192, 8192, 8192)]
        for name, M, N, K in cases:
            if a.only and a.only not in name:
                continue
            x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
            b = torch.randn(N, device=dev, generator=g)
            bh = b.to(torch.bfloat16)
            fl = 2.0 * M * N * K
            ms = timeit(lambda: F.linear(x, w, bh), a.reps)
            emit(case=name, impl="torch", ms=round(ms, 4), TFs=round(fl / ms / 1e9, 1))
            ms = timeit(lambda: gb._call(x, w, torch.empty(M, N, device=dev, dtype=torch.bfloat16), M, N, K, K, K, N,
                                         0, 0, gb.E_BIAS, bias=b, cfg=0), a.reps)
            emit(case=name, impl="gemm_bf16 cfg0", ms=round(ms, 4), TFs=round(fl / ms / 1e9, 1))
            for c in cfgs:
                ms = timeit(lambda: pp.linear(x, w, b, cfg=c), a.reps)
                emit(case=name, impl=f"pp cfg{c}", ms=round(ms, 4), TFs=round(fl / ms / 1e9, 1))
            del x, w
        dcases = [("dgrad qkv b8", 8192, 1024, 3072, False), ("dgrad lin1 b8", 8192, 1024, 4096, False),
                  ("dgrad proj b8", 8192, 1024, 1024, False), ("dgrad lin2+dgelu b8", 8192, 4096, 1024, True)]
        for name, M, N, K, dg in dcases:
            if a.only and a.only not in name:
                continue
            dy = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
            w = (torch.randn(K, N, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
            f = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
            db = torch.empty(N, device=dev)
            fl = 2.0 * M * N * K
            if dg:
                from bioengine_worker_amd.ops import vit_train as vt

                zero = torch.zeros(N, device=dev)
                ms = timeit(lambda: vt.gelu_bwd(torch.mm(dy, w), f, zero, out_db=db), a.reps)
            else:
                ms = timeit(lambda: torch.mm(dy, w), a.reps)
            emit(case=name, impl="torch", ms=round(ms, 4), TFs=round(fl / ms / 1e9, 1))
            for c in cfgs:
                if N % pp.TILES[c][1]:
                    continue
                fn = (lambda: pp.mm_dgelu(dy, w, f, out_db=db, cfg=c)) if dg else (lambda: pp.mm(dy, w, cfg=c))
                ms = timeit(fn, a.reps)
                emit(case=name, impl=f"pp cfg{c}", ms=round(ms, 4), TFs=round(fl / ms / 1e9, 1))
            del dy, w, f
        wcases = [("wgrad qkv b8", 8192, 3072, 1024), ("wgrad proj b8", 8192, 1024, 1024),
                  ("wgrad lin1 b8", 8192, 4096, 1024), ("wgrad lin2 b8", 8192, 1024, 4096),
                  ("wgrad qkv b1", 1024, 3072, 1024), ("wgrad lin1 b1", 1024, 4096, 1024)]
        for name, m, n, k in wcases:
            if a.only and a.only not in name:
                continue
            dy = torch.randn(m, n, device=dev, generator=g).to(torch.bfloat16)
            x = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
            out = torch.empty(n, k, device=dev)
            fl = 2.0 * m * n * k
            ms = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32, out=out), a.reps)
            emit(case=name, impl="torch", ms=round(ms, 4), TFs=round(fl / ms / 1e9, 1))
            ms = timeit(lambda: gb.wgrad(dy, x, out), a.reps)
            emit(case=name, impl="gemm_bf16", ms=round(ms, 4), TFs=round(fl / ms / 1e9, 1))
            for c in cfgs:
                bm, bn = pp.TILES[c]
                if n % bm or k % bn:
                    continue
                ms = timeit(lambda: pp.wgrad(dy, x, out, cfg=c), a.reps)
                emit(case=name, impl=f"pp cfg{c}", split=pp.wgrad_split(n, k, m, c), ms=round(ms, 4),
                     TFs=round(fl / ms / 1e9, 1))
            del dy, x, out
    if "conv" in a.what:
        from bioengine_worker_amd.ops import conv as convops
        from bioengine_worker_amd.ops import conv_igemm as ig

        shapes = [("L3 256->256 @28", 288, 28, 28, 256, 256), ("L2 128->128 @56", 288, 56, 56, 128, 128),
                  ("L3in 128->256 @28", 288, 28, 28, 128, 256), ("L2up 256->128 @56", 288, 56, 56, 256, 128),
                  ("L1 64->64 @112", 288, 112, 112, 64, 64)]
        for name, N, H, W, cin, cout in shapes:
            if a.only and a.only not in name:
                continue
            x = torch.randn(N, H, W, cin, device=dev, generator=g).to(torch.bfloat16)
            w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) / (9 * cin) ** 0.5
            b = 0.1 * torch.randn(cout, device=dev, generator=g)
            res = torch.randn(N, H, W, cout, device=dev, generator=g).to(torch.bfloat16)
            s = torch.ones(cout, device=dev)
            t = torch.zeros(cout, device=dev)
            fl = 2.0 * N * H * W * cin * cout * 9
            wp = pp.pack_conv3(w)
            out = torch.empty(N, H, W, cout, device=dev, dtype=torch.bfloat16)
            aout = torch.empty_like(out)
            for c in cfgs:
                for variant, kw in (("plain", {}), ("res+act", dict(residual=res, ascale=s, ashift=t, aout=aout))):
                    ms = timeit(lambda: pp.conv3(x, wp, b, out=out, cfg=c, **kw), a.reps)
                    emit(case=name, impl=f"pp cfg{c}", variant=variant, ms=round(ms, 4), TFs=round(fl / ms / 1e9, 1))
            pc = convops.PackedConv.from_weight(w, b).to(dev)
            sc, shf = torch.ones(cin, device=dev), torch.zeros(cin, device=dev)
            for variant, kw in (("plain", {}), ("res", dict(residual=res))):
                ms = timeit(lambda: convops.fused_conv2d(x, pc, scale=sc, shift=shf, relu=True, **kw), a.reps)
                emit(case=name, impl="conv2d_nhwc", variant=variant, ms=round(ms, 4), TFs=round(fl / ms / 1e9, 1))
            if cout % 64 == 0 and cin % 16 == 0 and ig.supported(N, H, W, cout, 1065):
                pk = ig.IgemmConv.from_weight(w, b, bn=1065).to(dev)
                ms = timeit(lambda: ig.conv3_igemm(x, pk, out=out), a.reps)
                emit(case=name, impl="igemm bn1065", variant="plain", ms=round(ms, 4), TFs=round(fl / ms / 1e9, 1))
            del x, res, out, aout


if __name__ == "__main__":
    main()
