#!/usr/bin/env python3
"""A/B of the CPnet inference engine with and without the fused two-conv kernels
(ops/conv_pair.py) at the headline batch (32 x 512^2 images = 288 tiles of 224^2), interleaved
rounds in ONE process (cdna_hip_programming.md §5.4 rule 24), plus per-call timings of each fused
half-block.  Prints JSON lines."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from bioengine_worker_amd.models.cpnet import CPnet, CPnetEngine  # noqa: E402
from bioengine_worker_amd.ops import conv_pair as cp  # noqa: E402


def timed(fn, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        ev[0].record()
        fn()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=288)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only-pairs", action="store_true", help="skip the engine A/B (profiling passes)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    net = CPnet().randomize_(0).eval()
    eng_pair = CPnetEngine(net, dev)
    os.environ["BE_CPNET_PAIR"] = "0"
    eng_layer = CPnetEngine(net, dev)
    os.environ["BE_CPNET_PAIR"] = "1"
    x = torch.randn(args.tiles, 224, 224, 8, device=dev).bfloat16()
    x[..., 2:] = 0
    res = {"pair": [], "layer": []}
    if args.only_pairs:
        args.rounds = 0
    with torch.no_grad():
        ya, _ = eng_pair(x)
        yb, _ = eng_layer(x)
    d = (ya - yb).abs().max().item()
    print(json.dumps({"check": "pair_vs_layer_max_abs", "value": d, "ref_max": yb.abs().max().item()}), flush=True)
    for r in range(args.rounds):
        for name, eng in (("pair", eng_pair), ("layer", eng_layer)):
            with torch.no_grad():
                med, mn = timed(lambda: eng(x), args.reps)
            res[name].append(med)
    for k, v in res.items():
        if not v:
            continue
        v.sort()
        print(json.dumps({"engine": k, "tiles": args.tiles, "ms_median": v[len(v) // 2], "ms_min": v[0],
                          "rounds": v}), flush=True)
    # per fused half-block (inputs of the right shapes, random)
    N = args.tiles
    P = eng_pair.pair
    shp = {("down", 0, 0): (224, 8, None, None), ("down", 0, 1): (224, 32, None, "full"),
           ("down", 1, 0): (224, 32, None, "full"), ("down", 1, 1): (112, 64, None, "full"),
           ("up", 1, 0): (56, 128, True, "up2"), ("up", 1, 1): (112, 64, None, "full"),
           ("up", 0, 0): (112, 64, True, "up2"), ("up", 0, 1): (224, 32, None, "full")}
    for key, (hs, cin, hx2, res) in shp.items():
        spec = P[key]
        xs = torch.randn(N, hs, hs, cin, device=dev).bfloat16()
        H, W = cp._out_hw(xs, spec.inmode)
        cm = spec.cm
        x2 = torch.randn(N, H, W, cm, device=dev).bfloat16() if hx2 else None
        rr = None
        if res == "full":
            rr = torch.randn(N, H, W, cm, device=dev).bfloat16()
        elif res == "up2":
            rr = torch.randn(N, H // 2, W // 2, cm, device=dev).bfloat16()
        ta = spec.ta if spec.ta is not None else None
        tb = spec.tb if spec.tb is not None else torch.zeros(N, cm, device=dev)
        if key[0] == "up" and key[2] == 1:
            ta = torch.zeros(N, cin, device=dev)
        out = torch.empty(N, H, W, cm, device=dev, dtype=torch.bfloat16)
        med, mn = timed(lambda: cp.conv_pair(xs, spec, ta=ta, tb=tb, x2=x2, res=rr, res_mode=res or "none", out=out),
                        args.reps * 2)
        px = N * H * W
        flop = 2 * px * 9 * cm * (cin + cm) * (612 / 512 if False else 1)
        byts = xs.numel() * 2 + out.numel() * 2 + (x2.numel() * 2 if x2 is not None else 0) + (rr.numel() * 2 if rr is not None else 0)
        print(json.dumps({"pair": "/".join(map(str, key)), "cin": cin, "cm": cm, "inmode": spec.inmode, "H": H,
                          "ms": round(med, 4), "ms_min": round(mn, 4), "TFLOPs": round(flop / med / 1e9, 1),
                          "min_bytes_GBs": round(byts / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
