#!/usr/bin/env python3
"""gemm_8p (two-group ping-pong 256x256) vs gemm_mt (static table) vs hipBLASLt (F.linear) on the
Cellpose-SAM forward GEMMs, graph-replayed and interleaved in one process (tools/gemm_mt_bench.py
method), after a correctness check of every shape against an fp32 matmul."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from bioengine_worker_amd.ops import gemm_8p, gemm_mt

DEV = torch.device("cuda", 0)


def graph_of(fn, reps):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    return g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--shapes", default="8192x3072x1024,8192x4096x1024,8192x1024x4096,8192x1024x1024,"
                                        "1024x3072x1024,1024x4096x1024,4096x4096x4096")
    args = ap.parse_args()
    g = torch.Generator(device="cpu").manual_seed(0)
    # correctness incl. ragged M / N and every epilogue
    for M, N, K in ((300, 200, 128), (8192, 3072, 1024), (1000, 1028, 256)):
        x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
        w = (torch.randn(N, K, generator=g) * 0.05).to(DEV, torch.bfloat16)
        b = torch.randn(N, generator=g).to(DEV)
        r = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
        ref = x.float() @ w.float().t() + b
        outs = {"bias": gemm_8p.linear(x, w, b).float(), "res": gemm_8p.linear_res(x, w, b, r).float() - r.float()}
        gg, f = gemm_8p.linear_gelu(x, w, b)
        outs["gelu_f"] = f.float()
        for k, v in outs.items():
            err = ((v - ref).abs().max() / ref.abs().max()).item()
            print(json.dumps({"check": k, "M": M, "N": N, "K": K, "rel_err": round(err, 5)}), flush=True)
            assert err < 2e-2, (k, M, N, K, err)
        gerr = (gg.float() - F.gelu(f.float())).abs().max().item()
        assert gerr < 2e-2, gerr
    for s in args.shapes.split(","):
        M, N, K = (int(v) for v in s.split("x"))
        flops = 2.0 * M * N * K
        x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
        w = (torch.randn(N, K, generator=g) * 0.03).to(DEV, torch.bfloat16)
        b = torch.randn(N, generator=g).to(DEV)
        arms = {"lib": lambda: F.linear(x, w, b.to(torch.bfloat16)), "mt": lambda: gemm_mt.linear(x, w, b),
                "8p": lambda: gemm_8p.linear(x, w, b)}
        graphs = {k: graph_of(fn, args.reps) for k, fn in arms.items()}
        times = {k: [] for k in arms}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(args.rounds):
            for k, gr in graphs.items():
                e0.record()
                gr.replay()
                e1.record()
                e1.synchronize()
                times[k].append(e0.elapsed_time(e1) * 1e3 / args.reps)
        for k, t in times.items():
            us = statistics.median(t)
            print(json.dumps({"M": M, "N": N, "K": K, "impl": k, "us": round(us, 2), "us_min": round(min(t), 2),
                              "TFs": round(flops / us / 1e6, 1)}), flush=True)
        del graphs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
