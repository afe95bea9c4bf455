#!/usr/bin/env python3
"""Cellpose-SAM inference linears at the bench's batch (8 images x 9 tiles x 1024 tokens = 73,728
rows): hipBLASLt (F.linear, + the separate bias+GELU pass for lin1) vs the in-house GEMMs with the
bias / bias+GELU epilogue fused (gemm_8p, gemm_mt).  Graph-replayed, interleaved, median us."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from bioengine_worker_amd.ops import gemm_8p, gemm_mt
from bioengine_worker_amd.ops.transformer import bias_gelu_
from tools.gemm_8p_bench import graph_of

DEV = torch.device("cuda", 0)
ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=73728)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--rounds", type=int, default=7)
a = ap.parse_args()
g = torch.Generator().manual_seed(0)
M = a.M
for name, N, K, gelu in (("qkv", 3072, 1024, False), ("proj", 1024, 1024, False), ("lin1", 4096, 1024, True),
                         ("lin2", 1024, 4096, False)):
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.03).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV)
    bb = b.to(torch.bfloat16)
    if gelu:
        arms = {"lib": lambda: bias_gelu_(F.linear(x, w), b), "8p": lambda: gemm_8p.linear_gelu_only(x, w, b),
                "mt": lambda: gemm_mt.linear_gelu_only(x, w, b)}
    else:
        arms = {"lib": lambda: F.linear(x, w, bb), "8p": lambda: gemm_8p.linear(x, w, bb),
                "mt": lambda: gemm_mt.linear(x, w, bb)}
    ref = arms["lib"]().float()
    for k, fn in arms.items():
        err = ((fn().float() - ref).abs().max() / ref.abs().max()).item()
        assert err < 3e-2, (name, k, err)
    graphs = {k: graph_of(fn, a.reps) for k, fn in arms.items()}
    times = {k: [] for k in arms}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for k, gr in graphs.items():
            e0.record()
            gr.replay()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) * 1e3 / a.reps)
    for k, t in times.items():
        us = statistics.median(t)
        print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "impl": k, "us": round(us, 1),
                          "TFs": round(2.0 * M * N * K / us / 1e6, 1)}), flush=True)
    del graphs
    torch.cuda.empty_cache()
