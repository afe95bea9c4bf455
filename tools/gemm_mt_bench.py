#!/usr/bin/env python3
"""Per-shape sweep of the macro-tile GEMM (csrc/kernels/gemm_mt.hip) against the library GEMM that the
Cellpose-SAM engine used before (hipBLASLt through PyTorch: F.linear / torch.mm / the engine's
split-K weight gradient), on the 12 GEMMs of one ViT-L block at batch 1 and 8.

Timing: each candidate runs as a captured HIP graph of R back-to-back calls, replayed several times
(the GPU time of the kernels, not the host launch path), interleaved round-robin over candidates in
one process.  One JSON line per (shape, candidate) with the median us and TF/s; --table prints the
static table entries (fastest in-house candidate per shape) for ops/gemm_mt.py."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from bioengine_worker_amd.ops import gemm_mt
from bioengine_worker_amd.train import cpsam_engine

DEV = torch.device("cuda", 0)


def shapes(B: int):
    M = 1024 * B
    out = []
    for name, N, K in (("qkv", 3072, 1024), ("proj", 1024, 1024), ("lin1", 4096, 1024), ("lin2", 1024, 4096)):
        out.append(("nt", f"{name} fwd b{B}", M, N, K))
        out.append(("nn", f"{name} dgrad b{B}", M, K, N))     # dy [M, N] @ W [N, K]
        out.append(("tn", f"{name} wgrad b{B}", N, K, M))     # dW [N, K] = dy^T x over M tokens
    return out


def candidates(kind, M, N, K):
    c = []
    for cfg in (0, 1, 2, 3, 4):
        if not gemm_mt._valid(kind, cfg, M, N):
            continue
        if kind == "tn":
            bm, bn = gemm_mt.TILES[cfg]
            tiles = (M // bm) * (N // bn)
            for split in (1, 2, 3, 4, 5, 6, 8, 12, 16):
                if tiles * split <= 2 * 256 and (K // 64) // split >= 4:
                    c.append((cfg, split))
        else:
            c.append((cfg, 1))
    return c


def make_fn(kind, M, N, K, impl):
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    if kind == "nt":
        x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
        w = (torch.randn(N, K, generator=g) * 0.03).to(DEV, torch.bfloat16)
        b = torch.randn(N, generator=g).to(DEV)
        if impl == "lib":
            return lambda: F.linear(x, w, b.to(torch.bfloat16))
        return lambda: gemm_mt.linear(x, w, b)
    if kind == "nn":
        x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
        w = (torch.randn(K, N, generator=g) * 0.03).to(DEV, torch.bfloat16)
        if impl == "lib":
            return lambda: torch.mm(x, w)
        return lambda: gemm_mt.mm(x, w)
    dy = torch.randn(K, M, generator=g).to(DEV, torch.bfloat16)
    x = torch.randn(K, N, generator=g).to(DEV, torch.bfloat16)
    out = torch.empty(M, N, device=DEV)
    if impl == "lib":
        return lambda: cpsam_engine._wgrad(dy, x, out)
    return lambda: gemm_mt.wgrad(dy, x, out)


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
    ap.add_argument("--batches", default="8,1")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--only", default="")
    ap.add_argument("--table", action="store_true")
    args = ap.parse_args()
    best = {}
    for B in [int(b) for b in args.batches.split(",")]:
        for kind, name, M, N, K in shapes(B):
            if args.only and args.only not in name:
                continue
            flops = 2.0 * M * N * K
            arms = [("lib", None)] + [("mt", c) for c in candidates(kind, M, N, K)]
            graphs = []
            for impl, c in arms:
                if c is not None:
                    os.environ["BE_GEMM_MT_CFG"] = f"{c[0]},{c[1]}"
                else:
                    os.environ.pop("BE_GEMM_MT_CFG", None)
                try:
                    graphs.append(graph_of(make_fn(kind, M, N, K, impl), args.reps))
                except Exception as e:  # noqa: BLE001
                    graphs.append(None)
                    print(json.dumps({"case": name, "impl": impl, "cfg": c, "error": str(e)[:200]}), flush=True)
            os.environ.pop("BE_GEMM_MT_CFG", None)
            times = [[] for _ in arms]
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(args.rounds):
                for i, g in enumerate(graphs):
                    if g is None:
                        continue
                    ev0.record()
                    g.replay()
                    ev1.record()
                    ev1.synchronize()
                    times[i].append(ev0.elapsed_time(ev1) * 1e3 / args.reps)
            for (impl, c), t in zip(arms, times):
                if not t:
                    continue
                us = statistics.median(t)
                rec = {"case": name, "kind": kind, "M": M, "N": N, "K": K, "impl": impl, "cfg": c,
                       "us": round(us, 2), "us_min": round(min(t), 2), "TFs": round(flops / us / 1e6, 1)}
                print(json.dumps(rec), flush=True)
                if impl == "mt" and (best.get((kind, M, N, K)) is None or us < best[(kind, M, N, K)][0]):
                    best[(kind, M, N, K)] = (us, c)
            del graphs
            torch.cuda.empty_cache()
    if args.table:
        print("TABLE = {")
        for k, (us, c) in sorted(best.items()):
            print(f"    {k!r}: {tuple(c)!r},  # {us:.1f} us")
        print("}")


if __name__ == "__main__":
    main()
