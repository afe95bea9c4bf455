#!/usr/bin/env python3
"""Per-GEMM throughput of one Cellpose-SAM ViT-L block step (M = B*1024 tokens, D = 1024, MLP 4096)
as the training engine issues them (train/cpsam_engine.py): forward F.linear, dgrad torch.mm,
fp32-output wgrad.  HIP-event timing; one JSON line per GEMM with TF/s.
Usage: python tools/vit_gemm_bench.py [--B 8] [--iters 20]"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--impl", default="torch,lt", help="comma list: torch (F.linear / torch.mm), lt (ops/gemm.py)")
    a = ap.parse_args()
    from bioengine_worker_amd.ops import gemm
    from bioengine_worker_amd.ops import vit_train as vt
    from bioengine_worker_amd.train.cpsam_engine import _wgrad

    dev = torch.device("cuda", 0)
    M, D, F4 = a.B * 1024, 1024, 4096
    bf = dict(device=dev, dtype=torch.bfloat16)
    x = {n: torch.randn(M, k, **bf) * 0.5 for n, k in (("d", D), ("f", F4), ("q", 3 * D))}
    w = {"qkv": torch.randn(3 * D, D, **bf) * 0.03, "proj": torch.randn(D, D, **bf) * 0.03,
         "l1": torch.randn(F4, D, **bf) * 0.03, "l2": torch.randn(D, F4, **bf) * 0.03}
    b = {k: torch.randn(v.shape[0], **bf) * 0.1 for k, v in w.items()}
    g32 = {k: torch.empty(v.shape, device=dev, dtype=torch.float32) for k, v in w.items()}
    fpre = torch.randn(M, F4, **bf)
    db = torch.empty(F4, device=dev, dtype=torch.float32)
    b1f = b["l1"].float()
    torch_cases = [
        ("fwd qkv", lambda: F.linear(x["d"], w["qkv"], b["qkv"]), M, 3 * D, D),
        ("fwd proj", lambda: F.linear(x["d"], w["proj"], b["proj"]), M, D, D),
        ("fwd lin1 (+gelu/bias pass)", lambda: vt.gelu_fwd(F.linear(x["d"], w["l1"]), b1f), M, F4, D),
        ("fwd lin2", lambda: F.linear(x["f"], w["l2"], b["l2"]), M, D, F4),
        ("dgrad lin2 (+gelu bwd pass)", lambda: vt.gelu_bwd(torch.mm(x["d"], w["l2"]), fpre, b1f, out_db=db),
         M, F4, D),
        ("dgrad lin1", lambda: torch.mm(x["f"], w["l1"]), M, D, F4),
        ("dgrad proj", lambda: torch.mm(x["d"], w["proj"]), M, D, D),
        ("dgrad qkv", lambda: torch.mm(x["q"], w["qkv"]), M, D, 3 * D),
        ("wgrad lin2", lambda: _wgrad(x["d"], x["f"], g32["l2"]), D, F4, M),
        ("wgrad lin1", lambda: _wgrad(x["f"], x["d"], g32["l1"]), F4, D, M),
        ("wgrad proj", lambda: _wgrad(x["d"], x["d"], g32["proj"]), D, D, M),
        ("wgrad qkv", lambda: _wgrad(x["q"], x["d"], g32["qkv"]), 3 * D, D, M),
    ]
    lt_cases = [
        ("fwd qkv", lambda: gemm.linear(x["d"], w["qkv"], b["qkv"]), M, 3 * D, D),
        ("fwd proj", lambda: gemm.linear(x["d"], w["proj"], b["proj"]), M, D, D),
        ("fwd lin1 (+bias, +gelu pass)", lambda: gemm.linear_gelu(x["d"], w["l1"], b["l1"]), M, F4, D),
        ("fwd lin2", lambda: gemm.linear(x["f"], w["l2"], b["l2"]), M, D, F4),
        ("dgrad lin2 (+dgelu, +bias grad)", lambda: gemm.mm_dgelu(x["d"], w["l2"], fpre, out_db=db), M, F4, D),
        ("dgrad lin1", lambda: gemm.mm(x["f"], w["l1"]), M, D, F4),
        ("dgrad proj", lambda: gemm.mm(x["d"], w["proj"]), M, D, D),
        ("dgrad qkv", lambda: gemm.mm(x["q"], w["qkv"]), M, D, 3 * D),
        ("wgrad lin2", lambda: gemm.wgrad(x["d"], x["f"], g32["l2"]), D, F4, M),
        ("wgrad lin1", lambda: gemm.wgrad(x["f"], x["d"], g32["l1"]), F4, D, M),
        ("wgrad proj", lambda: gemm.wgrad(x["d"], x["d"], g32["proj"]), D, D, M),
        ("wgrad qkv", lambda: gemm.wgrad(x["q"], x["d"], g32["qkv"]), 3 * D, D, M),
    ]
    for impl in a.impl.split(","):
        cases = torch_cases if impl == "torch" else lt_cases
        tot_ms = tot_fl = 0.0
        for name, fn, m, n, k in cases:
            ms = timeit(fn, a.iters)
            fl = 2.0 * m * n * k
            tot_ms += ms
            tot_fl += fl
            print(json.dumps({"impl": impl, "gemm": name, "M": m, "N": n, "K": k, "B": a.B,
                              "us": round(ms * 1e3, 1), "tflops": round(fl / ms / 1e9, 1)}), flush=True)
        print(json.dumps({"impl": impl, "gemm": "block total (x24 per step)", "B": a.B, "us": round(tot_ms * 1e3, 1),
                          "tflops": round(tot_fl / tot_ms / 1e9, 1), "step_ms_x24": round(24 * tot_ms, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
