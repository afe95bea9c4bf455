#!/usr/bin/env python3
"""CPSAM (ViT-L/8, 1,024 tokens per image) training GEMMs: in-house bf16 MFMA GEMM
(``ops/gemm_bf16.py``) against PyTorch's hipBLASLt call for the same op, per shape, at batch 1 and 8.
HIP-event median of --reps, random data.  One JSON line per (gemm, impl)."""
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
    return ts[len(ts) // 2] * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batches", default="8,1")
    ap.add_argument("--only", default="", help="substring of the GEMM name")
    ap.add_argument("--impls", default="hip,torch")
    ap.add_argument("--cfgs", default="", help="comma list of BE_GEMM_CFG values to A/B for the hip impl")
    a = ap.parse_args()
    from bioengine_worker_amd.ops import gemm_bf16 as gb
    from bioengine_worker_amd.ops import vit_train as vt

    dev = torch.device("cuda", 0)
    D, Hd = 1024, 4096
    g = torch.Generator(device=dev).manual_seed(0)
    R = lambda *s: torch.randn(*s, device=dev, generator=g).to(torch.bfloat16)  # noqa: E731
    for B in [int(v) for v in a.batches.split(",")]:
        M = B * 1024
        x, h = R(M, D), R(M, Hd)
        wq, wp, w1, w2 = R(3 * D, D) * 0.03, R(D, D) * 0.03, R(Hd, D) * 0.03, R(D, Hd) * 0.03
        bq, bp, b1, b2 = (torch.randn(n, device=dev) for n in (3 * D, D, Hd, D))
        bqh, bph, b1h, b2h = (v.to(torch.bfloat16) for v in (bq, bp, b1, b2))
        dq, dD, dH = R(M, 3 * D), R(M, D), R(M, Hd)
        f = R(M, Hd)
        dbuf = torch.zeros(Hd, device=dev)
        zero = torch.zeros(Hd, device=dev)
        outs = {n: torch.empty(n_, k_, device=dev) for n, (n_, k_) in
                {"qkv": (3 * D, D), "proj": (D, D), "l1": (Hd, D), "l2": (D, Hd)}.items()}
        cases = [
            ("fwd qkv", 2 * M * 3 * D * D, lambda: gb.linear(x, wq, bq), lambda: F.linear(x, wq, bqh)),
            ("fwd proj", 2 * M * D * D, lambda: gb.linear(x, wp, bp), lambda: F.linear(x, wp, bph)),
            ("fwd lin1+gelu", 2 * M * Hd * D, lambda: gb.linear_gelu(x, w1, b1),
             lambda: vt.gelu_fwd(F.linear(x, w1, b1h), zero)),
            ("fwd lin2", 2 * M * D * Hd, lambda: gb.linear(h, w2, b2), lambda: F.linear(h, w2, b2h)),
            ("dgrad lin2+dgelu", 2 * M * Hd * D, lambda: gb.mm_dgelu(dD, w2, f, out_db=dbuf),
             lambda: vt.gelu_bwd(torch.mm(dD, w2), f, zero, out_db=dbuf)),
            ("dgrad lin1", 2 * M * D * Hd, lambda: gb.mm(dH, w1), lambda: torch.mm(dH, w1)),
            ("dgrad proj", 2 * M * D * D, lambda: gb.mm(dD, wp), lambda: torch.mm(dD, wp)),
            ("dgrad qkv", 2 * M * D * 3 * D, lambda: gb.mm(dq, wq), lambda: torch.mm(dq, wq)),
            ("wgrad lin2", 2 * M * D * Hd, lambda: gb.wgrad(dD, h, outs["l2"]),
             lambda: torch.mm(dD.t(), h, out_dtype=torch.float32, out=outs["l2"])),
            ("wgrad lin1", 2 * M * D * Hd, lambda: gb.wgrad(dH, x, outs["l1"]),
             lambda: torch.mm(dH.t(), x, out_dtype=torch.float32, out=outs["l1"])),
            ("wgrad proj", 2 * M * D * D, lambda: gb.wgrad(dD, x, outs["proj"]),
             lambda: torch.mm(dD.t(), x, out_dtype=torch.float32, out=outs["proj"])),
            ("wgrad qkv", 2 * M * D * 3 * D, lambda: gb.wgrad(dq, x, outs["qkv"]),
             lambda: torch.mm(dq.t(), x, out_dtype=torch.float32, out=outs["qkv"])),
        ]
        tot = {"hip": 0.0, "torch": 0.0}
        for name, fl, hip, ref in cases:
            if a.only and a.only not in name:
                continue
            runs = [("torch", ref, None)] + ([("hip", hip, c) for c in a.cfgs.split(",")] if a.cfgs else [("hip", hip, None)])
            for impl, fn, cfg in runs:
                if impl not in a.impls.split(","):
                    continue
                if cfg is not None:
                    os.environ["BE_GEMM_CFG"] = cfg
                else:
                    os.environ.pop("BE_GEMM_CFG", None)
                try:
                    us = timeit(fn, a.reps)
                except Exception as e:  # noqa: BLE001
                    print(json.dumps({"B": B, "gemm": name, "impl": impl, "cfg": cfg, "error": str(e)[:200]}), flush=True)
                    continue
                tot[impl] += us
                print(json.dumps({"B": B, "gemm": name, "impl": impl, "cfg": cfg, "us": round(us, 1),
                                  "TFs": round(fl / us / 1e6, 1)}), flush=True)
        print(json.dumps({"B": B, "block_total_us": {k: round(v, 1) for k, v in tot.items()},
                          "step_ms_x24": {k: round(24 * v / 1e3, 2) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
