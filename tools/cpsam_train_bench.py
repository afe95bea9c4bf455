#!/usr/bin/env python3
"""Cellpose-SAM (ViT-L/8, 256x256 crops) fine-tune step throughput on one GPU.

Engine = train/cpsam_engine.py (HIP attention fwd/bwd, fused LN/GELU/cast kernels, hipBLASLt GEMMs,
fused AdamW).  Baseline = the reference's algorithm: PyTorch autograd through the same CPSAM module
with bf16 autocast + torch AdamW(fused) (the reference runs fp32 autograd, main.py:1350-1358, which is
slower still).  Prints one JSON line per configuration.
Usage: python tools/cpsam_train_bench.py [--batch 1 8] [--steps 10] [--baseline]"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--depth", type=int, default=24)
    ap.add_argument("--baseline", action="store_true")
    ap.add_argument("--graph", type=int, default=-1, help="override TrainConfig.graph (0/1)")
    ap.add_argument("--overlap-adamw", type=int, default=-1,
                    help="override TrainConfig.cpsam_overlap_adamw (0/1): per-group AdamW inside the graph")
    args = ap.parse_args()
    from bioengine_worker_amd.models.cpsam import CPSAM
    from bioengine_worker_amd.ops import train_ops
    from bioengine_worker_amd.train.cellpose_train import TrainConfig, build_trainer, synthetic_train_batch

    dev = torch.device("cuda", 0)
    for B in args.batch:
        cfg = TrainConfig(batch_size=B, bsize=256, lr=1e-5, weight_decay=1e-4)
        if args.graph >= 0:
            cfg.graph = bool(args.graph)
        if args.overlap_adamw >= 0:
            cfg.cpsam_overlap_adamw = bool(args.overlap_adamw)
        net = CPSAM(depth=args.depth).randomize_(0)
        tr = build_trainer(cfg, dev, net=net)
        batch = synthetic_train_batch(B, 256, device=dev)
        for _ in range(args.warmup):
            tr.step(*batch)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            loss = tr.step(*batch)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        out = {"bench": "cpsam_finetune_step", "engine": "hip", "batch": B, "depth": args.depth,
               "ms_per_step": round(dt * 1e3, 3), "samples_per_sec": round(B / dt, 2), "loss": float(loss),
               "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 2),
               "gemm": os.environ.get("BE_CPSAM_GEMM", "lib"), "overlap_adamw": bool(cfg.cpsam_overlap_adamw),
               "adamw_bg_blocks": int(os.environ.get("BE_ADAMW_BG_BLOCKS", "256"))}
        if out["gemm"] == "auto":
            from bioengine_worker_amd.ops import gemm_auto

            ch = gemm_auto.choices()
            out["gemm_choices"] = {**{k: sum(c["impl"] == k for c in ch) for k in ("hip", "pp", "lib")}, "table": ch}
        print(json.dumps(out), flush=True)
        del tr
        torch.cuda.empty_cache()
        if args.baseline:
            net = CPSAM(depth=args.depth).randomize_(0).to(dev).train()
            opt = torch.optim.AdamW(net.parameters(), lr=1e-5, weight_decay=1e-4, fused=True)
            x = torch.randn(B, 3, 256, 256, device=dev)
            lbl = batch[1][:, :, :256, :256].contiguous()

            def step():
                opt.zero_grad(set_to_none=True)
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    y = net(x)[0]
                loss = train_ops.seg_loss_ref(y.float(), lbl)
                loss.backward()
                opt.step()
                return loss

            for _ in range(args.warmup):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.steps
            print(json.dumps({"bench": "cpsam_finetune_step", "engine": "torch-autograd-bf16-autocast", "batch": B,
                              "depth": args.depth, "ms_per_step": round(dt * 1e3, 3),
                              "samples_per_sec": round(B / dt, 2)}), flush=True)
            del net, opt
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
