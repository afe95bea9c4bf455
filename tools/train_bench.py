#!/usr/bin/env python3
"""Fine-tune step micro-bench: per-phase time of the CPnet training step (augment, fwd+loss, bwd,
AdamW) and whole-step samples/s, for batch/crop sweeps.  One JSON line per config.

    python tools/train_bench.py --batch 8 --bsize 256 --steps 20 [--norm batch|group] [--engine autograd|hip]
"""
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
    ap.add_argument("--batch", type=int, nargs="+", default=[8])
    ap.add_argument("--bsize", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--norm", default="batch")
    ap.add_argument("--engine", default=None)
    ap.add_argument("--phases", action="store_true", help="also time each phase with syncs in between")
    args = ap.parse_args()
    from bioengine_worker_amd.train.cellpose_train import TrainConfig, build_trainer, synthetic_train_batch

    dev = torch.device("cuda", 0)
    for B in args.batch:
        kw = dict(batch_size=B, bsize=args.bsize, lr=1e-5, weight_decay=1e-4, norm=args.norm)
        if args.engine:
            kw["engine"] = args.engine
        cfg = TrainConfig(**kw)
        tr = build_trainer(cfg, device=dev)
        batch = synthetic_train_batch(B, cfg.bsize, device=dev)
        for _ in range(3):
            tr.step(*batch)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            tr.step(*batch)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        out = {"batch": B, "bsize": args.bsize, "norm": args.norm, "engine": args.engine or "default",
               "ms_per_step": round(dt * 1e3, 3), "samples_per_s": round(B / dt, 1)}
        if args.phases:
            from bioengine_worker_amd.profiling import trace

            trace.clear()
            trace.enable(True)
            for _ in range(5):
                tr.step(*batch)
            torch.cuda.synchronize()
            out["phases_ms"] = {k: round(v["mean_ms"], 3) for k, v in trace.summary().items()} \
                if isinstance(trace.summary(), dict) else trace.summary()
            trace.enable(False)
        print(json.dumps(out), flush=True)
        del tr, batch
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
