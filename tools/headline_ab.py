#!/usr/bin/env python3
"""Headline A/B helper: the bench's pipelined + sequential Cellpose rates and batch-1 latency only
(bench.bench_infer / bench_latency), one JSON line.  Env knobs select the arm."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import bench


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    a.chunks, a.sequential, a.trace = 1, False, None
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dt, runner, imgs, p, extra = bench.bench_infer(a, 1, 0, dev)
    p50, p95 = bench.bench_latency(runner, imgs, p)
    out = {"imgs_per_s": round(a.batch * a.steps / dt, 2), "ms_per_step": round(dt / a.steps * 1e3, 3),
           "p50_ms_b1": round(p50, 3), "p95_ms_b1": round(p95, 3),
           "env": {k: v for k, v in os.environ.items() if k.startswith("BE_")}}
    out.update(extra)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
