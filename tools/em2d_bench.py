#!/usr/bin/env python3
"""Run only bench.py's 2-D EM line (bench_em_volume) on one GPU: `python tools/em2d_bench.py
[--em-z Z --em-yx YX] [--sweep tile:overlap:batch,...]`."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import bench

ap = argparse.ArgumentParser()
ap.add_argument("--em-z", type=int, default=256)
ap.add_argument("--em-yx", type=int, default=2048)
ap.add_argument("--em-tile-batch", type=int, default=32)
ap.add_argument("--sweep", default="", help="tile:overlap:batch,... configurations to run in this process")
args = ap.parse_args()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
for cfg in (args.sweep.split(",") if args.sweep else [""]):
    if cfg:
        args.em_tile, args.em_overlap, args.em_tile_batch = (int(v) for v in cfg.split(":"))
    torch.cuda.reset_peak_memory_stats(dev)
    out = bench.bench_em_volume(args, 1, 0, dev)
    out["max_memory_allocated_gb"] = round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 2)
    print(json.dumps(out), flush=True)
