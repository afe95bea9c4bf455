#!/usr/bin/env python3
"""Run only bench.py's 3-D EM line (bench_em_volume3d) on one GPU, default config scale
(256 x 2048^2 slab): `python tools/em3d_bench.py [--em3d-z Z --em3d-yx YX]`."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import bench

ap = argparse.ArgumentParser()
ap.add_argument("--em3d-z", type=int, default=256)
ap.add_argument("--em3d-yx", type=int, default=2048)
ap.add_argument("--sweep", default="", help="tile_z:tile:batch,... configurations to run in this process")
args = ap.parse_args()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
for cfg in (args.sweep.split(",") if args.sweep else [""]):
    if cfg:
        args.em3d_tile_z, args.em3d_tile, args.em3d_batch = (int(v) for v in cfg.split(":"))
    torch.cuda.reset_peak_memory_stats(dev)
    out = bench.bench_em_volume3d(args, 1, 0, dev)
    out["max_memory_allocated_gb"] = round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 2)
    print(json.dumps(out), flush=True)
