#!/usr/bin/env python3
"""Minimal drivers for kernel traces (rocprofv3 --kernel-trace --stats -- python3 tools/kt_driver.py
<what>): 'vit' = the bench's DINOv2 ViT-B/14 fp8 embedding line (batch 64), 'cpsam_infer' = the
bench's Cellpose-SAM inference line (8 images of 512^2, 9 tiles each).  Prints the bench result."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    what = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if what == "vit":
        print(json.dumps({"vit_embed_imgs_per_s": bench.bench_vit_embed(dev, 64, steps)}))
    elif what == "cpsam_infer":
        print(json.dumps(bench.bench_cpsam_infer(dev, 8, steps, lat_n=3)))
    else:
        raise SystemExit(f"unknown driver {what}")


if __name__ == "__main__":
    main()
