#!/usr/bin/env python3
"""A/B of the ViT-B/14 fp8 embedder's qkv GEMM (DINOv2, batch 64, 224^2): the HIP block-scaled MX-fp8
GEMM fed by the LayerNorm's MX output vs hipBLASLt row-scaled fp8.  Interleaved rounds, one process."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from bioengine_worker_amd.models.vit import ViT, ViTConfig, ViTEngine


def main(rounds=5, steps=20, batch=64):
    dev = torch.device("cuda", 0)
    net = ViT(ViTConfig.dinov2("vitb14")).randomize_(0).eval()
    engs = {}
    for q in ("hip", "hipblaslt"):
        os.environ["BE_VIT_QKV_GEMM"] = q
        engs[q] = ViTEngine(net, dev, precision="fp8", fp8_gemm="hip")
    ref = ViTEngine(net, dev)
    x = torch.randn(batch, 3, 224, 224, device=dev)
    r = ref.embed(x)
    cos = {q: float(torch.nn.functional.cosine_similarity(e.embed(x), r, dim=1).min()) for q, e in engs.items()}
    t = {q: [] for q in engs}
    for _ in range(rounds):
        for q, e in engs.items():
            for _ in range(3):
                e.embed(x)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                e.embed(x)
            torch.cuda.synchronize()
            t[q].append(batch * steps / (time.perf_counter() - t0))
    for q in engs:
        print(json.dumps({"qkv_gemm": q, "imgs_per_s_median": round(statistics.median(t[q]), 1),
                          "imgs_per_s": [round(v, 1) for v in t[q]], "cos_min_vs_bf16": round(cos[q], 5)}), flush=True)


if __name__ == "__main__":
    main()
