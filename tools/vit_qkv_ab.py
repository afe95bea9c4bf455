#!/usr/bin/env python3
"""DINOv2 ViT-B/14 fp8 embedding throughput (batch 64, 224^2) with qkv on hipBLASLt vs the HIP fp8
GEMM (BE_VIT_QKV_GEMM), same process, alternating to cancel clock drift.  One JSON line per arm."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from bioengine_worker_amd.search.ingestion import default_engine_factory

    dev = torch.device("cuda", 0)
    x = torch.randn(64, 3, 224, 224, device=dev)
    engs = {}
    for arm in ("hipblaslt", "hip"):
        os.environ["BE_VIT_QKV_GEMM"] = arm
        engs[arm] = default_engine_factory(dev, "vitb14")
        for _ in range(5):
            engs[arm].embed(x)
    torch.cuda.synchronize()
    res = {a: [] for a in engs}
    for _ in range(5):
        for arm, eng in engs.items():
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(20):
                eng.embed(x)
            torch.cuda.synchronize()
            res[arm].append((time.perf_counter() - t) / 20)
    ref = engs["hip"].embed(x[:8])
    for arm, ts in res.items():
        ts.sort()
        cos = torch.nn.functional.cosine_similarity(engs[arm].embed(x[:8]), ref, dim=1).min().item()
        print(json.dumps({"qkv_gemm": arm, "ms_per_batch64": round(ts[len(ts) // 2] * 1e3, 3),
                          "imgs_per_s": round(64 / ts[len(ts) // 2], 1), "cos_min_vs_hip_qkv": round(cos, 5)}),
              flush=True)


if __name__ == "__main__":
    main()
