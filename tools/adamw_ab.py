#!/usr/bin/env python3
"""Fused AdamW over a ViT-L-sized flat buffer (304,688,322 fp32 params + bf16 mirror): the two
kernels of csrc/kernels/adamw.hip alternated in one process; HIP-event median, GB/s moved."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from bioengine_worker_amd.ops import _native, train_ops

    dev = torch.device("cuda", 0)
    n = 304_688_322
    p, g, m, v = (torch.randn(n, device=dev) for _ in range(4))
    v.abs_()
    mirror = torch.empty(n, device=dev, dtype=torch.bfloat16)
    ts = {0: [], 1: []}
    for r in range(12):
        for var in (0, 1):
            _native.call("be_adamw_set_variant", var)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            train_ops.adamw_flat_(p, g, m, v, lr=1e-6, step=r + 1, weight_decay=1e-4, p_bf16=mirror)
            e.record()
            e.synchronize()
            if r >= 2:
                ts[var].append(s.elapsed_time(e))
    _native.call("be_adamw_set_variant", 0)
    moved = n * (4 * 4 + 3 * 4 + 2)
    for var, t in ts.items():
        t.sort()
        ms = t[len(t) // 2]
        print(json.dumps({"variant": var, "ms": round(ms, 4), "GBps": round(moved / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
