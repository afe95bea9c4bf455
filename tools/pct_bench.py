#!/usr/bin/env python3
"""normalize99 on MI355X: HIP radix select vs the torch sort formulation (32 x 2 x 512² uint16-like)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bioengine_worker_amd.cellpose.gpu import normalize99, normalize99_sort  # noqa: E402


def t(fn, x, reps=20):
    for _ in range(3):
        fn(x)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn(x)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for B in (1, 8, 32):
    x = (torch.rand(B, 2, 512, 512, device="cuda") ** 4 * 4000).round()
    print(json.dumps({"batch": B, "radix_select_ms": round(t(normalize99, x), 4),
                      "torch_sort_ms": round(t(normalize99_sort, x), 4)}), flush=True)
