#!/usr/bin/env python3
"""A/B of the fine-tune step's two data-parallel schedules on one GPU: HIP-graph fwd+bwd (then a
bucketed all-reduce) vs eager fwd+bwd with per-bucket readiness (the overlap schedule).  On one GPU
the all-reduce itself is absent, so this isolates what graph replay saves in launch overhead;
``--allreduce-ms`` adds the measured/estimated RCCL time to judge the crossover."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bioengine_worker_amd.train.cellpose_train import TrainConfig, build_trainer, synthetic_train_batch  # noqa: E402


def run(batch: int, graph: bool, steps: int) -> float:
    cfg = TrainConfig(batch_size=batch, bsize=256, lr=1e-5, weight_decay=1e-4, graph=graph)
    tr = build_trainer(cfg, device="cuda")
    b = synthetic_train_batch(batch, 256, device="cuda")
    for _ in range(3):
        tr.step(*b)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        tr.step(*b)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    for batch in (8, 32):
        g, e = run(batch, True, a.steps), run(batch, False, a.steps)
        print(json.dumps({"batch": batch, "graph_ms": round(g, 3), "eager_ms": round(e, 3),
                          "graph_samples_s": round(batch / g * 1e3, 1), "eager_samples_s": round(batch / e * 1e3, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
