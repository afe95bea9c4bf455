#!/usr/bin/env python3
"""Batch-1 latency anatomy of the headline pipeline (what a lone served client waits for): runs
``runner.eval`` on ONE 512x512 image N times with per-stage trace spans.  Run under
``rocprofv3 --kernel-trace --stats`` for the per-kernel view."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bioengine_worker_amd.cellpose.pipeline import CellposeRunner, EvalParams, synthetic_cells  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--host", action="store_true", help="host uint16 input (served path) instead of device")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    runner = CellposeRunner(device=dev, seed=0)
    img = torch.from_numpy(synthetic_cells(1, 512, 512, nchan=2, ncells=60, seed=0))
    if not a.host:
        img = img.to(dev)
    p = EvalParams(niter=200, flow_threshold=0.4, cellprob_threshold=0.0, min_size=15)
    for _ in range(5):
        runner.eval(img, p)
    torch.cuda.synchronize()
    lat = []
    for _ in range(a.iters):
        t = time.perf_counter()
        m, _, _ = runner.eval(img, p)
        torch.cuda.synchronize()
        lat.append((time.perf_counter() - t) * 1e3)
    lat.sort()
    print(json.dumps({"p50_ms": round(lat[len(lat) // 2], 3), "min_ms": round(lat[0], 3), "host_input": a.host,
                      "masks": int(m.max())}))


if __name__ == "__main__":
    main()
