#!/usr/bin/env python3
"""Process-replica hop cost on the host: round-trip time of a call to a child-process replica
(serve/replica.py ProcessReplica: socket header + shared-memory ring payloads) against payload size
and direction, with no GPU work in the replica.  The served-Cellpose c=1 gap (served p50 minus the
direct pipeline) is this hop plus H2D/D2H; run it with different ``BE_RING_COPY_THREADS`` /
``MALLOC_*`` settings to A/B the copy path.

Usage: ``python tools/replica_hop_bench.py [--reps 400] [--sizes 0,262144,1048576,2097152]``;
prints one JSON line per (direction, size).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np  # noqa: E402


class HopEcho:
    """Replica class: ``sink`` takes a payload and returns nothing big, ``src`` returns one."""

    def __init__(self, sizes):
        self.outs = {n: np.zeros(n, np.uint8) for n in sizes}

    async def sink(self, arr):
        return 1

    async def src(self, n):
        return self.outs[n]


async def main_async(a) -> list[dict]:
    from bioengine_worker_amd.serve.replica import ProcessReplica

    sizes = [int(s) for s in a.sizes.split(",")]
    r = ProcessReplica("hop", "bench", HopEcho, (sizes,), {}, [])
    await r.start()
    rows = []
    try:
        for n in sizes:
            x = np.ones(n, np.uint8)
            for direction, method, args in (("in", "sink", [x]), ("out", "src", [n])):
                for _ in range(30):
                    await r.call(method, args, {})
                ts = []
                for _ in range(a.reps):
                    t = time.perf_counter()
                    await r.call(method, args, {})
                    ts.append(time.perf_counter() - t)
                ms = np.array(ts) * 1e3
                row = {"direction": direction, "bytes": n, "p50_ms": round(float(np.percentile(ms, 50)), 4),
                       "p10_ms": round(float(np.percentile(ms, 10)), 4), "p90_ms": round(float(np.percentile(ms, 90)), 4),
                       "copy_threads": os.environ.get("BE_RING_COPY_THREADS", "4"),
                       "malloc_tuned": os.environ.get("BE_REPLICA_MALLOC", "1")}
                rows.append(row)
                print(json.dumps(row), flush=True)
    finally:
        await r.stop()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=400)
    ap.add_argument("--sizes", default="0,262144,1048576,2097152")
    asyncio.run(main_async(ap.parse_args()))


if __name__ == "__main__":
    main()
