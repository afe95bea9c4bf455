#!/usr/bin/env python3
"""Router <-> process-replica transfer: Unix socket only vs the C++ shared-memory rings.

Echoes float32 arrays of several sizes through a process replica (request and result both carry the
array) and reports the round-trip time per size.  Usage: ``python tools/ring_bench.py [--reps 20]``.
"""
import argparse
import asyncio
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from bioengine_worker_amd.compat import install  # noqa: E402

install()
from ray import serve  # noqa: E402

from bioengine_worker_amd.serve import controller as ctrl_mod  # noqa: E402


@serve.deployment(ray_actor_options={"num_cpus": 0})
class Echo:
    async def echo(self, a):
        return a


async def run(ring_mb: int, sizes, reps: int) -> dict:
    os.environ["BIOENGINE_REPLICA_MODE"] = "process"
    os.environ["BE_REPLICA_RING_MB"] = str(ring_mb)
    ctrl_mod.set_controller(None)
    h = await serve.run(Echo.bind(), name=f"echo{ring_mb}")
    out = {}
    for kib in sizes:
        a = np.ones(kib * 256, np.float32)
        await h.echo.remote(a)
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            await h.echo.remote(a)
            t.append(time.perf_counter() - t0)
        ms = 1e3 * float(np.median(t))
        out[f"{kib}KiB"] = {"ms": round(ms, 3), "GB/s": round(2 * a.nbytes / ms / 1e6, 2)}
    await serve.delete(f"echo{ring_mb}")
    ctrl_mod.set_controller(None)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--sizes", default="4,1024,16384,65536,262144", help="payload sizes in KiB")
    a = ap.parse_args()
    sizes = [int(s) for s in a.sizes.split(",")]
    res = {"socket": asyncio.run(run(0, sizes, a.reps)), "shm_ring": asyncio.run(run(512, sizes, a.reps))}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
