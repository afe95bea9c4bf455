"""Composition demo runtime B: numpy statistics (reference API: apps/composition-demo/runtime_b.py:40-52)."""
import time

import numpy as np
from ray import serve


@serve.deployment(ray_actor_options={"num_cpus": 1, "num_gpus": 0, "memory": 512 * 1024**2})
class RuntimeB:
    def __init__(self) -> None:
        self.start = time.time()

    async def test_deployment(self) -> None:
        assert (await self.analyze([1, 2, 3]))["mean"] == 2.0

    async def ping(self) -> str:
        return "pong"

    async def get_status(self) -> dict:
        return {"name": "runtime_b", "status": "ok", "numpy_version": np.__version__, "uptime": time.time() - self.start}

    async def analyze(self, values: list) -> dict:
        arr = np.asarray(values, dtype=float)
        if arr.size == 0:
            return {"count": 0, "sorted": []}
        return {"mean": float(arr.mean()), "std": float(arr.std()), "min": float(arr.min()), "max": float(arr.max()),
                "sum": float(arr.sum()), "count": int(arr.size), "sorted": sorted(values)}

    async def compute_stats(self, numbers: list) -> dict:
        r = await self.analyze(numbers)
        return {k: r[k] for k in ("mean", "std", "min", "max")}
