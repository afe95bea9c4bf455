import time

import numpy as np
from ray import serve


@serve.deployment(ray_actor_options={"num_cpus": 1, "num_gpus": 0})
class RuntimeB:
    def __init__(self) -> None:
        self.start = time.time()

    async def ping(self) -> str:
        return "pong"

    async def get_status(self) -> dict:
        return {"name": "RuntimeB", "uptime": time.time() - self.start}

    async def compute_stats(self, numbers: list) -> dict:
        x = np.asarray(numbers, dtype=float)
        return {"mean": float(x.mean()), "std": float(x.std()), "min": float(x.min()), "max": float(x.max())}
