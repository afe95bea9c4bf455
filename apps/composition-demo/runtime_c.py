import asyncio
import time

from ray import serve


@serve.deployment(ray_actor_options={"num_cpus": 1, "num_gpus": 0})
class RuntimeC:
    def __init__(self) -> None:
        self.start = time.time()

    async def ping(self) -> str:
        return "pong"

    async def get_status(self) -> dict:
        return {"name": "RuntimeC", "uptime": time.time() - self.start}

    async def wait(self, delay: float) -> float:
        t0 = time.time()
        await asyncio.sleep(delay)
        return time.time() - t0
