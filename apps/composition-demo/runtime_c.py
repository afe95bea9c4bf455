"""Composition demo runtime C: time operations (reference API: apps/composition-demo/runtime_c.py:42-60)."""
import asyncio
import datetime
import time

from ray import serve


@serve.deployment(ray_actor_options={"num_cpus": 1, "num_gpus": 0, "memory": 512 * 1024**2})
class RuntimeC:
    def __init__(self) -> None:
        self.start = time.time()

    async def test_deployment(self) -> None:
        assert (await self.time_ops(2))["count"] == 2

    async def ping(self) -> str:
        return "pong"

    async def get_status(self) -> dict:
        return {"name": "runtime_c", "status": "ok", "current_time": datetime.datetime.now().isoformat(),
                "uptime": time.time() - self.start}

    async def time_ops(self, count: int = 5) -> dict:
        now = datetime.datetime.now()
        stamps = [(now + datetime.timedelta(seconds=i)).isoformat() for i in range(max(0, int(count)))]
        return {"current_timestamp": now.isoformat(), "unix_timestamp": time.time(), "timestamps": stamps,
                "formatted": now.strftime("%Y-%m-%d %H:%M:%S"), "day_of_week": now.strftime("%A"), "count": count}

    async def wait(self, delay: float) -> float:
        t0 = time.time()
        await asyncio.sleep(delay)
        return time.time() - t0
