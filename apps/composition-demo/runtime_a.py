import time

from ray import serve


@serve.deployment(ray_actor_options={"num_cpus": 1, "num_gpus": 0})
class RuntimeA:
    def __init__(self) -> None:
        self.start = time.time()

    async def ping(self) -> str:
        return "pong"

    async def get_status(self) -> dict:
        return {"name": "RuntimeA", "uptime": time.time() - self.start}

    async def transform_text(self, text: str) -> dict:
        return {"upper": text.upper(), "words": len(text.split())}
