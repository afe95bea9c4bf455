"""Composition entry: the extra deployments are bound to __init__ params named after their files."""
import asyncio
import time

from hypha_rpc.utils.schema import schema_method
from pydantic import Field
from ray import serve
from ray.serve.handle import DeploymentHandle


@serve.deployment(ray_actor_options={"num_cpus": 0, "num_gpus": 0})
class EntryDeployment:
    def __init__(self, runtime_a: DeploymentHandle, runtime_b: DeploymentHandle, runtime_c: DeploymentHandle) -> None:
        self.runtime_a, self.runtime_b, self.runtime_c = runtime_a, runtime_b, runtime_c
        self.start_time = time.time()

    async def test_deployment(self) -> None:
        for h in (self.runtime_a, self.runtime_b, self.runtime_c):
            assert await h.ping.remote() == "pong"

    @schema_method
    async def status(self) -> dict:
        """Uptime of the entry plus each runtime's status."""
        a, b, c = await asyncio.gather(self.runtime_a.get_status.remote(), self.runtime_b.get_status.remote(),
                                       self.runtime_c.get_status.remote())
        return {"entry_uptime": time.time() - self.start_time, "runtime_a": a, "runtime_b": b, "runtime_c": c}

    @schema_method
    async def process(self, text: str = Field(..., description="Text"), numbers: list = Field(..., description="Numbers"),
                      delay: float = Field(0.01, description="Seconds runtime C sleeps")) -> dict:
        """Fan out to the three runtimes concurrently and combine their answers."""
        a, b, c = await asyncio.gather(self.runtime_a.transform_text.remote(text),
                                       self.runtime_b.compute_stats.remote(numbers), self.runtime_c.wait.remote(delay))
        return {"text": a, "stats": b, "waited": c}
