"""Composition entry: the extra deployments are bound to __init__ params named after their files.

Service API of the reference composition demo (apps/composition-demo/entry_deployment.py:53-131):
``status``, ``process_text`` (runtime A), ``analyze_numbers`` (runtime B), ``time_operations``
(runtime C), ``run_all`` (all three concurrently); plus ``process`` (one fan-out call)."""
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
    async def process_text(self, text: str = Field(..., description="Text to process")) -> dict:
        """Text operations through runtime A: word/char counts, reversed, upper/lower/title case."""
        return await self.runtime_a.process_text.remote(text)

    @schema_method
    async def analyze_numbers(self, values: list = Field(..., description="List of numbers to analyze")) -> dict:
        """Statistics through runtime B (numpy): mean, std, min, max, sum, count, sorted."""
        return await self.runtime_b.analyze.remote(values)

    @schema_method
    async def time_operations(self, count: int = Field(5, description="Number of timestamps to generate")) -> dict:
        """Time-based string operations through runtime C."""
        return await self.runtime_c.time_ops.remote(count)

    @schema_method
    async def run_all(self, text: str = Field("hello bioengine", description="Text input for runtime A"),
                      values: list = Field(None, description="Numbers for runtime B (default [1, 2, 3, 4, 5])"),
                      count: int = Field(3, description="Count for runtime C")) -> dict:
        """All three runtimes concurrently, results combined."""
        values = [1, 2, 3, 4, 5] if values is None else values
        a, b, c = await asyncio.gather(self.runtime_a.process_text.remote(text), self.runtime_b.analyze.remote(values),
                                       self.runtime_c.time_ops.remote(count))
        return {"text_result": a, "data_result": b, "time_result": c}

    @schema_method
    async def process(self, text: str = Field(..., description="Text"), numbers: list = Field(..., description="Numbers"),
                      delay: float = Field(0.01, description="Seconds runtime C sleeps")) -> dict:
        """Fan out to the three runtimes concurrently and combine their answers."""
        a, b, c = await asyncio.gather(self.runtime_a.transform_text.remote(text),
                                       self.runtime_b.compute_stats.remote(numbers), self.runtime_c.wait.remote(delay))
        return {"text": a, "stats": b, "waited": c}
