"""Demo app: the smallest complete BioEngine app (lifecycle hooks, schema methods, multiplexing).

Same contract as the reference demo app (apps/demo-app/demo_deployment.py in aicell-lab/bioengine-worker):
async_init / test_deployment / check_health hooks, @serve.multiplexed loader, @schema_method API.
"""
import asyncio
import logging
import os
import time
from datetime import datetime

from hypha_rpc.utils.schema import schema_method
from pydantic import Field
from ray import serve

log = logging.getLogger("ray.serve")

BANNER = [
    "+------------------------------------------+",
    "|   ___  _      ___           _            |",
    "|  | _ )(_) ___| __|_ _  __ _(_)_ _  ___   |",
    "|  | _ \\| |/ _ \\ _|| ' \\/ _` | | ' \\/ -_)  |",
    "|  |___/|_|\\___/___|_||_\\__, |_|_||_\\___|  |",
    "|                       |___/   on MI355X  |",
    "+------------------------------------------+",
]


@serve.deployment(
    ray_actor_options={"num_cpus": 1, "num_gpus": 0, "memory": 0.5 * 1024 ** 3,
                       "runtime_env": {"env_vars": {"EXAMPLE_ENV_VAR": "example_value"}}},
    max_ongoing_requests=10,
)
class DemoDeployment:
    def __init__(self, greeting: str = "Hello from the DemoDeployment!") -> None:
        self.greeting = greeting
        self.start_time = time.time()
        self.fail_health_check = False
        self.loaded_models = []

    async def async_init(self) -> None:
        await asyncio.sleep(0.01)

    async def test_deployment(self) -> None:
        assert os.environ["EXAMPLE_ENV_VAR"] == "example_value"
        await self._get_model("test_model")
        assert (await self.ping())["status"] == "ok"
        assert (await self.reverse_text(text="hello"))["reversed"] == "olleh"

    async def check_health(self) -> None:
        if self.fail_health_check:
            raise RuntimeError("Simulated health check failure.")

    @serve.multiplexed(max_num_models_per_replica=3)
    async def _get_model(self, model_id: str):
        log.info(f"loading model {model_id}")
        self.loaded_models.append(model_id)
        return {"model_id": model_id}

    @schema_method
    async def ping(self) -> dict:
        """Connectivity check: status, greeting, timestamp and replica uptime."""
        return {"status": "ok", "message": self.greeting, "timestamp": datetime.now().isoformat(),
                "timezone": time.tzname[0], "uptime": time.time() - self.start_time}

    @schema_method
    async def ascii_art(self) -> list:
        """ASCII banner."""
        return list(BANNER)

    @schema_method
    async def list_datasets(self) -> dict:
        """Datasets (and their files) visible through the BioEngine datasets server."""
        out = {}
        for ds in await self.bioengine_datasets.list_datasets():
            out[ds] = await self.bioengine_datasets.list_files(ds)
        return out

    @schema_method
    async def reverse_text(self, text: str = Field(..., description="Text to reverse")) -> dict:
        """Reverse a string."""
        return {"original": text, "reversed": text[::-1], "length": len(text)}

    @schema_method
    async def get_model(self, model_id: str = Field("default", description="Model id to load (multiplexed)")) -> dict:
        """Load (or fetch from the per-replica LRU) a model by id."""
        m = await self._get_model(model_id)
        return {"model": m, "loads": len(self.loaded_models)}

    @schema_method
    async def set_fail_health_check(self) -> None:
        """Fault injection: make the next health checks fail."""
        self.fail_health_check = True
