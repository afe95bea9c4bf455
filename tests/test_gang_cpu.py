"""Gang-scheduled multi-process jobs (serve/gang.py) on CPU ranks (gloo): results in rank order,
resources reserved all-or-nothing and released, and a failing rank tears the whole gang down."""
import asyncio

import pytest

from bioengine_worker_amd.serve.controller import ResourcePool
from bioengine_worker_amd.serve.gang import GangError, GangManager


@pytest.mark.timeout(180)
def test_gang_collective_and_teardown():
    async def main():
        mgr = GangManager(ResourcePool(num_cpus=4, gpu_ids=[]))
        res = await mgr.run("bioengine_worker_amd.serve.gang:collective_probe", {"payload_mb": 0.01}, world_size=3,
                            timeout_s=120)
        assert [r["rank"] for r in res] == [0, 1, 2]
        assert all(r["sum"] == 6.0 and r["gathered"] == [0.0, 1.0, 2.0] and r["backend"] == "gloo" for r in res)
        assert mgr.resources.used_cpu == 0
        with pytest.raises(GangError, match="rank 1"):
            await mgr.run("bioengine_worker_amd.serve.gang:collective_probe", {"fail_rank": 1}, world_size=2,
                          timeout_s=120)
        assert mgr.resources.used_cpu == 0
        states = [j["state"] for j in mgr.status().values()]
        assert states == ["completed", "failed"]

    asyncio.run(main())
