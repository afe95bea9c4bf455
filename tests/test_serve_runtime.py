"""Native serving runtime with the Ray-Serve-compatible API (no Ray installed)."""
import asyncio
import os
import time

import pytest

from bioengine_worker_amd.compat import install

install()

from ray import serve  # noqa: E402  (the native shim)
from ray.serve.handle import DeploymentHandle  # noqa: E402

from bioengine_worker_amd.serve import controller as ctrl_mod  # noqa: E402


@pytest.fixture(autouse=True)
def fresh_controller():
    ctrl_mod.set_controller(None)
    yield
    ctrl_mod.set_controller(None)


@serve.deployment(ray_actor_options={"num_cpus": 0})
class Adder:
    def __init__(self, k: int = 1):
        self.k = k
        self.tag = serve.get_replica_context().replica_tag

    async def add(self, x):
        return x + self.k

    def sync_mul(self, x):
        return x * self.k

    @serve.multiplexed(max_num_models_per_replica=2)
    async def get_model(self, model_id: str):
        self.loads = getattr(self, "loads", 0) + 1
        return f"model-{model_id}"

    async def use_model(self):
        return await self.get_model(serve.get_multiplexed_model_id())


@serve.deployment(ray_actor_options={"num_cpus": 0})
class Entry:
    def __init__(self, adder: DeploymentHandle):
        self.adder = adder

    async def __call__(self, x):
        return await self.adder.add.remote(x)

    async def mux(self, mid):
        return await self.adder.options(multiplexed_model_id=mid).use_model.remote()


@pytest.mark.unit
def test_compose_route_and_multiplex():
    async def main():
        h = await serve.run(Entry.bind(Adder.bind(5)), name="app1")
        assert await h.remote(1) == 6
        assert await h.mux.remote("a") == "model-a"
        st = serve.status()
        assert st.applications["app1"].status == "RUNNING"
        assert set(st.applications["app1"].deployments) == {"Adder", "Entry"}
        await serve.delete("app1")
        assert "app1" not in serve.status().applications

    asyncio.run(main())


@serve.deployment(ray_actor_options={"num_cpus": 0}, max_ongoing_requests=1, max_queued_requests=2)
class Slow:
    async def work(self, t):
        await asyncio.sleep(t)
        return t


@pytest.mark.unit
def test_admission_queue_and_backpressure():
    from ray.serve.exceptions import BackPressureError

    async def main():
        h = await serve.run(Slow.bind(), name="slow")
        rs = [h.work.remote(0.2) for _ in range(3)]
        await asyncio.sleep(0.05)
        with pytest.raises(BackPressureError):
            await h.work.remote(0.0)
        assert await asyncio.gather(*rs) == [0.2] * 3
        await serve.delete("slow")

    asyncio.run(main())


@serve.deployment(ray_actor_options={"num_cpus": 0}, max_ongoing_requests=64)
class Batcher:
    def __init__(self):
        self.sizes = []

    @serve.batch(max_batch_size=8, batch_wait_timeout_s=0.05)
    async def infer(self, xs):
        self.sizes.append(len(xs))
        await asyncio.sleep(0.01)
        return [x * 2 for x in xs]

    async def sizes_seen(self):
        return self.sizes


@pytest.mark.unit
def test_continuous_batching():
    async def main():
        h = await serve.run(Batcher.bind(), name="b")
        out = await asyncio.gather(*[h.infer.remote(i) for i in range(20)])
        assert out == [2 * i for i in range(20)]
        sizes = await h.sizes_seen.remote()
        assert sum(sizes) == 20 and max(sizes) == 8 and len(sizes) <= 4
        await serve.delete("b")

    asyncio.run(main())


@serve.deployment(ray_actor_options={"num_cpus": 0}, max_ongoing_requests=1,
                  autoscaling_config={"min_replicas": 1, "max_replicas": 3, "target_ongoing_requests": 1,
                                      "upscale_delay_s": 0.0, "downscale_delay_s": 0.0})
class Scaler:
    async def work(self, t):
        await asyncio.sleep(t)
        return serve.get_replica_context().replica_tag


@pytest.mark.unit
def test_autoscaling_up_and_down():
    async def main():
        ctrl_mod.set_controller(ctrl_mod.ServeController(tick_s=0.05))
        h = await serve.run(Scaler.bind(), name="s")
        rs = [h.work.remote(0.6) for _ in range(6)]
        await asyncio.sleep(0.4)
        n_up = len(ctrl_mod.get_controller().apps["s"].deployments["Scaler"].running())
        tags = set(await asyncio.gather(*rs))
        assert n_up >= 2 and len(tags) >= 2
        await asyncio.sleep(0.5)
        assert len(ctrl_mod.get_controller().apps["s"].deployments["Scaler"].running()) == 1
        await serve.delete("s")

    asyncio.run(main())


@serve.deployment(ray_actor_options={"num_cpus": 0}, health_check_period_s=0.1)
class Flaky:
    def __init__(self):
        self.fail = False

    async def set_fail(self):
        self.fail = True

    async def check_health(self):
        if self.fail:
            raise RuntimeError("boom")

    async def tag(self):
        return serve.get_replica_context().replica_tag


@pytest.mark.unit
def test_unhealthy_replica_is_replaced():
    async def main():
        ctrl_mod.set_controller(ctrl_mod.ServeController(tick_s=0.05))
        h = await serve.run(Flaky.bind(), name="f")
        t0 = await h.tag.remote()
        await h.set_fail.remote()
        for _ in range(60):
            await asyncio.sleep(0.1)
            ds = ctrl_mod.get_controller().apps["f"].deployments["Flaky"]
            if ds.running() and ds.running()[0].tag != t0:
                break
        assert await h.tag.remote() != t0
        assert ds.history and "boom" in (ds.history[-1]["error"] or "")
        await serve.delete("f")

    asyncio.run(main())


@pytest.mark.integration
def test_process_replica_and_handle_callback(monkeypatch):
    monkeypatch.setenv("BIOENGINE_REPLICA_MODE", "process")

    async def main():
        h = await serve.run(Entry.bind(Adder.bind(3)), name="proc")
        assert await h.remote(4) == 7
        assert await h.mux.remote("z") == "model-z"
        ds = ctrl_mod.get_controller().apps["proc"].deployments["Adder"]
        assert ds.running()[0].pid != os.getpid()
        await serve.delete("proc")

    asyncio.run(main())


@pytest.mark.unit
def test_remote_tasks_thread_and_isolated():
    import ray

    @ray.remote
    def sq(x):
        return x * x

    assert ray.get([sq.remote(i) for i in range(4)]) == [0, 1, 4, 9]

    def whoami():
        return os.getpid()

    pid = ray.get(ray.remote(whoami).options(isolate=True).remote())
    assert pid != os.getpid()

    def bad():
        raise ValueError("nope")

    from ray.exceptions import RayTaskError

    with pytest.raises(RayTaskError):
        ray.get(ray.remote(bad).remote())


@serve.deployment(ray_actor_options={"num_cpus": 0})
class Volume:
    async def scale(self, arr, k):
        return arr * k, {"sum": float(arr.sum())}


@serve.deployment(ray_actor_options={"num_cpus": 0})
class VolumeEntry:
    def __init__(self, volume: DeploymentHandle):
        self.volume = volume

    async def __call__(self, arr):
        return await self.volume.scale.remote(arr, 2)


@pytest.mark.unit
def test_process_replica_bulk_data_through_shm_rings(monkeypatch):
    """ndarray payloads above RING_MIN_BYTES cross router<->replica through the C++ shared-memory
    rings (both directions, nested handle calls too); the ring names are unlinked once the child
    has mapped them, so nothing is left in /dev/shm."""
    import numpy as np

    monkeypatch.setenv("BIOENGINE_REPLICA_MODE", "process")
    monkeypatch.setenv("BE_REPLICA_RING_MB", "16")

    async def main():
        h = await serve.run(VolumeEntry.bind(Volume.bind()), name="vol")
        rng = np.random.default_rng(0)
        for shape in [(16, 16), (32, 256, 256), (3, 1000, 1000)]:  # socket-only, ring, > ring (fallback)
            a = rng.standard_normal(shape).astype(np.float32)
            out, st = await h.remote(a)
            np.testing.assert_array_equal(out, a * 2)
            assert st["sum"] == pytest.approx(float(a.sum()), rel=1e-5)
        dss = ctrl_mod.get_controller().apps["vol"].deployments
        frames = 0
        for ds in dss.values():
            r = ds.running()[0]
            assert r.tx is not None and r.rx is not None
            assert not os.path.exists("/dev/shm" + r.tx.name) and not os.path.exists("/dev/shm" + r.rx.name)
            frames += r.tx.stats()["frames"] + r.rx.stats()["frames"]
        assert frames >= 4  # request + result of the 8 MiB call, on both hops
        await serve.delete("vol")

    asyncio.run(main())


@serve.deployment(ray_actor_options={"num_cpus": 0, "num_gpus": 1}, num_replicas=4, max_ongoing_requests=64)
class GpuEcho:
    def __init__(self):
        self.dev = os.environ.get("HIP_VISIBLE_DEVICES", "?")
        self.pid = os.getpid()

    async def work(self, i):
        await asyncio.sleep(0.01)
        return self.dev, self.pid


@pytest.mark.unit
def test_router_fans_requests_over_gpu_pinned_process_replicas(monkeypatch):
    """Node-level serving: one process replica per GPU, each pinned with
    HIP_VISIBLE_DEVICES, and the router spreading concurrent requests over all of them (the
    reference's replica scaling, bioengine/apps/proxy_deployment.py:35-44)."""
    monkeypatch.setenv("BIOENGINE_REPLICA_MODE", "process")
    monkeypatch.setenv("BIOENGINE_GPU_IDS", "0,1,2,3")

    async def main():
        h = await serve.run(GpuEcho.bind(), name="fan")
        res = await asyncio.gather(*[h.work.remote(i) for i in range(256)])
        await serve.delete("fan")
        return res

    res = asyncio.run(main())
    devs = {}
    for d, pid in res:
        devs.setdefault(d, set()).add(pid)
    assert sorted(devs) == ["0", "1", "2", "3"], devs
    assert all(len(p) == 1 for p in devs.values())  # one process per GPU
    counts = {d: sum(1 for r in res if r[0] == d) for d in devs}
    assert min(counts.values()) >= 256 // 4 // 3, counts  # every replica carries load
