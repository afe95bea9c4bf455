"""Failure detection + fault injection (runtime/faults.py): per-request deadlines enforced by the
router and propagated into process replicas, the replica watchdog (a call wedged past its deadline
fails the health check and the controller replaces the replica), fault-injection rules at traced
stage boundaries, and the GPU-hang probe (GPU-marked)."""
import asyncio
import time

import pytest

from bioengine_worker_amd.compat import install

install()

from ray import serve  # noqa: E402

from bioengine_worker_amd.profiling import trace  # noqa: E402
from bioengine_worker_amd.runtime import faults  # noqa: E402
from bioengine_worker_amd.serve import controller as ctrl_mod  # noqa: E402


@pytest.fixture(autouse=True)
def fresh():
    ctrl_mod.set_controller(None)
    faults.clear()
    yield
    faults.clear()
    ctrl_mod.set_controller(None)


@serve.deployment(ray_actor_options={"num_cpus": 0}, request_timeout_s=0.3)
class Slow:
    async def nap(self, s):
        await asyncio.sleep(s)
        return s

    def busy(self, s):  # sync: runs on a thread the router cannot cancel
        time.sleep(s)
        return s

    async def ok(self):
        return "ok"

    async def tag(self):
        return serve.get_replica_context().replica_tag


def test_rules_and_stage_points():
    faults.inject("cellpose.*", "error", count=2)
    for _ in range(2):
        with pytest.raises(faults.InjectedFault):
            with trace.span("cellpose.masks"):
                pass
    with trace.span("cellpose.masks"):  # count exhausted
        pass
    with trace.span("train.adamw"):  # not matched
        pass
    faults.clear()
    faults._parse_env("train.backward=delay:1:1:0.05;x.*=oom")
    t = time.perf_counter()
    faults.point("train.backward")
    assert time.perf_counter() - t >= 0.05
    import torch

    with pytest.raises(torch.cuda.OutOfMemoryError):
        faults.point("x.y")
    faults.clear()
    r = faults.inject("p", "error", prob=0.5, seed=3)
    hits = 0
    for _ in range(200):
        try:
            faults.point("p")
        except faults.InjectedFault:
            hits += 1
    assert 60 < hits < 140 and r.fired == hits


def test_deadline_scope_nesting():
    assert faults.current_deadline() is None
    with faults.deadline_scope(10.0) as d1:
        with faults.deadline_scope(100.0) as d2:
            assert d2 == d1  # the earlier deadline wins
        with faults.deadline_scope(0.01):
            time.sleep(0.02)
            with pytest.raises(faults.DeadlineExceeded):
                faults.point("stage")
    assert faults.current_deadline() is None


def test_router_deadline_and_injected_replica_fault():
    async def main():
        h = await serve.run(Slow.bind(), name="slow")
        assert await h.nap.remote(0.01) == 0.01
        t = time.perf_counter()
        with pytest.raises(faults.DeadlineExceeded):
            await h.nap.remote(5)
        assert time.perf_counter() - t < 2
        ds = ctrl_mod.get_controller().apps["slow"].deployments["Slow"]
        assert ds.status_dict()["deadline_exceeded"] == 1
        faults.inject("replica_entry.ok", "error", count=1)
        with pytest.raises(faults.InjectedFault):
            await h.ok.remote()
        assert await h.ok.remote() == "ok"
        # the caller's own (tighter) deadline also bounds queueing + execution
        with faults.deadline_scope(0.05):
            with pytest.raises(faults.DeadlineExceeded):
                await h.nap.remote(1)
        await serve.delete("slow")

    asyncio.run(main())


def test_watchdog_replaces_wedged_local_replica(monkeypatch):
    monkeypatch.setenv("BIOENGINE_WATCHDOG_GRACE_S", "0.1")

    async def main():
        ctrl_mod.set_controller(ctrl_mod.ServeController(tick_s=0.05))
        h = await serve.run(Slow.options(health_check_period_s=0.1).bind(), name="wd")
        t0 = await h.tag.remote()
        with pytest.raises(faults.DeadlineExceeded):
            await h.busy.remote(2.0)  # thread keeps running past the deadline: wedged
        ds = ctrl_mod.get_controller().apps["wd"].deployments["Slow"]
        for _ in range(80):
            await asyncio.sleep(0.05)
            if ds.running() and ds.running()[0].tag != t0:
                break
        assert await h.tag.remote() != t0
        assert any("watchdog" in (x.get("error") or "") for x in ds.history)
        await serve.delete("wd")

    asyncio.run(main())


@pytest.mark.integration
def test_deadline_reaches_process_replica(monkeypatch):
    monkeypatch.setenv("BIOENGINE_REPLICA_MODE", "process")
    monkeypatch.setenv("BIOENGINE_WATCHDOG_GRACE_S", "0.1")

    async def main():
        h = await serve.run(Slow.bind(), name="pw")
        with pytest.raises(faults.DeadlineExceeded):
            await h.busy.remote(1.5)
        r = ctrl_mod.get_controller().apps["pw"].deployments["Slow"].running()[0]
        await asyncio.sleep(0.3)
        with pytest.raises(Exception, match="watchdog"):
            await r.check_health()  # the child still runs the call, 0.1 s past its deadline
        await asyncio.sleep(1.5)
        assert await r.check_health()  # call finished: healthy again
        await serve.delete("pw")

    asyncio.run(main())


@pytest.mark.gpu
def test_gpu_probe_and_event_wait():
    import torch

    dt = faults.gpu_probe(timeout_s=10)
    assert dt < 5
    a = torch.randn(4096, 4096, device="cuda")
    for _ in range(4):
        a = a @ a.T * 1e-3
    assert faults.gpu_wait(timeout_s=30) >= 0
    torch.cuda.synchronize()
