"""The periodic cluster monitor must not stall the shared event loop.

The GPU telemetry query (an SMI subprocess, ~100-150 ms) used to run synchronously inside
``NodeCluster.monitor_cluster``; every request the hub / router had in flight waited it out
(profiles/r06/serve/timeline_s11.jsonl). Here a slow fake telemetry must leave a concurrent
ticker coroutine on time, and the snapshot must still carry the telemetry it returned.
"""
import asyncio
import time

from bioengine_worker_amd.cluster import node as node_mod


def test_monitor_cluster_runs_telemetry_off_the_loop(monkeypatch):
    calls = []

    def slow_telemetry(ids=None):
        calls.append(list(ids or []))
        time.sleep(0.4)  # a blocking call, like subprocess.run
        return [{"index": i, "name": "fake-gpu", "total_memory": 10, "used_memory": 1} for i in ids]

    monkeypatch.setattr(node_mod, "gpu_telemetry", slow_telemetry)
    monkeypatch.setattr(node_mod, "detect_gpu_ids", lambda: [0, 1])
    cluster = node_mod.NodeCluster(mode="single-machine", head_num_cpus=4)

    async def main():
        gaps = []

        async def ticker():
            last = time.perf_counter()
            for _ in range(30):
                await asyncio.sleep(0.02)
                now = time.perf_counter()
                gaps.append(now - last)
                last = now

        t = asyncio.create_task(ticker())
        await cluster.monitor_cluster()
        await t
        return gaps

    gaps = asyncio.run(main())
    assert calls == [[0, 1]]
    assert max(gaps) < 0.25, f"event loop stalled {max(gaps) * 1e3:.0f} ms during monitoring"
    snap = next(reversed(cluster.history.values()))
    head = next(iter(snap["nodes"].values()))
    assert head["accelerator_type"] == "fake-gpu"
    assert head["total_gpu_memory"] == 20 and head["used_gpu_memory"] == 2
