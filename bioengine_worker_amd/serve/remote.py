"""Replicas on other nodes (SLURM jobs / external machines) of the native serving runtime.

Replaces the reference's multi-node Ray cluster (RayCluster + SlurmWorkers + BioEngineProxyActor,
SURVEY.md §2.1 rows 5-7; C2/C3 in §2.6): every worker node runs a :mod:`node agent
<bioengine_worker_amd.cluster.node_agent>` that registers a ``bioengine-node`` service on the hub;
the head controller mirrors each node's resources in a :class:`RemoteNode` and places replicas
there when the head is full.  A :class:`RemoteReplica` forwards ``start / call / check_health /
stop / logs`` to the node agent, which runs the replica as a GPU-pinned process exactly like a
head-local :class:`~bioengine_worker_amd.serve.replica.ProcessReplica`.  Payloads (the deployment
class, init args, call args and results) travel as cloudpickle bytes inside the hub RPC.
"""
from __future__ import annotations

import time

import cloudpickle

from .replica import DEAD, RUNNING, STOPPING, ReplicaBase


class RemoteNode:
    def __init__(self, node_id: str, service, resources: dict):
        from .controller import ResourcePool

        self.node_id = node_id
        self.service = service
        self.pool = ResourcePool(resources.get("num_cpus", 1), list(resources.get("gpu_ids", [])),
                                 resources.get("memory", 0) or None)
        self.info = dict(resources)
        self.last_seen = time.time()
        self.last_busy = time.time()
        self.replicas: set[str] = set()

    def status(self) -> dict:
        p = self.pool
        return {"node_ip": self.info.get("hostname", ""), "head": False, "total_cpu": p.total_cpu, "used_cpu": p.used_cpu,
                "total_gpu": p.total_gpu, "used_gpu": p.used_gpu, "gpu_memory": self.info.get("gpu_memory", 0),
                "used_gpu_memory": self.info.get("used_gpu_memory", 0), "memory": p.total_memory,
                "used_memory": p.used_memory, "object_store_memory": 0,
                "accelerator_type": self.info.get("accelerator_type"), "slurm_job_id": self.info.get("slurm_job_id"),
                "replicas": sorted(self.replicas)}


class RemoteReplica(ReplicaBase):
    def __init__(self, node: RemoteNode, *a, **k):
        super().__init__(*a, **k)
        self.node = node
        self.node_id = node.node_id

    async def start(self):
        # The node counts as busy from the moment a replica is placed on it, not once the start RPC
        # returns: a slow start (replica imports on a loaded host) otherwise leaves it looking idle
        # and the SLURM idle scale-down stops the node under the starting replica.
        self.node.replicas.add(self.tag)
        self.node.last_busy = time.time()
        try:
            res = await self.node.service.start_replica(
                tag=self.tag, app=self.app, dep=self.dep, payload=cloudpickle.dumps((self.cls, self.args, self.kwargs)),
                gpu_ids=self.gpu_ids, env=self.env)
        except BaseException:
            self.node.replicas.discard(self.tag)
            self.node.last_busy = time.time()
            raise
        self.pid = res.get("pid")
        self.state = RUNNING

    async def call(self, method: str, args, kwargs, model_id: str = ""):
        if self.state == DEAD:
            raise RuntimeError(f"replica {self.tag} is dead: {self.error}")
        self.ongoing += 1
        self.node.last_busy = time.time()
        try:
            blob = await self.node.service.call_replica(tag=self.tag, method=method,
                                                       payload=cloudpickle.dumps((args, kwargs)), model_id=model_id)
            ok, val = cloudpickle.loads(blob)
            if not ok:
                raise val if isinstance(val, BaseException) else RuntimeError(str(val))
            return val
        finally:
            self.ongoing -= 1
            self.node.last_busy = time.time()

    async def check_health(self):
        await self.node.service.check_replica(tag=self.tag)
        return True

    async def stop(self, timeout: float = 20.0):
        self.state = STOPPING
        try:
            await self.node.service.stop_replica(tag=self.tag, timeout=timeout)
        finally:
            self.node.replicas.discard(self.tag)
            self.state = DEAD

    def logs(self, n: int = 100) -> list[str]:
        return list(getattr(self, "_log_cache", []))[-n:]

    async def refresh_logs(self, n: int = 200) -> None:
        try:
            self._log_cache = await self.node.service.replica_logs(tag=self.tag, n=n)
        except Exception:  # noqa: BLE001
            pass
