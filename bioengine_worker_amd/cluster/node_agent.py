"""Worker-node agent: ``python -m bioengine_worker_amd.cluster.node_agent --server-url ... --token ...``.

Runs on every non-head node (a SLURM job started by :mod:`.slurm`, or any machine added to an
external cluster).  It registers a ``bioengine-node`` service on the hub (same workspace as the
head worker) and executes replicas the head places on it as GPU-pinned processes
(``HIP_VISIBLE_DEVICES``), so a node's GPUs serve apps exactly like the head's.  Handle calls made
inside those replicas are routed back through the head worker's ``route_call`` method.

Replaces the reference's ``ray start --address`` worker process + BioEngineProxyActor bookkeeping
(SURVEY.md §2.1 rows 6-7, §2.6 C2/C3).
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import os
import socket
import sys
import time

import cloudpickle

from ..serve.replica import ProcessReplica
from .node import detect_gpu_ids, gpu_telemetry

log = logging.getLogger("bioengine.node")


class _HeadRouter:
    """Routes DeploymentHandle calls of replicas on this node to the head controller."""

    def __init__(self, agent: "NodeAgent"):
        self.agent = agent

    async def call(self, app, dep, method, args, kwargs, model_id=""):
        head = await self.agent.head()
        blob = await head.route_call(payload=cloudpickle.dumps((app, dep, method, args, kwargs, model_id)))
        ok, val = cloudpickle.loads(blob)
        if not ok:
            raise val if isinstance(val, BaseException) else RuntimeError(str(val))
        return val


class NodeAgent:
    def __init__(self, server_url: str, token: str | None, head_service_id: str | None = None,
                 node_id: str | None = None, num_cpus: float | None = None, gpu_ids: list[int] | None = None,
                 slurm_job_id: str | None = None, log_dir: str | None = None):
        self.server_url = server_url
        self.token = token
        self.head_service_id = head_service_id
        self.slurm_job_id = slurm_job_id or os.environ.get("SLURM_JOB_ID")
        self.node_id = node_id or f"node-{socket.gethostname()}-{self.slurm_job_id or os.getpid()}"
        self.num_cpus = float(num_cpus if num_cpus is not None else (os.cpu_count() or 1))
        self.gpu_ids = list(gpu_ids if gpu_ids is not None else detect_gpu_ids())
        self.log_dir = log_dir
        self.replicas: dict[str, ProcessReplica] = {}
        self.server = None
        self._head = None
        self._stop = asyncio.Event()
        self.started = time.time()

    async def head(self):
        if self._head is None:
            if not self.head_service_id:
                svcs = await self.server.list_services({"type": "bioengine-worker"})
                if not svcs:
                    raise RuntimeError("no bioengine-worker service found to route calls to")
                self.head_service_id = svcs[0]["id"]
            self._head = await self.server.get_service(self.head_service_id)
        return self._head

    # ------------------------------------------------------------------ service methods
    async def get_resources(self) -> dict:
        # the SMI subprocess off the event loop (it would stall this agent's replica RPCs)
        gpus = await asyncio.to_thread(gpu_telemetry, self.gpu_ids) if self.gpu_ids else []
        return {"node_id": self.node_id, "hostname": socket.gethostname(), "num_cpus": self.num_cpus,
                "gpu_ids": self.gpu_ids, "slurm_job_id": self.slurm_job_id,
                "gpu_memory": sum((g.get("total_memory") or 0) for g in gpus),
                "used_gpu_memory": sum((g.get("used_memory") or 0) for g in gpus),
                "accelerator_type": (gpus[0].get("name") if gpus else None) or ("AMD-Instinct-MI355X" if self.gpu_ids else None),
                "n_replicas": len(self.replicas), "uptime": time.time() - self.started}

    async def start_replica(self, tag: str, app: str, dep: str, payload: bytes, gpu_ids: list, env: dict | None = None):
        # unpickling the deployment class imports its app module (torch, numpy, ...): off the event
        # loop, or a slow import on a loaded host starves the hub connection's heartbeat and the hub
        # drops this node mid-start ("client disconnected")
        cls, args, kwargs = await asyncio.to_thread(cloudpickle.loads, payload)
        r = ProcessReplica(app, dep, cls, args, kwargs, list(gpu_ids or []), env or {}, log_dir=self.log_dir)
        r.tag = tag
        r.node_id = self.node_id
        self.replicas[tag] = r
        try:
            await r.start()
        except BaseException:
            self.replicas.pop(tag, None)
            raise
        return {"pid": r.pid, "node_id": self.node_id}

    async def call_replica(self, tag: str, method: str, payload: bytes, model_id: str = ""):
        r = self.replicas.get(tag)
        if r is None:
            return cloudpickle.dumps((False, RuntimeError(f"no replica {tag} on {self.node_id}")))
        args, kwargs = cloudpickle.loads(payload)
        try:
            val = await r.call(method, args, kwargs, model_id)
            return cloudpickle.dumps((True, val))
        except BaseException as e:  # noqa: BLE001
            return cloudpickle.dumps((False, e))

    async def check_replica(self, tag: str):
        r = self.replicas.get(tag)
        if r is None:
            raise RuntimeError(f"no replica {tag} on {self.node_id}")
        return await r.check_health()

    async def stop_replica(self, tag: str, timeout: float = 20.0):
        r = self.replicas.pop(tag, None)
        if r is not None:
            await r.stop(timeout)
        return True

    def replica_logs(self, tag: str, n: int = 200) -> list:
        r = self.replicas.get(tag)
        return r.logs(n) if r is not None else []

    async def shutdown(self):
        for tag in list(self.replicas):
            await self.stop_replica(tag, 10.0)
        self._stop.set()
        return True

    # ------------------------------------------------------------------ lifecycle
    async def start(self, route_via_head: bool = False):
        """Connect and register.  ``route_via_head`` (the standalone agent process) sends nested
        DeploymentHandle calls of this node's replicas to the head worker; an agent embedded in a
        process that also hosts the head controller leaves routing to that controller."""
        from ..serve.controller import _set_child_router
        from ..transport import connect_to_server

        cfg = {"server_url": self.server_url, "client_id": self.node_id}
        if self.token:
            cfg["token"] = self.token
        self.server = await connect_to_server(cfg)
        if route_via_head:
            _set_child_router(_HeadRouter(self))
        await self.server.register_service({
            "id": "bioengine-node", "name": f"BioEngine node {self.node_id}", "type": "bioengine-node",
            "config": {"visibility": "protected"}, "node_id": self.node_id,
            "get_resources": self.get_resources, "start_replica": self.start_replica, "call_replica": self.call_replica,
            "check_replica": self.check_replica, "stop_replica": self.stop_replica, "replica_logs": self.replica_logs,
            "shutdown": self.shutdown})
        log.info("node %s registered (%d GPUs, %g CPUs)", self.node_id, len(self.gpu_ids), self.num_cpus)

    async def run_forever(self):
        await self.start(route_via_head=True)
        await self._stop.wait()
        try:
            await self.server.disconnect()
        except Exception:  # noqa: BLE001
            pass


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="BioEngine worker-node agent")
    ap.add_argument("--server-url", required=True)
    ap.add_argument("--token", default=os.environ.get("HYPHA_TOKEN"))
    ap.add_argument("--token-file", default=None, help="Read the token from this file (SLURM jobs).")
    ap.add_argument("--head-service-id", default=None)
    ap.add_argument("--node-id", default=None)
    ap.add_argument("--num-cpus", type=float, default=None)
    ap.add_argument("--num-gpus", type=int, default=None)
    ap.add_argument("--log-dir", default=None)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    gpus = detect_gpu_ids()
    if a.num_gpus is not None:
        gpus = gpus[: a.num_gpus]
    token = a.token
    if a.token_file:
        with open(a.token_file) as f:
            token = f.read().strip()
    agent = NodeAgent(a.server_url, token, a.head_service_id, a.node_id, a.num_cpus, gpus, log_dir=a.log_dir)
    try:
        asyncio.run(agent.run_forever())
    except KeyboardInterrupt:
        return 130
    return 0


if __name__ == "__main__":
    sys.exit(main())
