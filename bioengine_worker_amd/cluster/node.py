"""Node agent + cluster state (replaces RayCluster + BioEngineProxyActor).

Reference: ``bioengine/cluster/ray_cluster.py`` (3 modes, lock file, port scan, status history of
100 snapshots; ``:64-981``) and ``proxy_actor.py:289-436`` (per-node resource state incl. GPU
memory, pending demands).  Here there is no Ray: each node runs one worker/agent that owns a
:class:`~bioengine_worker_amd.serve.controller.ResourcePool`; GPU telemetry comes from
``amd-smi``/``rocm-smi`` (JSON) or, failing that, from torch's HIP device properties.

``status`` keeps the reference's shape::

    {"head_address", "start_time", "mode", "cluster": {total_cpu, used_cpu, total_gpu, used_gpu,
     pending_resources?}, "nodes": {node_id: {node_ip, head, total_cpu, used_cpu, total_gpu, used_gpu,
     total_gpu_memory, used_gpu_memory, total_memory, used_memory, total_object_store_memory,
     used_object_store_memory, accelerator_type, slurm_job_id, gpus: [...]}}}

plus per-GPU telemetry (HBM used/total, power, temperature) under ``nodes[*].gpus``.
"""
from __future__ import annotations

import collections
import json
import os
import shutil
import socket
import asyncio
import subprocess
import time
from pathlib import Path

from ..serve.controller import ResourcePool
from ..utils.network import get_internal_ip

MODES = ("single-machine", "slurm", "external-cluster")


def _run_json(cmd: list[str], timeout: float = 5.0):
    exe = shutil.which(cmd[0]) or (f"/opt/rocm/bin/{cmd[0]}" if Path(f"/opt/rocm/bin/{cmd[0]}").exists() else None)
    if exe is None:
        return None
    try:
        out = subprocess.run([exe] + cmd[1:], capture_output=True, text=True, timeout=timeout)
        if out.returncode != 0:
            return None
        return json.loads(out.stdout)
    except Exception:
        return None


def gpu_telemetry(indices: list[int] | None = None) -> list[dict]:
    """Per-GPU {index, name, total_memory, used_memory, power_w, temperature_c}; best effort."""
    gpus: list[dict] = []
    data = _run_json(["rocm-smi", "--showmeminfo", "vram", "--showproductname", "--showpower", "--showtemp", "--json"])
    if isinstance(data, dict):
        for k, v in sorted(data.items()):
            if not k.startswith("card"):
                continue
            try:
                idx = int(k[4:])
            except ValueError:
                continue
            def num(*names):
                for n in names:
                    for kk, vv in v.items():
                        if n.lower() in kk.lower():
                            try:
                                return float(str(vv).split()[0])
                            except ValueError:
                                pass
                return None
            gpus.append({"index": idx, "name": v.get("Card series") or v.get("Card Series") or "AMD Instinct",
                         "total_memory": num("VRAM Total Memory"), "used_memory": num("VRAM Total Used Memory"),
                         "power_w": num("Average Graphics Package Power", "Current Socket Graphics Package Power"),
                         "temperature_c": num("Temperature (Sensor junction)", "Temperature (Sensor edge)")})
    if not gpus and indices:
        # No SMI tool: report the devices without telemetry.  Deliberately no torch.cuda query
        # here: the worker process must not create a HIP context (replicas own the GPUs).
        gpus = [{"index": i, "name": "AMD Instinct", "total_memory": None, "used_memory": None,
                 "power_w": None, "temperature_c": None} for i in indices]
    if indices is not None:
        gpus = [g for g in gpus if g["index"] in indices] or gpus[: len(indices)]
    return gpus


def detect_gpu_ids() -> list[int]:
    env = os.environ.get("BIOENGINE_GPU_IDS")
    if env is not None:
        return [int(x) for x in env.split(",") if x.strip()]
    try:
        import torch

        return list(range(torch.cuda.device_count()))  # count only: does not initialise HIP
    except Exception:
        return []


class NodeCluster:
    """Cluster runtime for one worker (head node) and optional remote node agents."""

    def __init__(self, mode: str = "single-machine", head_num_cpus: float | None = None, head_num_gpus: int | None = None,
                 head_memory_in_gb: float | None = None, status_interval_seconds: float = 10.0, history_len: int = 100,
                 slurm_workers=None, logger=None):
        if mode not in MODES:
            raise ValueError(f"Invalid mode '{mode}'. Must be one of {MODES}")
        if mode == "single-machine" and head_num_cpus is not None and head_num_cpus <= 0:
            raise ValueError("single-machine mode needs head_num_cpus > 0")
        self.mode = mode
        ids = detect_gpu_ids()
        if head_num_gpus is not None:
            ids = ids[:head_num_gpus] if head_num_gpus <= len(ids) else ids
            if head_num_gpus == 0:
                ids = []
        mem = head_memory_in_gb * 1024 ** 3 if head_memory_in_gb else None
        self.resources = ResourcePool(head_num_cpus, ids, mem)
        self.address = get_internal_ip()
        self.hostname = socket.gethostname()
        self.start_time = time.time()
        self.history: collections.OrderedDict = collections.OrderedDict()
        self.history_len = history_len
        self.status_interval = status_interval_seconds
        self.remote_nodes: dict[str, dict] = {}
        self.slurm = slurm_workers
        self.pending_demands: list = []
        self.log = logger
        self.is_ready = False
        self.server = None
        self.controller = None

    def attach(self, server, controller) -> None:
        """Give the cluster the hub connection (node discovery) and the serving controller
        (placement on remote nodes; in SLURM mode unplaceable replicas wait for a new node)."""
        self.server = server
        self.controller = controller
        if self.mode == "slurm":
            controller.wait_for_nodes_s = float(getattr(self.slurm, "node_wait_timeout", 900.0) or 900.0)
        if self.slurm is not None:
            self.slurm.controller = controller

    async def discover_nodes(self) -> None:
        """Track ``bioengine-node`` services (node agents) of this workspace."""
        if self.server is None or self.controller is None or self.mode == "single-machine":
            return
        from ..serve.remote import RemoteNode

        try:
            infos = await self.server.list_services({"type": "bioengine-node"})
        except Exception as e:  # noqa: BLE001
            if self.log:
                self.log.warning("node discovery failed: %s", e)
            return
        seen = set()
        for info in infos:
            sid = info["id"]
            seen.add(sid)
            node = self.controller.remote_nodes.get(sid)
            try:
                if node is None:
                    svc = await self.server.get_service(sid)
                    res = await svc.get_resources()
                    self.controller.add_remote_node(RemoteNode(sid, svc, res))
                    if self.log:
                        self.log.info("node joined: %s (%d GPUs)", sid, len(res.get("gpu_ids", [])))
                else:
                    node.info.update(await node.service.get_resources())
                    node.last_seen = time.time()
            except Exception as e:  # noqa: BLE001
                if self.log:
                    self.log.warning("node %s unreachable: %s", sid, e)
        for nid in list(self.controller.remote_nodes):
            if nid not in seen:
                self.controller.remove_remote_node(nid)
                if self.log:
                    self.log.info("node left: %s", nid)

    async def start(self):
        self.is_ready = True
        self.monitor()

    async def stop(self):
        if self.slurm is not None:
            await self.slurm.close_all()
        self.is_ready = False

    def check_connection(self) -> bool:
        return self.is_ready

    def node_state(self, gpus: list[dict] | None = None) -> dict:
        r = self.resources
        if gpus is None:
            gpus = gpu_telemetry(r.gpu_ids) if r.gpu_ids else []
        tot_gm = sum(g["total_memory"] or 0 for g in gpus) if gpus else (0 if not r.gpu_ids else "NA")
        used_gm = sum(g["used_memory"] or 0 for g in gpus) if gpus else (0 if not r.gpu_ids else "NA")
        accel = "NA"
        if r.gpu_ids:
            accel = (gpus[0].get("name") if gpus else None) or "AMD-Instinct-MI355X"
        return {"node_ip": self.address, "head": True, "total_cpu": r.total_cpu, "used_cpu": r.used_cpu,
                "total_gpu": r.total_gpu, "used_gpu": r.used_gpu, "total_gpu_memory": tot_gm,
                "used_gpu_memory": used_gm, "total_memory": r.total_memory, "used_memory": r.used_memory,
                "total_object_store_memory": 0, "used_object_store_memory": 0, "accelerator_type": accel,
                "slurm_job_id": None, "gpus": gpus, "hostname": self.hostname}

    def monitor(self, gpus: list[dict] | None = None) -> dict:
        nodes = {f"head-{self.hostname}": self.node_state(gpus)}
        nodes.update(self.remote_nodes)
        if self.controller is not None:
            nodes.update({nid: n.status() for nid, n in self.controller.remote_nodes.items()})
        cluster = {"total_cpu": 0.0, "used_cpu": 0.0, "total_gpu": 0.0, "used_gpu": 0.0}
        for n in nodes.values():
            for k in cluster:
                cluster[k] += float(n.get(k) or 0)
        if self.mode == "slurm":
            from ..serve.controller import get_controller

            demands = list(get_controller().pending_demands) + list(self.pending_demands)
            cluster["pending_resources"] = {"actors": demands, "jobs": [], "tasks": [], "total": len(demands)}
        snap = {"cluster": cluster, "nodes": nodes}
        self.history[time.time()] = snap
        while len(self.history) > self.history_len:
            self.history.popitem(last=False)
        return snap

    @property
    def status(self) -> dict:
        last = next(reversed(self.history.values())) if self.history else self.monitor()
        return {"head_address": self.address, "start_time": self.start_time if self.mode != "external-cluster" else "N/A",
                "mode": self.mode, "cluster": last["cluster"], "nodes": last["nodes"]}

    async def monitor_cluster(self):
        await self.discover_nodes()
        # The SMI query is a ~100-150 ms subprocess.  Run on the event loop it stalled the hub, router
        # and app bridges that share this loop once per monitoring interval: every request in flight
        # at that moment waited it out (the c = 64 router p99 of ~150 ms against a ~30 ms p50,
        # profiles/r06/serve/timeline_s11.txt).  The query runs in a worker thread; the snapshot is
        # assembled back on the loop.
        r = self.resources
        gpus = await asyncio.to_thread(gpu_telemetry, r.gpu_ids) if r.gpu_ids else []
        self.monitor(gpus)
        if self.slurm is not None:
            await self.slurm.check_scaling(self.status)
