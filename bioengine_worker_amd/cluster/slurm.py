"""SLURM autoscaler for the head worker (reference SlurmWorkers, bioengine/cluster/slurm_workers.py:
sbatch script generation :153-296, submit / poll / cancel :298-515, scale-up with cooldown and
max_workers :688-774, idle scale-down :817-903, node stop :645-659).

MI355X/native differences: a job runs the :mod:`node agent <.node_agent>` (not ``ray start``)
inside ``apptainer exec --rocm`` (ROCm device pass-through instead of ``--nv``) or directly with
the worker's Python; the node joins by registering a ``bioengine-node`` service on the hub; the
token reaches the job through a 0600 token file, never the script text.  Demand comes from the
controller's ``pending_demands`` (replicas waiting for resources), and idle nodes are stopped
through their agent before ``scancel``.
"""
from __future__ import annotations

import asyncio
import os
import shlex
import shutil
import sys
import time
import uuid
from pathlib import Path

JOB_NAME = "bioengine-worker"


class SlurmWorkers:
    def __init__(self, server_url: str, token: str | None, workspace_dir: str | Path, head_service_id: str | None = None,
                 image: str | None = None, worker_cache_dir: str | None = None, worker_data_dir: str | None = None,
                 default_num_gpus: int = 1, default_num_cpus: int = 8, default_mem_in_gb_per_cpu: float = 16.0,
                 default_time_limit: str = "4:00:00", further_slurm_args: list | None = None,
                 apptainer_args: list | None = None, max_workers: int = 4, scale_up_cooldown_seconds: float = 60.0,
                 scale_down_check_interval_seconds: float = 60.0, scale_down_threshold_seconds: float = 300.0,
                 node_wait_timeout: float = 900.0, python: str | None = None, sbatch: str = "sbatch",
                 squeue: str = "squeue", scancel: str = "scancel", logger=None):
        self.server_url = server_url
        self.token = token
        self.dir = Path(workspace_dir).expanduser() / "slurm"
        self.dir.mkdir(parents=True, exist_ok=True)
        self.head_service_id = head_service_id
        self.image = image
        self.worker_cache_dir = worker_cache_dir
        self.worker_data_dir = worker_data_dir
        self.default_num_gpus = default_num_gpus
        self.default_num_cpus = default_num_cpus
        self.mem_per_cpu = default_mem_in_gb_per_cpu
        self.time_limit = default_time_limit
        self.further_args = list(further_slurm_args or [])
        self.apptainer_args = list(apptainer_args or [])
        self.max_workers = max_workers
        self.cooldown = scale_up_cooldown_seconds
        self.down_interval = scale_down_check_interval_seconds
        self.down_threshold = scale_down_threshold_seconds
        self.node_wait_timeout = node_wait_timeout
        self.python = python or sys.executable
        self.sbatch, self.squeue, self.scancel = sbatch, squeue, scancel
        self.log = logger
        self.jobs: dict[str, dict] = {}  # job_id -> {state, submitted, num_gpus, script}
        self.last_scale_up = 0.0
        self.last_down_check = 0.0
        self.controller = None

    # ------------------------------------------------------------------ job handling
    def _token_file(self) -> Path:
        p = self.dir / "token"
        if self.token and (not p.exists() or p.read_text() != self.token):
            p.write_text(self.token)
            os.chmod(p, 0o600)
        return p

    def job_script(self, num_gpus: int, num_cpus: int, time_limit: str | None = None) -> str:
        root = str(Path(__file__).resolve().parents[2])
        agent = [self.python, "-u", "-m", "bioengine_worker_amd.cluster.node_agent", "--server-url", self.server_url,
                 "--token-file", str(self._token_file()), "--num-cpus", str(num_cpus), "--num-gpus", str(num_gpus),
                 "--node-id", "slurm-${SLURM_JOB_ID}", "--log-dir", str(self.dir / "replica_logs")]
        if self.head_service_id:
            agent += ["--head-service-id", self.head_service_id]
        agent_cmd = " ".join(a if a.startswith("slurm-${") else shlex.quote(a) for a in agent)
        if self.image:
            binds = [f"--bind {shlex.quote(root)}", f"--bind {shlex.quote(str(self.dir))}"]
            for d in (self.worker_cache_dir, self.worker_data_dir):
                if d:
                    binds.append(f"--bind {shlex.quote(d)}")
            extra = " ".join(shlex.quote(a) for a in self.apptainer_args)
            run = f"apptainer exec --rocm --cleanenv {' '.join(binds)} {extra} {shlex.quote(self.image)} {agent_cmd}"
        else:
            run = agent_cmd
        lines = ["#!/bin/bash", f"#SBATCH --job-name={JOB_NAME}", f"#SBATCH --cpus-per-task={num_cpus}",
                 f"#SBATCH --mem-per-cpu={self.mem_per_cpu:g}G", f"#SBATCH --time={time_limit or self.time_limit}",
                 f"#SBATCH --output={self.dir}/%x-%j.out"]
        if num_gpus:
            lines.append(f"#SBATCH --gpus={num_gpus}")
        lines += [f"#SBATCH {a}" for a in self.further_args]
        lines += ["set -euo pipefail", "export HSA_ENABLE_IPC_MODE_LEGACY=0",
                  f"export PYTHONPATH={shlex.quote(root)}${{PYTHONPATH:+:$PYTHONPATH}}",
                  f'echo "bioengine node ${{SLURM_JOB_ID:-?}} on $(hostname)"', f"exec {run}", ""]
        return "\n".join(lines)

    async def _run(self, *cmd, timeout: float = 30.0) -> tuple[int, str]:
        p = await asyncio.create_subprocess_exec(*cmd, stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.STDOUT)
        try:
            out, _ = await asyncio.wait_for(p.communicate(), timeout)
        except asyncio.TimeoutError:
            p.kill()
            return 124, "timeout"
        return p.returncode, out.decode(errors="replace")

    async def submit(self, num_gpus: int | None = None, num_cpus: int | None = None) -> str:
        g = self.default_num_gpus if num_gpus is None else num_gpus
        c = self.default_num_cpus if num_cpus is None else num_cpus
        script = self.dir / f"job_{uuid.uuid4().hex[:8]}.sh"
        script.write_text(self.job_script(g, c))
        rc, out = await self._run(self.sbatch, "--parsable", str(script))
        if rc != 0:
            raise RuntimeError(f"sbatch failed ({rc}): {out.strip()}")
        job_id = out.strip().split(";")[0].split()[-1]
        self.jobs[job_id] = {"state": "PENDING", "submitted": time.time(), "num_gpus": g, "script": str(script)}
        if self.log:
            self.log.info("submitted SLURM worker job %s (%d GPUs)", job_id, g)
        return job_id

    async def refresh(self) -> dict:
        rc, out = await self._run(self.squeue, "-h", "-o", "%i %T %j", "--name", JOB_NAME)
        if rc != 0:
            return self.jobs
        live = {}
        for line in out.splitlines():
            parts = line.split()
            if len(parts) >= 2:
                live[parts[0]] = parts[1]
        for jid in list(self.jobs):
            if jid in live:
                self.jobs[jid]["state"] = live[jid]
            else:
                self.jobs.pop(jid)  # finished / cancelled / failed
        return self.jobs

    async def cancel(self, job_id: str) -> None:
        await self._run(self.scancel, job_id)
        self.jobs.pop(job_id, None)

    # ------------------------------------------------------------------ scaling
    def _nodes_by_job(self) -> dict:
        if self.controller is None:
            return {}
        out = {}
        for n in self.controller.remote_nodes.values():
            jid = str(n.info.get("slurm_job_id") or "")
            if jid:
                out[jid] = n
        return out

    async def check_scaling(self, cluster_status: dict | None = None) -> None:
        await self.refresh()
        now = time.time()
        demands = list(self.controller.pending_demands) if self.controller is not None else \
            list(((cluster_status or {}).get("cluster", {}).get("pending_resources") or {}).get("actors", []))
        joined = self._nodes_by_job()
        starting = [j for j in self.jobs if j not in joined]
        if demands and not starting and len(self.jobs) < self.max_workers and now - self.last_scale_up >= self.cooldown:
            need_gpus = max(int(-(-float(d.get("num_gpus", 0)) // 1)) for d in demands)
            need_cpus = max(int(-(-float(d.get("num_cpus", 1)) // 1)) for d in demands)
            self.last_scale_up = now
            await self.submit(max(need_gpus, self.default_num_gpus if need_gpus else 0),
                              max(need_cpus, self.default_num_cpus))
        if now - self.last_down_check >= self.down_interval:
            self.last_down_check = now
            for jid, node in joined.items():
                if not node.replicas and now - node.last_busy >= self.down_threshold:
                    if self.log:
                        self.log.info("scaling down idle node %s (job %s)", node.node_id, jid)
                    try:
                        await node.service.shutdown()
                    except Exception:  # noqa: BLE001
                        pass
                    self.controller.remove_remote_node(node.node_id)
                    await self.cancel(jid)

    async def close_all(self) -> None:
        for jid, node in self._nodes_by_job().items():
            try:
                await node.service.shutdown()
            except Exception:  # noqa: BLE001
                pass
        for jid in list(self.jobs):
            await self.cancel(jid)

    @staticmethod
    def available() -> bool:
        return shutil.which("sbatch") is not None
