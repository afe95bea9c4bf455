"""``python -m bioengine.worker`` / ``python -m bioengine_worker_amd.worker`` — start a worker.

Option groups follow the reference CLI (bioengine/worker/__main__.py:58-576): Core, Hub (Hypha),
Cluster (the reference's "Ray Cluster" group — here the native node cluster), SLURM job and
autoscaler.  ``--startup-applications`` takes JSON objects (one per flag or a JSON list);
``--further-slurm-args`` / ``--apptainer-args`` are shell-split.  ``--start-hub HOST:PORT``
additionally starts an embedded hub server so a worker can run fully offline.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import shlex
import sys


def create_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="python -m bioengine.worker",
                                description="BioEngine worker (MI355X): serve BioEngine apps on local or SLURM GPUs.")
    core = p.add_argument_group("Core")
    core.add_argument("--mode", choices=["single-machine", "slurm", "external-cluster"], default="single-machine")
    core.add_argument("--admin-users", nargs="*", default=None, help="Admin user ids / emails ('*' = everyone).")
    core.add_argument("--workspace-dir", default="~/.bioengine", help="Worker state, app workdirs, logs.")
    core.add_argument("--startup-applications", action="append", default=None, metavar="JSON",
                      help='App to deploy at start, e.g. \'{"artifact_id": "demo-app", "disable_gpu": true}\'.')
    core.add_argument("--monitoring-interval-seconds", type=float, default=10.0)
    core.add_argument("--graceful-shutdown-timeout", type=float, default=60.0)
    core.add_argument("--log-file", default=None, help="Log file path ('off' disables file logging).")
    core.add_argument("--debug", action="store_true")
    core.add_argument("--data-server-url", default="auto", help="Datasets server URL ('auto' discovers, 'none' disables).")

    hub = p.add_argument_group("Hub (Hypha-compatible server)")
    hub.add_argument("--server-url", default=os.environ.get("BIOENGINE_SERVER_URL", "https://hypha.aicell.io"))
    hub.add_argument("--workspace", default=None)
    hub.add_argument("--token", default=None, help="Admin token (env HYPHA_TOKEN).")
    hub.add_argument("--client-id", default=None)
    hub.add_argument("--service-id", default="bioengine-worker")
    hub.add_argument("--worker-name", default=None)
    hub.add_argument("--start-hub", default=None, metavar="HOST:PORT",
                     help="Start an embedded hub server and connect to it (offline deployments).")

    cl = p.add_argument_group("Cluster")
    cl.add_argument("--head-num-cpus", type=float, default=None)
    cl.add_argument("--head-num-gpus", type=int, default=None)
    cl.add_argument("--head-memory-in-gb", type=float, default=None)

    sj = p.add_argument_group("SLURM job")
    sj.add_argument("--image", default=None, help="Apptainer image (.sif or docker:// URI) for worker jobs.")
    sj.add_argument("--worker-cache-dir", default=None)
    sj.add_argument("--worker-data-dir", default=None)
    sj.add_argument("--default-num-gpus", type=int, default=1)
    sj.add_argument("--default-num-cpus", type=int, default=8)
    sj.add_argument("--default-mem-in-gb-per-cpu", type=float, default=16.0)
    sj.add_argument("--default-time-limit", default="4:00:00")
    sj.add_argument("--further-slurm-args", default="", help="Extra sbatch arguments (shell-split).")
    sj.add_argument("--apptainer-args", default="", help="Extra apptainer exec arguments (shell-split).")

    au = p.add_argument_group("Autoscaler")
    au.add_argument("--max-workers", type=int, default=4)
    au.add_argument("--scale-up-cooldown-seconds", type=float, default=60.0)
    au.add_argument("--scale-down-check-interval-seconds", type=float, default=60.0)
    au.add_argument("--scale-down-threshold-seconds", type=float, default=300.0)
    return p


def parse_startup_applications(values) -> list[dict]:
    out: list[dict] = []
    for v in values or []:
        try:
            obj = json.loads(v)
        except json.JSONDecodeError as e:
            raise SystemExit(f"--startup-applications: invalid JSON {v!r}: {e}")
        items = obj if isinstance(obj, list) else [obj]
        for it in items:
            if not isinstance(it, dict) or "artifact_id" not in it:
                raise SystemExit(f"--startup-applications entries need an 'artifact_id': {it!r}")
            out.append(it)
    return out


def worker_kwargs(a: argparse.Namespace) -> dict:
    kw = dict(mode=a.mode, admin_users=a.admin_users, workspace_dir=a.workspace_dir, server_url=a.server_url,
              workspace=a.workspace, token=a.token, client_id=a.client_id, service_id=a.service_id,
              worker_name=a.worker_name, startup_applications=parse_startup_applications(a.startup_applications),
              monitoring_interval_seconds=a.monitoring_interval_seconds,
              graceful_shutdown_timeout=a.graceful_shutdown_timeout, log_file=a.log_file, debug=a.debug,
              data_server_url=None if str(a.data_server_url).lower() == "none" else a.data_server_url,
              head_num_cpus=a.head_num_cpus, head_num_gpus=a.head_num_gpus, head_memory_in_gb=a.head_memory_in_gb)
    if a.mode == "slurm":
        kw["slurm_config"] = dict(image=a.image, worker_cache_dir=a.worker_cache_dir, worker_data_dir=a.worker_data_dir,
                                  default_num_gpus=a.default_num_gpus, default_num_cpus=a.default_num_cpus,
                                  default_mem_in_gb_per_cpu=a.default_mem_in_gb_per_cpu,
                                  default_time_limit=a.default_time_limit,
                                  further_slurm_args=shlex.split(a.further_slurm_args),
                                  apptainer_args=shlex.split(a.apptainer_args), max_workers=a.max_workers,
                                  scale_up_cooldown_seconds=a.scale_up_cooldown_seconds,
                                  scale_down_check_interval_seconds=a.scale_down_check_interval_seconds,
                                  scale_down_threshold_seconds=a.scale_down_threshold_seconds)
    return kw


async def _amain(a) -> int:
    from .worker import BioEngineWorker

    kw = worker_kwargs(a)
    if a.start_hub:
        from ..transport.hub_server import HubServer

        host, port = a.start_hub.rsplit(":", 1)
        hub = HubServer(data_dir=os.path.join(os.path.expanduser(a.workspace_dir), "hub"), name="server")
        base = await hub.start_http(host, int(port))
        hub.ws_server_url = base.replace("http://", "ws://")
        admin = a.admin_users[0] if a.admin_users else "admin"
        kw["server_url"] = hub.ws_server_url
        kw["token"] = kw["token"] or hub.issue_token(admin, workspace=f"ws-user-{admin}", roles=["admin"],
                                                     expires_in=3600 * 24 * 30)
        print(f"embedded hub on {base}; worker token issued for '{admin}'", flush=True)
    w = BioEngineWorker(**kw)
    await w.start(blocking=True)
    return 0


def main(argv=None) -> int:
    a = create_parser().parse_args(argv)
    try:
        return asyncio.run(_amain(a))
    except KeyboardInterrupt:
        return 130


if __name__ == "__main__":
    sys.exit(main())
