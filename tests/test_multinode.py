"""Multi-node serving on the native runtime (CPU): a node agent joins the head's workspace, the head
places replicas that do not fit locally on it, calls and nested handle calls work across nodes;
SLURM autoscaling with stand-in sbatch/squeue/scancel executables that run jobs locally."""
import asyncio
import os
import stat
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


async def _wait(pred, timeout=60, step=0.2):
    for _ in range(int(timeout / step)):
        r = pred()
        if asyncio.iscoroutine(r):
            r = await r
        if r:
            return r
        await asyncio.sleep(step)
    raise TimeoutError


@pytest.mark.end_to_end
def test_remote_node_placement(tmp_path, monkeypatch):
    from bioengine_worker_amd.cluster.node_agent import NodeAgent
    from bioengine_worker_amd.transport import connect_to_server
    from bioengine_worker_amd.transport.hub import get_local_hub, reset_local_hubs
    from bioengine_worker_amd.worker.worker import BioEngineWorker

    monkeypatch.setenv("BIOENGINE_LOCAL_ARTIFACT_PATH", str(ROOT / "apps"))
    monkeypatch.delenv("BIOENGINE_REPLICA_MODE", raising=False)
    reset_local_hubs()

    async def main():
        hub = get_local_hub("mn")
        await hub.start_http()
        tok = hub.issue_token("admin-user", workspace="ws-admin")
        w = BioEngineWorker(mode="external-cluster", workspace_dir=tmp_path / "be", server_url="local://mn", token=tok,
                            client_id="head", log_file="off", head_num_cpus=0.5, head_num_gpus=0,
                            monitoring_interval_seconds=0.2, data_server_url=None)
        await w.start(blocking=False)
        agent = NodeAgent("local://mn", tok, node_id="node-a", num_cpus=4, gpu_ids=[], log_dir=str(tmp_path / "nl"))
        await agent.start()
        await _wait(lambda: len(w.controller.remote_nodes) == 1)
        admin = await connect_to_server({"server_url": "local://mn", "token": tok})
        svc = await admin.get_service(w.full_service_id)
        st = await svc.get_status()
        assert len(st["ray_cluster"]["nodes"]) == 2
        aid = await svc.deploy_app(artifact_id="bioengine-composition-demo", application_id="comp")
        assert await w.apps_manager.wait_for(aid, timeout=120) == "RUNNING", \
            (await svc.get_app_status(application_ids=[aid]))["message"]
        placed = {r.node_id for d in w.controller.apps["comp"].deployments.values() for r in d.replicas}
        assert "node-a" in placed or any("node-a" in p for p in placed)
        a = await admin.get_service((await svc.get_app_status(application_ids=[aid]))["service_ids"][0]["websocket_service_id"])
        out = await a.process(text="multi node", numbers=[1, 2, 3], delay=0.0)
        assert out["text"]["upper"] == "MULTI NODE" and out["stats"]["mean"] == 2.0
        assert len(agent.replicas) >= 1
        await svc.stop_app(application_id="comp")
        assert len(agent.replicas) == 0
        await agent.shutdown()
        await svc.stop_worker(blocking=True)

    asyncio.run(asyncio.wait_for(main(), 300))
    reset_local_hubs()


FAKE_SBATCH = r'''#!/bin/bash
# stand-in sbatch: run the job script locally in the background
set -e
script="${@: -1}"
dir="$(dirname "$0")"
id=$(( $(cat "$dir/next_id" 2>/dev/null || echo 1000) + 1 ))
echo $id > "$dir/next_id"
( export SLURM_JOB_ID=$id; exec setsid bash "$script" > "$dir/job_$id.log" 2>&1 ) &
echo $! > "$dir/job_$id.pid"
echo $id
'''
FAKE_SQUEUE = r'''#!/bin/bash
dir="$(dirname "$0")"
for f in "$dir"/job_*.pid; do
  [ -e "$f" ] || continue
  id=$(basename "$f" .pid); id=${id#job_}
  if kill -0 "$(cat "$f")" 2>/dev/null; then echo "$id RUNNING bioengine-worker"; fi
done
'''
FAKE_SCANCEL = r'''#!/bin/bash
dir="$(dirname "$0")"
f="$dir/job_$1.pid"
[ -e "$f" ] && kill -- -"$(cat "$f")" 2>/dev/null || kill "$(cat "$f")" 2>/dev/null || true
rm -f "$f"
'''


@pytest.mark.end_to_end
def test_slurm_autoscaling_with_fake_slurm(tmp_path, monkeypatch):
    from bioengine_worker_amd.cluster.slurm import SlurmWorkers
    from bioengine_worker_amd.transport import connect_to_server
    from bioengine_worker_amd.transport.hub_server import HubServer
    from bioengine_worker_amd.worker.worker import BioEngineWorker

    bindir = tmp_path / "bin"
    bindir.mkdir()
    for name, body in (("sbatch", FAKE_SBATCH), ("squeue", FAKE_SQUEUE), ("scancel", FAKE_SCANCEL)):
        p = bindir / name
        p.write_text(body)
        p.chmod(p.stat().st_mode | stat.S_IEXEC)
    monkeypatch.setenv("BIOENGINE_LOCAL_ARTIFACT_PATH", str(ROOT / "apps"))
    monkeypatch.delenv("BIOENGINE_REPLICA_MODE", raising=False)

    async def main():
        hub = HubServer(data_dir=str(tmp_path / "hub"), name="server")
        base = await hub.start_http("127.0.0.1", 0)
        url = base.replace("http://", "ws://")
        tok = hub.issue_token("admin-user", workspace="ws-admin", roles=["admin"])
        slurm = SlurmWorkers(url, tok, tmp_path / "be", sbatch=str(bindir / "sbatch"), squeue=str(bindir / "squeue"),
                             scancel=str(bindir / "scancel"), default_num_gpus=0, default_num_cpus=2,
                             max_workers=1, scale_up_cooldown_seconds=0, scale_down_check_interval_seconds=0.5,
                             scale_down_threshold_seconds=2.0, node_wait_timeout=120, python=sys.executable)
        w = BioEngineWorker(mode="slurm", workspace_dir=tmp_path / "be", server_url=url, token=tok, client_id="head",
                            log_file=str(tmp_path / "w.log"), head_num_cpus=0.5, head_num_gpus=0, monitoring_interval_seconds=0.3,
                            data_server_url=None, slurm_workers=slurm)
        await w.start(blocking=False)
        script = slurm.job_script(0, 2)
        assert "#SBATCH --job-name=bioengine-worker" in script and tok not in script
        admin = await connect_to_server({"server_url": url, "token": tok})
        svc = await admin.get_service(w.full_service_id)
        aid = await svc.deploy_app(artifact_id="demo-app", application_id="demo", disable_gpu=True)
        # the replica cannot fit the head: demand -> sbatch -> node agent joins -> replica placed there
        assert await w.apps_manager.wait_for(aid, timeout=180) == "RUNNING", \
            (await svc.get_app_status(application_ids=[aid]))["message"]
        assert len(slurm.jobs) == 1 and len(w.controller.remote_nodes) == 1
        st = await svc.get_status()
        assert any(n.get("slurm_job_id") for n in st["ray_cluster"]["nodes"].values())
        a = await admin.get_service((await svc.get_app_status(application_ids=[aid]))["service_ids"][0]["websocket_service_id"])
        assert (await a.reverse_text(text="slurm"))["reversed"] == "mruls"
        await svc.stop_app(application_id="demo")
        # idle node is scaled down: agent shut down + scancel
        await _wait(lambda: len(slurm.jobs) == 0 and len(w.controller.remote_nodes) == 0, timeout=60)
        await svc.stop_worker(blocking=True)
        await admin.disconnect()

    asyncio.run(asyncio.wait_for(main(), 400))
