"""``bioengine cluster status`` — GPU / VRAM / CPU per node (reference bioengine/cli/cluster.py:53-131)."""
from __future__ import annotations

import click

from . import common


@click.group("cluster")
def cluster_group():
    """Inspect the worker's compute resources."""


@cluster_group.command("status")
@click.option("--json", "as_json", is_flag=True)
@common.worker_options
def cluster_status(as_json, worker_service_id, token, server_url):
    """Per-node CPUs, GPUs and GPU memory."""
    async def go():
        _, w = await common.worker(worker_service_id, token, server_url)
        st = await w.get_status()
        rc = st.get("ray_cluster") or {}
        if as_json:
            common.print_json(rc)
            return
        cl = rc.get("cluster") or {}
        click.secho(f"mode: {rc.get('mode')}  cpus {cl.get('used_cpu', 0)}/{cl.get('total_cpu', 0)}  "
                    f"gpus {cl.get('used_gpu', 0)}/{cl.get('total_gpu', 0)}", bold=True)
        rows = []
        for nid, n in (rc.get("nodes") or {}).items():
            gm = n.get("gpu_memory") or 0
            gmu = n.get("used_gpu_memory") or 0
            rows.append([nid[:16], n.get("node_ip", ""), f"{n.get('used_cpu', 0)}/{n.get('total_cpu', 0)}",
                         f"{n.get('used_gpu', 0)}/{n.get('total_gpu', 0)}",
                         f"{gmu / 2 ** 30:.1f}/{gm / 2 ** 30:.1f} GiB" if gm else "-", n.get("accelerator_type") or "-",
                         n.get("slurm_job_id") or "-"])
        common.print_table(rows, ["node", "ip", "cpu", "gpu", "vram", "accelerator", "slurm_job"])
    common.run(go())
