"""``bioengine apps upload|run|deploy|list|status|logs|stop`` (reference bioengine/cli/apps.py:117-679)."""
from __future__ import annotations

from pathlib import Path

import click

from . import common


def _env_pairs(pairs) -> dict:
    """``Class:KEY=VALUE`` (or ``KEY=VALUE`` for every deployment, as ``*``) -> {Class: {KEY: VALUE}}."""
    out: dict = {}
    for p in pairs:
        if "=" not in p:
            common.fail(f"--env '{p}' must be [Class:]KEY=VALUE")
        k, v = p.split("=", 1)
        cls, key = k.split(":", 1) if ":" in k else ("*", k)
        out.setdefault(cls, {})[key] = v
    return out


@click.group("apps")
def apps_group():
    """Upload, deploy and manage BioEngine apps on a worker."""


@apps_group.command("upload")
@click.argument("app_dir", type=click.Path(exists=True, file_okay=False))
@common.worker_options
def upload(app_dir, worker_service_id, token, server_url):
    """Upload APP_DIR (manifest.yaml + code) as an artifact; prints the artifact id."""
    from ..utils.artifact_utils import create_file_list_from_directory

    async def go():
        _, w = await common.worker(worker_service_id, token, server_url)
        files = create_file_list_from_directory(Path(app_dir))
        aid = await w.upload_app(files=files)
        click.echo(aid)
    common.run(go())


def _deploy_opts(f):
    f = click.option("--id", "application_id", default=None, help="Application id (random if omitted).")(f)
    f = click.option("--no-gpu", "disable_gpu", is_flag=True, help="Deploy without GPUs.")(f)
    f = click.option("--env", "env_vars", multiple=True, metavar="[Class:]KEY=VALUE",
                     help="Environment variable for a deployment class ('_'-prefixed keys are secret).")(f)
    f = click.option("--hypha-token", default=None, help="Token injected into the app as HYPHA_TOKEN.")(f)
    return f


@apps_group.command("run")
@click.argument("artifact_id")
@click.option("--version", default=None, help="Artifact version.")
@_deploy_opts
@common.worker_options
def run_app(artifact_id, version, application_id, disable_gpu, env_vars, hypha_token, worker_service_id, token,
            server_url):
    """Deploy an uploaded artifact ARTIFACT_ID."""
    async def go():
        _, w = await common.worker(worker_service_id, token, server_url)
        app_id = await w.deploy_app(artifact_id=artifact_id, version=version, application_id=application_id,
                                    disable_gpu=disable_gpu, application_env_vars=_env_pairs(env_vars) or None,
                                    hypha_token=hypha_token)
        click.echo(app_id)
    common.run(go())


@apps_group.command("deploy")
@click.argument("app_dir", type=click.Path(exists=True, file_okay=False))
@_deploy_opts
@common.worker_options
def deploy(app_dir, application_id, disable_gpu, env_vars, hypha_token, worker_service_id, token, server_url):
    """Upload APP_DIR and deploy it in one step."""
    from ..utils.artifact_utils import create_file_list_from_directory

    async def go():
        _, w = await common.worker(worker_service_id, token, server_url)
        aid = await w.upload_app(files=create_file_list_from_directory(Path(app_dir)))
        app_id = await w.deploy_app(artifact_id=aid, application_id=application_id, disable_gpu=disable_gpu,
                                    application_env_vars=_env_pairs(env_vars) or None, hypha_token=hypha_token)
        click.echo(f"artifact: {aid}\napplication: {app_id}")
    common.run(go())


@apps_group.command("list")
@click.option("--json", "as_json", is_flag=True)
@common.worker_options
def list_apps(as_json, worker_service_id, token, server_url):
    """Uploaded app artifacts."""
    async def go():
        _, w = await common.worker(worker_service_id, token, server_url)
        apps = await w.list_apps()
        if as_json:
            common.print_json(apps)
            return
        rows = [[aid, (m.get("manifest") or m).get("name", ""), (m.get("manifest") or m).get("version", "")]
                for aid, m in apps.items()]
        common.print_table(rows, ["artifact_id", "name", "version"])
    common.run(go())


@apps_group.command("status")
@click.argument("app_ids", nargs=-1)
@click.option("--logs", "logs_tail", default=0, type=int, help="Include this many log lines per replica.")
@click.option("--json", "as_json", is_flag=True)
@common.worker_options
def status(app_ids, logs_tail, as_json, worker_service_id, token, server_url):
    """Status of running applications (all when no APP_ID is given)."""
    async def go():
        _, w = await common.worker(worker_service_id, token, server_url)
        res = await w.get_app_status(application_ids=list(app_ids) or None, logs_tail=logs_tail)
        if as_json:
            common.print_json(res)
            return
        items = {app_ids[0]: res} if len(app_ids) == 1 else res
        if not items:
            click.echo("no running applications")
        for aid, info in items.items():
            click.secho(f"{aid}: {info.get('status')}", bold=True)
            if info.get("message"):
                click.echo(f"  {info['message']}")
            for dn, d in (info.get("deployments") or {}).items():
                click.echo(f"  {dn}: {d.get('status')}")
            for sid in info.get("service_ids") or []:
                click.echo(f"  service: {sid.get('websocket_service_id')}")
    common.run(go())


@apps_group.command("logs")
@click.argument("app_id")
@click.option("--tail", default=50, type=int)
@click.option("--json", "as_json", is_flag=True)
@common.worker_options
def logs(app_id, tail, as_json, worker_service_id, token, server_url):
    """Replica logs of an application."""
    async def go():
        _, w = await common.worker(worker_service_id, token, server_url)
        info = await w.get_app_status(application_ids=[app_id], logs_tail=tail)
        if as_json:
            common.print_json(info)
            return
        for dn, d in (info.get("deployments") or {}).items():
            click.secho(f"== {dn}", bold=True)
            logs_ = d.get("logs") or {}
            for rep, lines in (logs_.items() if isinstance(logs_, dict) else [("", logs_)]):
                if rep:
                    click.echo(f"-- {rep}")
                for ln in (lines if isinstance(lines, list) else str(lines).splitlines()):
                    click.echo(ln)
    common.run(go())


@apps_group.command("stop")
@click.argument("app_id")
@click.option("--yes", "-y", is_flag=True, help="Do not ask for confirmation.")
@common.worker_options
def stop(app_id, yes, worker_service_id, token, server_url):
    """Stop a running application."""
    if not yes and not click.confirm(f"Stop application '{app_id}'?"):
        return

    async def go():
        _, w = await common.worker(worker_service_id, token, server_url)
        await w.stop_app(application_id=app_id)
        click.echo(f"stopped {app_id}")
    common.run(go())
